"""Neural-network units (the Znicz-equivalent layer library) and model zoo."""
from veles_amd.models.all2all import *  # noqa: F401,F403
from veles_amd.models.gd import *  # noqa: F401,F403
from veles_amd.models.conv import *  # noqa: F401,F403
from veles_amd.models.gd_conv import *  # noqa: F401,F403
from veles_amd.models.pooling import *  # noqa: F401,F403
from veles_amd.models.normalization_units import *  # noqa: F401,F403
from veles_amd.models.dropout import *  # noqa: F401,F403
from veles_amd.models.activation import *  # noqa: F401,F403
from veles_amd.models.evaluator import *  # noqa: F401,F403
from veles_amd.models.decision import *  # noqa: F401,F403
from veles_amd.models.lr_adjust import *  # noqa: F401,F403
from veles_amd.models.standard_workflow import (  # noqa: F401
    StandardWorkflow, LAYER_TYPES, parse_mcdnnic)
