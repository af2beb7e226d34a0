"""Data layer: loader state machine, full-batch device loaders, synthetic
datasets, file / image / pickle / HDF5 / interactive / RESTful loaders."""
from veles_amd.loader.base import (  # noqa: F401
    Loader, LoaderMSE, LoaderMSEMixin, LoaderWithValidationRatio, ILoader,
    UserLoaderRegistry, TEST, VALID, TRAIN, CLASS_NAME)
from veles_amd.loader.fullbatch import (  # noqa: F401
    FullBatchLoader, FullBatchLoaderMSE)
from veles_amd.loader.synthetic import (  # noqa: F401
    SyntheticImageLoader, SyntheticMSELoader)
