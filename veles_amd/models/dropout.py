"""Dropout (Znicz ``dropout``): inverted dropout with a counter-based mask
(``hvk_dropout``).  The forward unit draws a fresh 32-bit seed per minibatch;
the backward unit re-applies the same mask to err_output from that seed -
no mask tensor is stored.  Identity when the workflow is testing or for
non-TRAIN minibatches (``forward_mode``).

Data parallel: the mask of element i of a rank's shard is drawn at index
rank x (shard elements) + i, so N ranks draw exactly the masks one process
draws over the global minibatch (the seed sequence is the same at every
rank: seeded from the unit's reproducible generator)."""
from __future__ import annotations

from veles_amd.accelerated_units import AcceleratedUnit
from veles_amd.memory import Array
from veles_amd.models.nn_units import GradientDescentBase
from veles_amd.prng import device_seed, random_generator
from veles_amd import ops

__all__ = ["DropoutForward", "DropoutBackward"]


class DropoutForward(AcceleratedUnit):
    MAPPING = "dropout"

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "WORKER")
        super().__init__(workflow, **kwargs)
        self.dropout_ratio = float(kwargs.get("dropout_ratio", 0.5))
        self.rand = kwargs.get("rand", random_generator.get())
        self.output = Array(shallow_pickle=True)
        self.seed = 0
        self.seed_dev_saved = None
        self.forward_mode = False
        self.demand("input")

    @property
    def activation(self):
        return 0

    def package_export(self):
        # inference: dropout is the identity
        return {}

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        import torch
        x = self.input.devmem
        self.output.devmem = torch.zeros(
            tuple(self.input.shape), dtype=x.dtype if x is not None else
            self.compute_dtype, device=self.torch_device)

    def run(self):
        import torch
        x = self.input.devmem
        train = not self.forward_mode and not bool(
            getattr(self.workflow, "testing", False))
        mc = getattr(self, "minibatch_class", None)
        if mc is not None and mc != 2:
            train = False
        if not train or self.dropout_ratio <= 0:
            self.output.devmem = x
            self.active_ = False
            return
        self.active_ = True
        y = self.output.devmem
        if y is None or y is x or y.shape != x.shape or y.dtype != x.dtype:
            self.output.devmem = y = torch.empty_like(x)
        if x.is_cuda:
            # the seed sequence lives on the device (seeded once from the
            # unit's reproducible generator): no host value enters the
            # kernel arguments, so a captured step replays with fresh masks
            # (restored from a snapshot: device_seed.get)
            sd = device_seed.get(self, x.device, self._draw_seed)
            ops.seed_advance(sd)
            ops.dropout(x, self.dropout_ratio, None, out=y, seed_dev=sd,
                        base=self.index_base(x))
            return
        self.seed = int(self.rand.randint(0, 2 ** 31 - 1))
        ops.dropout(x, self.dropout_ratio, self.seed, out=y,
                    base=self.index_base(x))

    def _draw_seed(self):
        self.seed = int(self.rand.randint(0, 2 ** 31 - 1))
        return self.seed

    def __getstate__(self):
        device_seed.save(self)   # exact resume of the device mask stream
        return super().__getstate__()

    def index_base(self, x):
        """Mask index of this rank's first element (see the module doc)."""
        ld = getattr(self.workflow, "loader", None)
        rank = int(getattr(ld, "rank", 0) or 0) if ld is not None else 0
        return rank * x.numel()

    def init_unpickled(self):
        super().init_unpickled()
        self.seed_dev_ = None


class DropoutBackward(GradientDescentBase):
    MAPPING = "dropout"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.demand("forward_unit")

    def run(self):
        fwd = self.forward_unit
        err = self.err_output.devmem
        if not getattr(fwd, "active_", True):
            out = err
        else:
            ei = self.alloc_err_input(tuple(err.shape))
            out = ops.dropout(err, fwd.dropout_ratio, fwd.seed, out=ei,
                              seed_dev=getattr(fwd, "seed_dev_", None)
                              if err.is_cuda else None,
                              base=fwd.index_base(err))
        aux, aux_act = self.aux_tensor()
        if aux is not None:
            ei = self.alloc_err_input(tuple(err.shape))
            ops.act_bwd(out, aux, aux_act, out=ei)
        else:
            self.err_input.devmem = out
