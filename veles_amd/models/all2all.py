"""Fully connected layers (Znicz ``all2all*`` types; docs/OPS.md §All2All).

y[B][out] = act(x[B][in] . W[out][in]^T + b) - one MFMA GEMM with the bias and
activation fused in the epilogue (``hvk_gemm`` NT layout, both operands
K-contiguous; under precision_type "float8" the e4m3 fp8 MFMA kernel,
veles_amd/ops/fp8.py).  Activations: linear, tanh (1.7159 tanh(0.6666x)), relu
(softplus log(1+e^x)), strict relu max(0,x), sigmoid; softmax is the linear
layer followed by the fused softmax kernel.

Class UUIDs follow the reference export fixture
(libVeles/tests/workflow_files/contents.json) so exported packages are
readable by both runtimes.
"""
from __future__ import annotations

import os

import numpy

from veles_amd.memory import Array
from veles_amd.models.nn_units import Forward
from veles_amd import ops
from veles_amd.ops import fp8

__all__ = ["All2All", "All2AllTanh", "All2AllRELU", "All2AllStrictRELU",
           "All2AllSigmoid", "All2AllSoftmax", "ResizableAll2All"]


class All2All(Forward):
    __id__ = "58a5eadf-ae1e-498f-bf35-7d93939c4c86"
    MAPPING = "all2all"
    ACTIVATION = 0
    FP8 = True  # fp8 forward / dgrad under precision_type "float8"
    FP8_MIN_TILES = int(os.environ.get("VELES_AMD_FP8_FC_MIN_TILES", "128"))

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        oss = kwargs.get("output_sample_shape",
                         kwargs.get("output_shape", 10))
        self.output_sample_shape = (oss,) if isinstance(oss, int) \
            else tuple(oss)
        self.output_samples_number = kwargs.get("output_samples_number")

    @property
    def neurons_number(self):
        return int(numpy.prod(self.output_sample_shape))

    def initialize(self, device=None, **kwargs):
        super().initialize(device=device, **kwargs)
        n_in = self.input.sample_size if self.input.mem is not None else \
            int(numpy.prod(self.input.shape[1:]))
        shape = (self.neurons_number, n_in) if not self.weights_transposed \
            else (n_in, self.neurons_number)
        self.register_params(shape, n_in)
        self.allocate_outputs(self.input.shape[0])
        # fp8 only where the 128 x 128 output tiles can fill the chip: the
        # fp8 kernel has no split-K, and a thin layer (VGG-16 fc6 / fc7 at
        # batch 128: 32 tiles) runs faster on the bf16 split-K GEMM, without
        # quantizing its weights every step (profiles/c3pad_r2/README.md)
        tiles = -(-int(self.input.shape[0]) // 128) * \
            -(-self.neurons_number // 128)
        self.fp8_ = bool(getattr(self.device, "fp8", False)) and \
            self.FP8 and not self.weights_transposed and \
            n_in % 16 == 0 and self.neurons_number % 16 == 0 and \
            (tiles >= self.FP8_MIN_TILES or
             not getattr(self.device, "is_gpu", False))
        if self.fp8_ and self.fp8_sx_ is None:
            self.fp8_sx_ = fp8.Scaler(self.torch_device, fp8.E4M3)
            self.fp8_sw_ = fp8.Scaler(self.torch_device, fp8.E4M3)
            fp8.restore_scaler(self, "fp8_sx_")
            fp8.restore_scaler(self, "fp8_sw_")

    def __getstate__(self):
        fp8.save_scalers(self, ("fp8_sx_", "fp8_sw_"))
        return super().__getstate__()

    def init_unpickled(self):
        super().init_unpickled()
        self.fp8_ = False
        self.fp8_sx_ = self.fp8_sw_ = None
        self.x8_ = self.w8_ = None

    def allocate_outputs(self, B):
        self.alloc_output((B,) + self.output_sample_shape)

    def _gemm(self, out2d, act):
        x = self.input.devmem
        B = x.shape[0]
        x2 = x.reshape(B, -1)
        if self.fp8_:
            self.x8_ = fp8.quantize(x2, self.fp8_sx_, out=self.x8_)
            self.w8_ = fp8.quantize(self.weights_lp, self.fp8_sw_,
                                    out=self.w8_)
            fp8.gemm(self.x8_, self.fp8_sx_, self.w8_, self.fp8_sw_,
                     bias=self.bias_master, act=act, out=out2d)
            return
        if x2.dtype != self.weights_lp.dtype:
            x2 = x2.to(self.weights_lp.dtype)
        ops.gemm(x2, self.weights_lp, trans_b=not self.weights_transposed,
                 bias=self.bias_master, act=act, out=out2d)

    def run(self):
        x = self.input.devmem
        B = x.shape[0]
        y = self.alloc_output((B,) + self.output_sample_shape)
        self._gemm(y.view(B, -1), self.activation)


class All2AllTanh(All2All):
    __id__ = "b3a2bd5c-3c01-46ef-978a-fef22e008f31"
    MAPPING = "all2all_tanh"
    ACTIVATION = 1


class All2AllRELU(All2All):
    __id__ = "5b7a8e5b-a0f3-4e0c-93e1-1b6a8d6c0a11"
    MAPPING = "all2all_relu"
    ACTIVATION = 2


class All2AllStrictRELU(All2All):
    __id__ = "a1e3c7a4-2e9f-47c1-8a47-5f6cbb2d6e02"
    MAPPING = "all2all_str"
    ACTIVATION = 3


class All2AllSigmoid(All2All):
    __id__ = "c6d19d1a-5a67-4c31-9f3d-34a0b6f3b7a9"
    MAPPING = "all2all_sigmoid"
    ACTIVATION = 4


class ResizableAll2All(All2All):
    MAPPING = "all2all_resizable"


class All2AllSoftmax(All2All):
    """Linear layer + softmax.  ``output`` holds probabilities (float32),
    ``max_idx`` the argmax; ``logits`` is what EvaluatorSoftmax consumes."""

    __id__ = "420219fc-3e1a-45b1-87f8-aaa0c1540de4"
    MAPPING = "softmax"
    ACTIVATION = 0
    FP8 = False  # float32 logits feed the loss: kept on the bf16 kernel

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.max_idx = Array(shallow_pickle=True)
        self.logits = Array(shallow_pickle=True)
        self.compute_probabilities = kwargs.get("compute_probabilities", True)

    def allocate_outputs(self, B):
        import torch
        n = self.neurons_number
        self.logits.devmem = torch.zeros(B, n, dtype=torch.float32,
                                         device=self.torch_device)
        self.max_idx.devmem = torch.zeros(B, dtype=torch.int32,
                                          device=self.torch_device)
        self.alloc_output((B, n), torch.float32)

    def run(self):
        import torch
        x = self.input.devmem
        B = x.shape[0]
        n = self.neurons_number
        lg = self.logits.devmem
        if lg is None or tuple(lg.shape) != (B, n) or \
                lg.device != self.torch_device:
            self.logits.devmem = lg = torch.zeros(
                B, n, dtype=torch.float32, device=self.torch_device)
        self._gemm(lg, 0)
        if self.compute_probabilities:
            y = self.alloc_output((B, n), torch.float32)
            mi = self.max_idx.devmem
            if mi is None or mi.shape[0] != B or mi.device != lg.device:
                self.max_idx.devmem = mi = torch.zeros(
                    B, dtype=torch.int32, device=self.torch_device)
            ops.softmax_ce(lg, None, probs=y, max_idx=mi)
        else:
            self.output.devmem = lg
