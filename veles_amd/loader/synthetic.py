"""Synthetic datasets of the benchmark shapes (no network on the GPU box).

The BASELINE configurations (MNIST 28x28x1, CIFAR-10 32x32x3, ImageNet
227x227x3 for AlexNet, 224x224x3 for VGG-16) are served as uint8 NHWC images
with a learnable structure: every class has a fixed random prototype image
and samples are prototype + per-sample noise, clipped to [0, 255].  Weights
of every model are random-init; BASELINE.md "data: synthetic".

Large sets are generated directly on the device (torch generator) so a
multi-GB uint8 ImageNet-shaped set materialises in HBM in milliseconds.
"""
from __future__ import annotations

import numpy

from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.fullbatch import FullBatchLoader, FullBatchLoaderMSE

__all__ = ["SyntheticImageLoader", "SyntheticMSELoader", "SHAPES"]

SHAPES = {
    "mnist": ((28, 28, 1), 10),
    "cifar10": ((32, 32, 3), 10),
    "imagenet": ((227, 227, 3), 1000),
    "imagenet224": ((224, 224, 3), 1000),
}


class SyntheticImageLoader(FullBatchLoader):
    """kwargs: ``dataset`` in SHAPES or ``sample_shape`` + ``n_classes``;
    ``class_lengths`` = (test, validation, train); ``noise`` (uint8 units);
    ``seed``; ``generate_on_device``."""

    MAPPING = "synthetic_images"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        ds = kwargs.get("dataset", "mnist")
        shape, ncls = SHAPES.get(ds, ((28, 28, 1), 10))
        self._sample_shape = tuple(kwargs.get("sample_shape", shape))
        self.n_classes = int(kwargs.get("n_classes", ncls))
        self.requested_lengths = list(kwargs.get(
            "class_lengths", (1000, 1000, 6000)))
        self.noise = float(kwargs.get("noise", 48.0))
        self.seed = int(kwargs.get("seed", 12345))
        self.generate_on_device = kwargs.get("generate_on_device", "auto")

    @property
    def sample_shape(self):
        return self._sample_shape

    def _want_device(self):
        dev = self.device
        if self.generate_on_device == "auto":
            total = sum(self.requested_lengths) * int(numpy.prod(
                self._sample_shape))
            return dev is not None and getattr(dev, "is_gpu", False) and \
                total > (64 << 20)
        return bool(self.generate_on_device) and dev is not None and \
            getattr(dev, "is_gpu", False)

    def load_data(self):
        import torch
        self.class_lengths = [int(x) for x in self.requested_lengths]
        self._apply_validation_ratio()
        n = sum(self.class_lengths)
        feat = int(numpy.prod(self._sample_shape))
        rs = numpy.random.RandomState(self.seed)
        # prototypes first: the same seed gives the same classes whatever
        # the set sizes (a test-only loader matches the training one)
        protos = rs.randint(32, 224, (self.n_classes, feat)).astype(
            numpy.float32)
        labels = rs.randint(0, self.n_classes, n).astype(numpy.int32)
        self.original_labels = labels
        if self._want_device():
            dev = self.device.torch_device
            g = torch.Generator(device=dev)
            g.manual_seed(self.seed)
            data = torch.empty((n,) + self._sample_shape, dtype=torch.uint8,
                               device=dev)
            tp = torch.from_numpy(protos).to(dev)
            tl = torch.from_numpy(labels).to(dev).long()
            flat = data.view(n, feat)
            step = max(1, (256 << 20) // (feat * 4))
            for i in range(0, n, step):
                j = min(n, i + step)
                noise = torch.randn(j - i, feat, generator=g, device=dev) * \
                    self.noise
                flat[i:j] = (tp[tl[i:j]] + noise).clamp_(0, 255).to(
                    torch.uint8)
            self.original_data.devmem = data
        else:
            out = numpy.empty((n, feat), dtype=numpy.uint8)
            step = 4096
            for i in range(0, n, step):
                j = min(n, i + step)
                v = protos[labels[i:j]] + rs.standard_normal(
                    (j - i, feat)).astype(numpy.float32) * self.noise
                numpy.clip(v, 0, 255, out=v)
                out[i:j] = v.astype(numpy.uint8)
            self.original_data.reset(out.reshape((n,) + self._sample_shape))
        self.labels_mapping = {i: i for i in range(self.n_classes)}
        self.reversed_labels_mapping = list(range(self.n_classes))

    def analyze_dataset(self):
        if self.original_data.devmem is not None and \
                self.original_data.devmem.is_cuda and \
                self.normalization_type != "none":
            # device-generated set: analyse a host copy of a TRAIN sample
            # subset (prototype + noise statistics are stationary)
            import torch
            b = self.class_end_offsets[VALID]
            e = min(self.class_end_offsets[TRAIN], b + 2048)
            sub = self.original_data.devmem[b:e].cpu().numpy().astype(
                numpy.float32)
            self.normalizer.analyze(sub)
            aff = self.normalizer.affine()
            feat = int(numpy.prod(self._sample_shape))
            if aff is None:
                raise ValueError("device-resident synthetic data needs an "
                                 "affine normalizer")
            self._affine = tuple(numpy.broadcast_to(
                numpy.asarray(a, numpy.float32), (feat,)).copy() for a in aff)
            del torch
            return
        super().analyze_dataset()


class SyntheticMSELoader(FullBatchLoaderMSE):
    """Regression / autoencoder target: target = the (scaled) input itself
    unless ``target_shape`` is given (then a fixed random linear map)."""

    MAPPING = "synthetic_mse"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._sample_shape = tuple(kwargs.get("sample_shape", (28, 28, 1)))
        self.target_shape = kwargs.get("target_shape")
        self.requested_lengths = list(kwargs.get("class_lengths",
                                                 (200, 200, 1000)))
        self.seed = int(kwargs.get("seed", 4321))

    @property
    def sample_shape(self):
        return self._sample_shape

    def load_data(self):
        self.class_lengths = [int(x) for x in self.requested_lengths]
        n = sum(self.class_lengths)
        feat = int(numpy.prod(self._sample_shape))
        rs = numpy.random.RandomState(self.seed)
        x = rs.uniform(-1, 1, (n, feat)).astype(numpy.float32)
        if self.target_shape:
            tf = int(numpy.prod(self.target_shape))
            m = rs.standard_normal((feat, tf)).astype(numpy.float32) / \
                numpy.sqrt(feat)
            t = numpy.tanh(x @ m).reshape((n,) + tuple(self.target_shape))
        else:
            t = x.copy().reshape((n,) + self._sample_shape)
        self.original_data.reset(x.reshape((n,) + self._sample_shape))
        self.original_targets.reset(t)
        self.original_labels = []
