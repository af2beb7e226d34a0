"""Image loaders (reference veles/loader/image.py:106-806,
file_image.py:53-183, fullbatch.py:349-433, base.py:925-1018): streaming
decode + prefetch, device-side crop / crop_number / mirror / rotations /
Sobel / background, samples_inflation, reproducibility from the workflow
PRNG, label statistics and the label-stratified validation split."""
import math
import os

import numpy
import pytest
import torch

from veles_amd import ops
from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher, DummyWorkflow
from veles_amd.loader import (
    FileImageLoader, FileListImageLoader, FullBatchFileImageLoader, TEST,
    TRAIN, VALID)
from veles_amd.loader.augment import Augmentation
from veles_amd.loader.labels import (LoaderError, distribution_pvalue,
                                     stratified_split)
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import gd_params
from veles_amd.prng import random_generator


def _make_images(root, classes=("cat", "dog"), per=6, size=(12, 10),
                 seed=0):
    from PIL import Image
    rs = numpy.random.RandomState(seed)
    for ci, c in enumerate(classes):
        d = os.path.join(root, c)
        os.makedirs(d, exist_ok=True)
        for i in range(per):
            a = (rs.rand(size[1], size[0], 3) * 60 + ci * 150).astype(
                numpy.uint8)
            Image.fromarray(a).save(os.path.join(d, "%s_%d.png" % (c, i)))
    return root


def _init(loader):
    loader.initialize(device=Device(backend="cpu"))
    return loader


def _serve(ld, n=1):
    out = []
    for _ in range(n):
        ld.run()
        out.append((ld.minibatch_class, ld.minibatch_size,
                    ld.minibatch_data.devmem.clone(),
                    ld.minibatch_labels.devmem.clone()
                    if ld.minibatch_labels.devmem is not None else None,
                    ld.minibatch_indices.devmem.clone()))
    return out


# ------------------------------------------------------------ augmentation
def test_augmentation_validation_and_inflation():
    assert Augmentation().samples_inflation == 1
    a = Augmentation(crop=(4, 5), crop_number=3, mirror=True,
                     rotations=(0.5, 0.0))
    assert a.samples_inflation == 2 * 2 * 3
    assert a.rotations == (0.0, 0.5)
    assert a.output_hw((10, 12)) == (4, 5)
    assert Augmentation(crop=(0.5, 0.25)).output_hw((10, 12)) == (5, 3)
    with pytest.raises(ValueError):
        Augmentation(crop_number=2)
    with pytest.raises(ValueError):
        Augmentation(mirror="sometimes")
    with pytest.raises(ValueError):
        Augmentation(rotations=(7.0,))
    with pytest.raises(ValueError):
        Augmentation(crop=(0, 3))
    # distortion slots: mirror True alternates, rotations by slot // 2
    prng = random_generator.RandomGenerator("t")
    prng.seed(1)
    assert a.distortion(0, prng) == (False, 0.0)
    assert a.distortion(3, prng) == (True, 0.0)     # crop 0, mirrored
    assert a.distortion(6, prng) == (False, 0.5)


def test_image_batch_geometry_reference():
    """Crop, mirror and a 90-degree rotation move pixels where expected;
    the Sobel channel is the gradient magnitude of the grey image."""
    g = torch.Generator().manual_seed(0)
    src = torch.randint(0, 256, (2, 9, 9, 3), dtype=torch.uint8, generator=g)
    idx = torch.tensor([1, 0], dtype=torch.int32)
    p = torch.tensor([[2, 1, 1, 0, 0, 0],
                      [0, 0, math.cos(math.pi / 2), math.sin(math.pi / 2),
                       0, 0]], dtype=torch.float32)
    out = ops.image_batch_ref(src, idx, p, 7, 7)
    assert torch.equal(out[0], src[1, 2:9, 1:8].float())
    # rotation by +90 deg about (3, 3): output (y, x) reads source
    # (3 + (x - 3), 3 - (y - 3)) = (x, 6 - y)
    sub = src[0, 0:7, 0:7].float()
    for y in range(7):
        for x in range(7):
            torch.testing.assert_close(out[1, y, x], sub[x, 6 - y],
                                       atol=1e-3, rtol=0)
    flat = torch.full((1, 5, 5, 1), 100, dtype=torch.uint8)
    s = ops.image_batch_ref(flat, torch.tensor([0], dtype=torch.int32),
                            torch.tensor([[0, 0, 1, 0, 0, 0]]), 5, 5,
                            sobel=True)
    assert s.shape == (1, 5, 5, 2) and float(s[..., 1].abs().max()) == 0.0


# ------------------------------------------------------------ full batch
def test_full_batch_crop_mirror_rotation_reproducible(tmp_path):
    root = _make_images(str(tmp_path / "train"), per=4)

    def make(seed):
        # the loader draws from the workflow PRNG (-r seeds it)
        random_generator.get().seed(seed)
        ld = FullBatchFileImageLoader(
            DummyWorkflow(), train_paths=[root], size=(12, 10),
            crop=(6, 8), crop_number=2, mirror="random",
            rotations=(0.0, 0.3), add_sobel=True, background_color=(9, 9, 9),
            minibatch_size=8, normalization_type="none")
        return _init(ld), _serve(ld, 3)

    (a, sa), (_, sb), (_, sc) = make(5), make(5), make(6)
    assert a.sample_shape == (6, 8, 4)
    assert a.class_lengths[TRAIN] == 8 * 2 * 2
    for x, y in zip(sa, sb):
        assert torch.equal(x[2], y[2]) and torch.equal(x[4], y[4])
    assert any(not torch.equal(x[2], y[2]) for x, y in zip(sa, sc))
    # labels follow the canvases: cat images are dark, dog images bright
    d, lab = sa[0][2], sa[0][3]
    mean_rgb = d[..., :3].mean(dim=(1, 2, 3))
    assert all((m > 100) == bool(v == a.labels_mapping["dog"])
               for m, v in zip(mean_rgb.tolist(), lab.tolist()))


def test_full_batch_mirror_true_serves_both_orientations(tmp_path):
    root = _make_images(str(tmp_path / "train"), per=1, classes=("a",))
    ld = _init(FullBatchFileImageLoader(
        DummyWorkflow(), train_paths=[root], size=(12, 10), mirror=True,
        minibatch_size=2, normalization_type="none", shuffle_limit=0))
    (cls, n, data, _, idx), = _serve(ld)
    assert n == 2
    canvas = torch.from_numpy(ld.original_data.mem[0]).float()
    imgs = {int(i): data[k] for k, i in enumerate(idx.tolist())}
    assert torch.equal(imgs[0], canvas)
    assert torch.equal(imgs[1], canvas.flip(1))


def test_full_batch_normalizer_sees_served_crops(tmp_path):
    root = _make_images(str(tmp_path / "train"), per=3)
    ld = _init(FullBatchFileImageLoader(
        DummyWorkflow(), train_paths=[root], size=(12, 10), crop=(4, 4),
        minibatch_size=6, normalization_type="mean_disp"))
    mean, rdisp = ld._affine_served()
    assert mean.shape == (4 * 4 * 3,)
    (_, n, data, _, _), = _serve(ld)
    # normalised over the TRAIN crops: roughly zero-mean
    assert abs(float(data[:n].mean())) < 1.0


# ------------------------------------------------------------- streaming
@pytest.mark.parametrize("prefetch,workers",
                         [(True, 2), (False, 2), (True, 1)])
@pytest.mark.timeout(60)
def test_streaming_file_image_loader_prefetches(tmp_path, prefetch, workers):
    """decode_workers=1 with prefetch: the prefetch job must not hold the
    only decode worker while it waits on the decode pool (it deadlocked)."""
    root = _make_images(str(tmp_path / "train"), per=6)
    ld = _init(FileImageLoader(
        DummyWorkflow(), train_paths=[root], size=(12, 10), crop=(8, 8),
        mirror="random", minibatch_size=4, normalization_type="mean_disp",
        prefetch=prefetch, decode_workers=workers))
    assert ld.class_lengths == [0, 0, 12]
    assert ld.reversed_labels_mapping == ["cat", "dog"]
    served = _serve(ld, 6)          # two epochs of 3 minibatches
    assert all(s[2].shape == (4, 8, 8, 3) for s in served)
    seen = torch.cat([s[4][:s[1]] for s in served[:3]]).sort().values
    assert seen.tolist() == list(range(12))
    if prefetch:
        # inside a pass the next minibatch was already decoded
        assert ld.prefetch_hits >= 2
    else:
        assert ld.prefetch_hits == 0
    ld.stop()


def test_streaming_equals_full_batch(tmp_path):
    """Same files, same seed, same augmentation: the streaming loader
    serves exactly what the full-batch one does."""
    root = _make_images(str(tmp_path / "train"), per=5)
    outs = []
    for cls in (FullBatchFileImageLoader, FileImageLoader):
        random_generator.get().seed(11)
        ld = _init(cls(DummyWorkflow(), train_paths=[root], size=(12, 10),
                       crop=(6, 6), crop_number=2, mirror=True,
                       minibatch_size=4, normalization_type="mean_disp"))
        outs.append(_serve(ld, 5))
    for a, b in zip(*outs):
        assert a[1] == b[1]
        assert torch.equal(a[4], b[4])
        torch.testing.assert_close(a[2], b[2], rtol=1e-5, atol=1e-4)
        assert torch.equal(a[3], b[3])


def test_file_list_streaming_trains(tmp_path):
    _make_images(str(tmp_path))
    lst = tmp_path / "train.txt"
    with open(lst, "w") as f:
        for c in ("cat", "dog"):
            for i in range(6):
                f.write("%s/%s_%d.png %s\n" % (c, c, i, c))
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="file_list_image",
        loader_config={"train_list": str(lst), "size": (12, 10),
                       "crop": (8, 8), "minibatch_size": 4,
                       "validation_ratio": 0.34,
                       "normalization_type": "mean_disp"},
        layers=[{"type": "conv_relu", "->": {"n_kernels": 4, "kx": 3,
                                             "ky": 3}, "<-": gd_params(0.1)},
                {"type": "softmax", "->": {"output_sample_shape": 2},
                 "<-": gd_params(0.1)}],
        decision_config={"max_epochs": 5})
    wf.initialize(device=Device(backend="cpu"))
    ld = wf.loader
    # stratified: 2 of 6 of each label in VALID
    assert ld.class_lengths == [0, 4, 8]
    v = [k for k in ld.class_keys[VALID]]
    assert sum("cat" in k for k in v) == 2 and sum("dog" in k for k in v) == 2
    wf.run()
    assert wf.decision.epoch_n_err_pt[VALID] <= 50.0
    ld.stop()


# ----------------------------------------------------------------- labels
def test_stratified_split_keeps_label_proportions():
    prng = random_generator.RandomGenerator("s")
    prng.seed(3)
    labels = [0] * 50 + [1] * 30 + [2] * 20
    v, t = stratified_split(labels, 0.2, prng)
    assert sorted(v + t) == list(range(100))
    lv = [labels[i] for i in v]
    assert (lv.count(0), lv.count(1), lv.count(2)) == (10, 6, 4)
    prng.seed(3)
    assert stratified_split(labels, 0.2, prng) == (v, t)
    with pytest.raises(LoaderError):
        stratified_split([0, 0, 1], 0.5, prng)


def test_full_batch_validation_ratio_is_stratified(tmp_path):
    root = _make_images(str(tmp_path / "train"), per=8)
    ld = _init(FullBatchFileImageLoader(
        DummyWorkflow(), train_paths=[root], size=(12, 10),
        validation_ratio=0.25, minibatch_size=4,
        normalization_type="none"))
    assert ld.class_lengths == [0, 4, 12]
    per = ld.class_labels()
    assert sorted(per[VALID]) == ["cat", "cat", "dog", "dog"]
    assert ld.label_stats["train"]["min"] == 6
    assert ld.label_distribution_p["validation"] > 0.95


def test_label_distribution_check_and_unknown_labels():
    same = distribution_pvalue({"a": 50, "b": 50}, {"a": 10, "b": 10})
    skew = distribution_pvalue({"a": 50, "b": 50}, {"a": 19, "b": 1})
    assert same > 0.95 and skew < 0.05

    class L(object):
        labels_mapping = {}
        reversed_labels_mapping = []
        msgs = []

        def info(self, *a):
            self.msgs.append(("info", a[0] % a[1:]))

        def warning(self, *a):
            self.msgs.append(("warning", a[0] % a[1:]))

    from veles_amd.loader.labels import setup_labels_mapping
    ld = L()
    setup_labels_mapping(ld, [{}, {"x": 2}, {"x": 5, "y": 5}])
    assert ld.labels_mapping == {"x": 0, "y": 1}
    assert any(k == "warning" and "never occur" in m for k, m in ld.msgs)
    ld2 = L()
    with pytest.raises(LoaderError):
        setup_labels_mapping(ld2, [{"z": 1}, {}, {"x": 5}])


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("sobel,bgimg", [(False, False), (True, True)])
def test_image_batch_kernel_matches_reference(sobel, bgimg):
    """hvk_image_batch against the f32 torch reference: crops, mirrors,
    arbitrary rotations (bilinear, background at the edges), the Sobel
    channel, per-feature normalisation, padding rows (idx -1)."""
    g = torch.Generator().manual_seed(1)
    src = torch.randint(0, 256, (5, 21, 23, 3), dtype=torch.uint8,
                        generator=g)
    B, Ho, Wo = 7, 15, 17
    idx = torch.tensor([4, 0, 2, -1, 1, 3, 0], dtype=torch.int32)
    ang = torch.rand(B, generator=g) * 6.0 - 3.0
    ang[0] = 0.0
    p = torch.stack([torch.randint(0, 7, (B,), generator=g).float(),
                     torch.randint(0, 7, (B,), generator=g).float(),
                     torch.cos(ang), torch.sin(ang),
                     (torch.rand(B, generator=g) < 0.5).float(),
                     torch.zeros(B)], 1)
    Co = 3 + (1 if sobel else 0)
    mean = torch.rand(Ho * Wo * Co, generator=g) * 100
    rdisp = torch.rand(Ho * Wo * Co, generator=g) * 0.05
    bg = torch.randint(0, 256, (Ho, Wo, 3), dtype=torch.uint8, generator=g) \
        if bgimg else None
    color = torch.tensor([10.0, 200.0, 30.0])
    ref = ops.image_batch_ref(src, idx, p, Ho, Wo, sobel, mean, rdisp, bg,
                              color)
    out = torch.zeros(B, Ho, Wo, Co, dtype=torch.bfloat16, device="cuda")
    cu = (lambda t: None if t is None else t.cuda())
    ops.image_batch(src.cuda(), idx.cuda(), p.cuda(), out, sobel, cu(mean),
                    cu(rdisp), cu(bg), cu(color))
    torch.cuda.synchronize()
    o = out.float().cpu()
    assert float(o[3].abs().max()) == 0.0
    # bf16 output; rotated taps can round to a neighbouring source pixel
    # where sx / sy lands within float error of an integer
    err = (o - ref).abs() / (ref.abs() + 1.0)
    assert float((err > 2e-2).float().mean()) < 2e-3
    assert float(err[0].max()) < 1e-2   # unrotated sample: exact taps


@pytest.mark.gpu
def test_streaming_loader_on_gpu(tmp_path):
    """Pinned staging, side-stream copies and the device kernel: the GPU
    streaming loader serves what the CPU one does."""
    root = _make_images(str(tmp_path / "train"), per=6)
    outs = []
    for backend in ("cpu", "hip"):
        random_generator.get().seed(4)
        ld = FileImageLoader(DummyWorkflow(), train_paths=[root],
                             size=(12, 10), crop=(8, 8), mirror="random",
                             minibatch_size=4,
                             normalization_type="mean_disp")
        ld.initialize(device=Device(backend=backend))
        outs.append(_serve(ld, 6))
        if backend == "hip":
            torch.cuda.synchronize()
            assert ld.prefetch_hits >= 2
        ld.stop()
    for a, b in zip(*outs):
        assert torch.equal(a[4].cpu(), b[4].cpu())
        torch.testing.assert_close(b[2].float().cpu(), a[2].float(),
                                   rtol=2e-2, atol=2e-2)
