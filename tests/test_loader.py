"""Loader serving order and normalizers."""
import numpy
import pytest

from veles_amd.backends import Device
from veles_amd.dummy import DummyWorkflow
from veles_amd.loader import SyntheticImageLoader, TEST, VALID, TRAIN
from veles_amd.normalization import normalizer


def make(lengths=(5, 7, 23), mb=4, **kw):
    wf = DummyWorkflow(device=Device(backend="cpu"))
    ld = SyntheticImageLoader(wf, dataset="mnist", class_lengths=lengths,
                              minibatch_size=mb, **kw)
    ld.initialize(device=wf.device)
    return ld


def test_serving_order_and_flags():
    ld = make()
    seen = []
    for _ in range(12):
        ld.run()
        seen.append((ld.minibatch_class, ld.minibatch_size,
                     bool(ld.last_minibatch), bool(ld.epoch_ended)))
    classes = [s[0] for s in seen]
    assert classes[:2] == [TEST, TEST]
    assert classes[2:4] == [VALID, VALID]
    assert classes[4:10] == [TRAIN] * 6
    sizes = [s[1] for s in seen]
    assert sizes[:4] == [4, 1, 4, 3] and sizes[9] == 3
    assert seen[3][3] is True          # epoch ends at the last VALID mb
    assert seen[9][2] is True and seen[9][3] is False
    assert classes[10] == TEST          # wrapped


def test_padding_and_shuffle_only_train():
    ld = make()
    before = ld.shuffled_indices.mem.copy()
    for _ in range(11):
        ld.run()
    after = ld.shuffled_indices.mem
    assert numpy.array_equal(before[:12], after[:12])
    assert sorted(after[12:]) == list(range(12, 35))
    ld2 = make()
    ld2.run()
    ld2.run()   # TEST remainder of 1
    lab = ld2.minibatch_labels.mem
    idx = ld2.minibatch_indices.mem
    assert (lab[1:] == -1).all() and (idx[1:] == -1).all()
    assert (ld2.minibatch_data.mem[1:] == 0).all()


def test_train_ratio():
    ld = make(train_ratio=0.5)
    assert ld.effective_total_samples == 12 + 23 - int(0.5 * 23)


def test_dp_shards_cover_global_batch():
    shards = []
    for r in range(3):
        ld = make(mb=8, rank=r, world_size=3)
        for _ in range(2):
            ld.run()
        shards.append((ld.minibatch_size,
                       ld.minibatch_indices.mem[:ld.minibatch_size].copy()))
        assert ld.global_minibatch_size == 7
    assert sum(s[0] for s in shards) == 7
    ref = make(mb=8)
    for _ in range(2):
        ref.run()
    allidx = numpy.concatenate([s[1] for s in shards])
    assert numpy.array_equal(allidx, ref.minibatch_indices.mem[:7])


@pytest.mark.parametrize("name", ["mean_disp", "linear", "range_linear",
                                  "pointwise", "internal_mean", "none",
                                  "exp"])
def test_normalizers(name):
    rs = numpy.random.RandomState(0)
    d = rs.uniform(0, 255, (20, 6)).astype(numpy.float64)
    n = normalizer(name)
    n.analyze(d)
    x = d.copy()
    n.normalize(x)
    if name == "mean_disp":
        ref = (d - d.mean(0)) / (d.max(0) - d.min(0))
        assert numpy.allclose(x, ref)
    if name == "pointwise":
        assert numpy.allclose(x.min(0), -1) and numpy.allclose(x.max(0), 1)
    if name == "range_linear":
        assert numpy.isclose(x.min(), -1) and numpy.isclose(x.max(), 1)
    if name in ("mean_disp", "pointwise", "range_linear", "internal_mean"):
        y = x.copy()
        n.denormalize(y)
        assert numpy.allclose(y, d)
        aff = n.affine()
        if aff is not None:
            m, r = aff
            assert numpy.allclose((d - m) * r, x, atol=1e-4)
