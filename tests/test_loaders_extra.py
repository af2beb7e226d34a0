"""File / image / pickle / ensemble / minibatch-file / HDF5 loaders
(reference loader/*.py)."""
import json
import os
import pickle

import numpy
import pytest
import torch

from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher, DummyWorkflow
from veles_amd.loader import (
    EnsembleLoader, FullBatchFileListImageLoader, FullBatchFileImageLoader,
    FullBatchHDF5Loader, MinibatchesLoader, MinibatchesSaver,
    PicklesImageFullBatchLoader, TRAIN, VALID, TEST)
from veles_amd.loader.file_loader import FileFilter, scan_files
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import gd_params


def _make_images(root, classes=("cat", "dog"), per=6, size=(10, 12)):
    from PIL import Image
    rs = numpy.random.RandomState(0)
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


def test_file_filter_and_scan(tmp_path):
    _make_images(str(tmp_path))
    open(tmp_path / "cat" / "notes.txt", "w").write("x")
    files = scan_files(str(tmp_path))
    assert len(files) == 12 and all(f.endswith(".png") for f in files)
    ff = FileFilter(ignored=[r"dog_[0-2]"])
    assert len(scan_files(str(tmp_path), ff)) == 9


def test_full_batch_file_image_loader_trains(tmp_path):
    tr = _make_images(str(tmp_path / "train"))
    va = _make_images(str(tmp_path / "valid"), per=2)
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="full_batch_file_image",
        loader_config={"train_paths": [tr], "validation_paths": [va],
                       "size": (8, 8), "minibatch_size": 4,
                       "mirror": True, "normalization_type": "mean_disp"},
        layers=[{"type": "conv_relu", "->": {"n_kernels": 4, "kx": 3,
                                             "ky": 3}, "<-": gd_params(0.1)},
                {"type": "softmax", "->": {"output_sample_shape": 2},
                 "<-": gd_params(0.1)}],
        decision_config={"max_epochs": 6})
    wf.initialize(device=Device(backend="cpu"))
    ld = wf.loader
    # mirror=True serves every canvas plain and flipped (inflation 2)
    assert ld.class_lengths == [0, 8, 24]
    assert tuple(ld.original_data.shape) == (16, 8, 8, 3)
    assert ld.reversed_labels_mapping == ["cat", "dog"]
    wf.run()
    assert wf.decision.epoch_n_err_pt[VALID] <= 25.0


def test_file_list_loader(tmp_path):
    _make_images(str(tmp_path))
    lst = tmp_path / "train.txt"
    with open(lst, "w") as f:
        for c in ("cat", "dog"):
            for i in range(3):
                f.write("%s/%s_%d.png %s\n" % (c, c, i, c))
    ld = FullBatchFileListImageLoader(DummyWorkflow(), train_list=str(lst),
                             size=(6, 6), color_space="GRAY",
                             minibatch_size=2)
    _init(ld)
    assert tuple(ld.original_data.shape) == (6, 6, 6, 1)
    assert list(ld.original_labels) == [0, 0, 0, 1, 1, 1]


def test_pickles_loader_cifar_layout(tmp_path):
    rs = numpy.random.RandomState(1)
    data = rs.randint(0, 255, (5, 3 * 4 * 4)).astype(numpy.uint8)
    labels = [3, 1, 3, 0, 1]
    p = tmp_path / "batch"
    with open(p, "wb") as f:
        pickle.dump({b"data": data, b"labels": labels}, f)
    ld = PicklesImageFullBatchLoader(DummyWorkflow(), train_pickles=[str(p)],
                                     shape=(4, 4, 3), minibatch_size=5)
    _init(ld)
    img = ld.original_data.mem
    assert img.shape == (5, 4, 4, 3)
    # channel-planar -> NHWC
    numpy.testing.assert_array_equal(img[2, 1, 3, 2], data[2, 2 * 16 + 1 * 4
                                                             + 3])
    assert ld.reversed_labels_mapping == [0, 1, 3]
    assert list(ld.original_labels) == [2, 1, 2, 0, 1]


def test_ensemble_loader(tmp_path):
    out_a = numpy.eye(3)[[0, 1, 2, 0]].tolist()
    out_b = numpy.eye(3)[[0, 2, 1, 0]][:, [1, 0, 2]].tolist()
    ens = {"models": [{"id": 0, "Output": out_a, "Labels": [0, 1, 2]},
                      {"id": 1, "Output": out_b, "Labels": [1, 0, 2]}]}
    fn = tmp_path / "ens.json"
    fn.write_text(json.dumps(ens))
    ld = EnsembleLoader(DummyWorkflow(), file=str(fn), labels=[0, 1, 2, 0],
                        minibatch_size=2)
    _init(ld)
    d = ld.original_data.mem
    assert d.shape == (4, 2, 3)
    # model b remapped into model a's label order
    numpy.testing.assert_array_equal(d[1, 1], [0, 0, 1])
    assert ld.class_lengths[TRAIN] == 4
    t = EnsembleLoader(DummyWorkflow(), file=str(fn), testing=True,
                       minibatch_size=2)
    _init(t)
    assert t.class_lengths[TEST] == 4


def test_minibatches_saver_and_loader_roundtrip(tmp_path):
    from veles_amd.loader.saver import read_minibatches
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (0, 20, 60),
                       "minibatch_size": 16, "seed": 3},
        layers=[{"type": "softmax", "->": {"output_sample_shape": 10},
                 "<-": gd_params(0.1)}], decision_config={"max_epochs": 2})
    fn = str(tmp_path / "mb.dat")
    saver = MinibatchesSaver(wf, file_name=fn, compression="xz")
    saver.link_from(wf.loader)
    saver.link_attrs(wf.loader, "minibatch_data", "minibatch_size",
                     "minibatch_class", "minibatch_labels",
                     "minibatch_indices")
    wf.forwards[0].unlink_from(wf.loader)
    wf.forwards[0].link_from(saver)
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    saver.stop()
    recs = list(read_minibatches(fn))
    # epoch 0 = the first validation pass, epoch 1 = train + validation
    assert sum(len(r["data"]) for c, r in recs if c == TRAIN) == 60
    assert sum(len(r["data"]) for c, r in recs if c == VALID) == 40
    ld = MinibatchesLoader(DummyWorkflow(), file_name=fn, minibatch_size=16)
    _init(ld)
    assert ld.class_lengths == [0, 40, 60]
    first = [r for c, r in recs if c == VALID][0]
    numpy.testing.assert_allclose(ld.original_data.mem[:len(first["data"])],
                                  first["data"])


def test_hdf5_loader_reports_missing_h5py():
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py present")
    except ImportError:
        pass
    ld = FullBatchHDF5Loader(DummyWorkflow(), train_path="x.h5")
    with pytest.raises(ImportError, match="h5py"):
        ld.load_data()


_ = torch


REF_WINE = "/root/reference/veles/tests/res/wine_ensemble.json"


@pytest.mark.skipif(not os.path.exists(REF_WINE),
                    reason="reference fixture absent")
def test_ensemble_loader_on_reference_wine_results():
    """The reference's own --ensemble-train result file (3 wine models,
    178 test outputs each; veles/tests/res/wine_ensemble.json): test mode
    stacks the members' outputs per sample; with labels (the members'
    consensus here: the reference file holds no ground truth) it trains an
    ensemble-of-outputs classifier input."""
    import json as _json
    ens = _json.load(open(REF_WINE))
    t = EnsembleLoader(DummyWorkflow(), file=REF_WINE, testing=True,
                       minibatch_size=32)
    _init(t)
    assert t.class_lengths[TEST] == 178
    d = t.original_data.mem
    assert d.shape == (178, 3, 3)
    for i, m in enumerate(ens["models"]):
        numpy.testing.assert_allclose(d[:, i], numpy.asarray(m["Output"]),
                                      rtol=1e-6)
    vote = numpy.asarray([m["Output"] for m in ens["models"]]).mean(0)
    labels = vote.argmax(1).tolist()
    tr = EnsembleLoader(DummyWorkflow(), file=REF_WINE, labels=labels,
                        minibatch_size=32)
    _init(tr)
    assert tr.class_lengths[TRAIN] == 178
    assert tr.reversed_labels_mapping == [0, 1, 2]
    assert list(tr.original_labels) == labels
