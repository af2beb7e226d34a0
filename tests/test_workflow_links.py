"""The optional StandardWorkflow link_* builders (reference
docs/source/manualrst_veles_workflow_creation.rst:103-640): a user
create_workflow() that wires every one of them around the canonical cycle,
trains on the CPU and checks what each unit produced."""
import os

import numpy
import pytest
import torch

from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import mnist_fc
from veles_amd.utils.config import root
import veles_amd.loader  # noqa: F401


class AllLinks(StandardWorkflow):
    """Serial (rule 1) and parallel (rules 1-2) linking of every builder."""

    def create_workflow(self):
        self.link_repeater(self.start_point)
        self.link_loader(self.repeater)
        self.link_data_saver(self.loader)
        self.link_forwards(("input", "minibatch_data"), self.data_saver)
        self.link_evaluator(self.forwards[-1])
        self.link_decision(self.evaluator)
        end_units = [link(self.decision) for link in (
            self.link_error_plotter, self.link_conf_matrix_plotter,
            self.link_min_max_plotter, self.link_multi_hist_plotter,
            self.link_weights_plotter, self.link_immediate_plotter,
            self.link_image_plotter)]
        end_units.append(self.link_similar_weights_plotter(self.decision))
        saver = self.link_image_saver(self.decision)
        shell = self.link_ipython(saver)
        last = self.link_result_unit(shell)
        self.link_gds(*end_units, last)
        self.link_table_plotter(self.gds[0])
        self.link_loop(self.table_plotter)
        # the report waits for the last plotter of every parallel branch
        self.link_publisher(*end_units)
        self.link_end_point(self.publisher)


@pytest.fixture
def plot_dirs(tmp_path):
    old = (root.common.dirs.plots, root.common.disable.plotting,
           root.common.disable.publishing)
    root.common.dirs.plots = str(tmp_path / "plots")
    root.common.disable.plotting = False
    root.common.disable.publishing = False
    yield tmp_path
    (root.common.dirs.plots, root.common.disable.plotting,
     root.common.disable.publishing) = old


def test_every_builder_in_one_workflow(plot_dirs):
    tmp = plot_dirs
    wf = AllLinks(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "mnist", "class_lengths": (60, 100, 400),
                       "minibatch_size": 50, "normalization_type":
                       "mean_disp", "seed": 7, "noise": 110.0},
        layers=mnist_fc(), decision_config={"max_epochs": 3,
                                            "fail_iterations": 100},
        data_saver_config={"file_name": str(tmp / "mb.dat")},
        image_saver_config={"out_dir": str(tmp / "images"), "limit": 5,
                            "only_errors": False},
        publisher_config={"output": str(tmp / "report.md")},
        result_unit_config={"package": str(tmp / "fwd.zip")})
    for p in wf.error_plotters + wf.min_max_plotters + \
            wf.multi_hist_plotters:
        p.redraw_threshold = 0
    for p in (wf.conf_matrix_plotter, wf.weights_plotter,
              wf.similar_weights_plotter, wf.immediate_plotter,
              wf.image_plotter, wf.table_plotter):
        p.redraw_threshold = 0
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    assert wf.finished
    wf.stop()  # the launcher does this at exit: finalises the data file
    # one accumulated point per epoch and class series
    assert [len(p.values) for p in wf.error_plotters] == [3, 3, 3]
    assert wf.error_plotters[1].values == pytest.approx(
        [h["train_err_pt"] for h in wf.decision.history])
    assert len(wf.min_max_plotters[0].values) == 3
    assert wf.min_max_plotters[0].values[0] >= wf.min_max_plotters[1].values[0]
    files = os.listdir(tmp / "plots")
    for name in ("errors_validation.png", "errors_train.png",
                 "confusion_matrix.png", "output_max.png",
                 "weights_all2all_tanh0.png",
                 "similar_weights_all2all_tanh0.png", "immediate.png",
                 "output_images.png", "histogram_all2all_tanh0.png"):
        assert name in files, files
    assert "max_min.txt" in files
    table = open(tmp / "plots" / "max_min.txt").read()
    assert "weights" in table and "gradient" in table
    # confusion matrix: validation samples by (true, predicted)
    cm = numpy.asarray(wf.evaluator.confusion_matrix.mem)
    assert cm.shape == (10, 10) and cm.sum() == 100
    # the (synthetic, quickly learnt) samples of the last improving pass,
    # `limit` per class, named true_as_predicted.index.png
    for cls in ("validation", "train"):
        d = tmp / "images" / cls
        pngs = sorted(f for f in os.listdir(d) if f.endswith(".png"))
        assert len(pngs) == 5
        true, _, pred = pngs[0].split(".")[0].partition("_as_")
        assert 0 <= int(true) < 10 and 0 <= int(pred) < 10
    # every served minibatch was saved
    from veles_amd.loader.saver import read_minibatches
    recs = list(read_minibatches(str(tmp / "mb.dat")))
    # 3 epochs end at the validation pass: 4 + 2 x (8 train + 4) minibatches
    assert len(recs) == 28 and {c for c, _ in recs} == {0, 1, 2}
    # the inference workflow was extracted and exported once, at the end
    assert wf.result_unit.extractions == 1
    assert wf.result_unit.forward_workflow is not None
    assert os.path.getsize(tmp / "fwd.zip") > 1000
    # the report lists the plots
    rep = open(tmp / "report.md").read()
    assert "errors" in rep


def test_meandispnorm_and_avatar_link():
    """link_meandispnorm feeds the forwards from the normalizer output and
    link_avatar clones the loader's minibatch (rule 6: loader from
    start_point)."""

    class Norm(StandardWorkflow):
        def create_workflow(self):
            self.link_loader(self.start_point)
            self.link_repeater(self.loader)
            self.link_avatar(self.repeater)
            self.link_meandispnorm(self.avatar)
            self.meandispnorm.link_attrs(self.avatar,
                                         ("input", "minibatch_data"))
            last = self.link_forwards(("input", "output"), self.meandispnorm)
            last = self.link_evaluator(last)
            last = self.link_decision(last)
            self.link_gds(last)
            self.link_loop(self.gds[0])
            self.link_end_point(self.decision)

    wf = Norm(DummyLauncher(), loader_name="synthetic_images",
              loader_config={"dataset": "mnist", "class_lengths": (0, 50, 200),
                             "minibatch_size": 50, "seed": 3,
                             "normalization_type": "mean_disp"},
              layers=mnist_fc(), decision_config={"max_epochs": 2})
    wf.initialize(device=Device(backend="cpu"))
    wf.run()
    assert wf.finished
    x = wf.avatar.minibatch_data.devmem
    y = wf.meandispnorm.output.devmem
    assert y.shape == x.shape
    assert wf.forwards[0].input is wf.meandispnorm.output
    # the loader served raw samples; the unit applied its mean / rdisp
    mean = torch.from_numpy(wf.loader.mean.mem)
    rdisp = torch.from_numpy(wf.loader.rdisp.mem)
    assert float(x.max()) > 10  # raw (uint8-range) pixels
    torch.testing.assert_close(y, (x - mean) * rdisp, rtol=1e-5, atol=1e-5)


def test_similarity_order_chains_similar_rows():
    from veles_amd.plotting_units import similarity_order
    rng = numpy.random.RandomState(0)
    base = rng.randn(3, 16)
    rows = numpy.stack([base[0], base[1], base[0] * 1.01, base[2],
                        base[1] + 1e-3])
    order = list(similarity_order(rows))
    assert sorted(order) == list(range(5))
    pos = {v: i for i, v in enumerate(order)}
    assert abs(pos[0] - pos[2]) == 1 and abs(pos[1] - pos[4]) == 1


def test_image_saver_keeps_only_misclassified(tmp_path):
    from veles_amd.memory import Array
    from veles_amd.models.image_saver import ImageSaver
    wf = StandardWorkflow(DummyLauncher(), loader_name="synthetic_images",
                          loader_config={"dataset": "mnist",
                                         "class_lengths": (0, 10, 20),
                                         "minibatch_size": 10},
                          layers=mnist_fc())
    s = ImageSaver(wf, out_dir=str(tmp_path), limit=3)
    x = numpy.random.RandomState(0).rand(6, 28, 28).astype(numpy.float32)
    out = numpy.eye(10, dtype=numpy.float32)[[1, 2, 3, 4, 5, 6]]
    s.input, s.output = Array(x), Array(out)
    s.labels = Array(numpy.array([1, 0, 3, 0, 0, 0], numpy.int32))
    s.indices = Array(numpy.arange(6, dtype=numpy.int32))
    s.minibatch_class, s.minibatch_size, s.minibatch_offset = 1, 6, 16
    s.initialize()
    s.run()
    files = sorted(os.listdir(tmp_path / "validation"))
    # 4 misclassified (indices 1, 3, 4, 5), at most limit=3 written
    assert files == ["0_as_2.1.png", "0_as_4.3.png", "0_as_5.4.png"]
    from PIL import Image
    assert Image.open(tmp_path / "validation" / files[0]).size == (28, 28)


def test_avatar_snapshots_host_state():
    """Avatar (reference veles/avatar.py:38-73): non-Array attributes are
    snapshots taken when the avatar runs - the producer can advance (its
    flags, offsets, lists, dicts, arrays) without the avatar's copy, or the
    identity of the objects consumers hold, changing."""
    from veles_amd.avatar import Avatar
    from veles_amd.dummy import DummyWorkflow
    from veles_amd.memory import Array
    from veles_amd.mutable import Bool
    from veles_amd.units import TrivialUnit

    wf = DummyWorkflow()
    src = TrivialUnit(wf)
    src.flag = Bool(False)
    src.offset = 10
    src.lengths = [1, 2, 3]
    src.table = {"a": 1}
    src.hist = numpy.arange(4, dtype=numpy.float32)
    src.data = Array(numpy.arange(6, dtype=numpy.float32))
    dev = Device(backend="cpu")
    src.data.initialize(dev)
    av = Avatar(wf)
    av.clone(src, "flag", "offset", "lengths", "table", "hist", "data")
    av.initialize(device=dev)
    held = (av.flag, av.lengths, av.table, av.hist)
    av.run()
    assert not av.flag and av.offset == 10 and av.lengths == [1, 2, 3]
    assert av.flag is not src.flag and av.lengths is not src.lengths
    # the producer runs ahead
    src.flag <<= True
    src.offset = 11
    src.lengths.append(4)
    src.table["b"] = 2
    src.hist += 1
    src.data.map_write()
    src.data.mem[:] = -1
    assert not av.flag and av.offset == 10 and av.lengths == [1, 2, 3]
    assert av.table == {"a": 1} and av.hist[0] == 0
    assert float(av.data.devmem[1]) == 1.0
    # the next run takes the new snapshot into the SAME objects
    av.run()
    assert av.flag and av.offset == 11 and av.lengths == [1, 2, 3, 4]
    assert av.table == {"a": 1, "b": 2} and av.hist[0] == 1
    assert float(av.data.devmem[1]) == -1.0
    assert all(a is b for a, b in zip(held, (av.flag, av.lengths, av.table,
                                             av.hist)))
