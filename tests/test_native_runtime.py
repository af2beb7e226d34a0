"""Native runtime (csrc/runtime, the libVeles equivalent): a package written
by Workflow.package_export must produce the same forward pass in C++ as the
Python units (reference test strategy: libVeles/tests/workflow_loader.cc,
memory_optimizer.cc)."""
import json
import subprocess
import zipfile

import numpy
import pytest
import torch

from veles_amd.backends import Device
from veles_amd.dummy import DummyLauncher
from veles_amd.models import StandardWorkflow
from veles_amd.models.zoo import gd_params
import veles_amd.loader  # noqa: F401

rt = pytest.importorskip("veles_amd.runtime")

LAYERS = [
    {"type": "conv_str", "->": {"n_kernels": 16, "kx": 3, "ky": 3,
                                "padding": 1}, "<-": gd_params(0.01)},
    {"type": "norm", "n": 5, "alpha": 1e-3, "beta": 0.75, "k": 1.0},
    {"type": "max_pooling", "->": {"kx": 3, "ky": 3, "sliding": 2}},
    {"type": "conv", "->": {"n_kernels": 24, "kx": 3, "ky": 3,
                            "sliding": 2}, "<-": gd_params(0.01)},
    {"type": "activation_tanh"},
    {"type": "avg_pooling", "->": {"kx": 2, "ky": 2, "sliding": 2}},
    {"type": "all2all_relu", "->": {"output_sample_shape": 40},
     "<-": gd_params(0.01)},
    {"type": "dropout", "dropout_ratio": 0.5},
    {"type": "softmax", "->": {"output_sample_shape": 10},
     "<-": gd_params(0.01)}]


def _trained_workflow():
    torch.manual_seed(3)
    wf = StandardWorkflow(
        DummyLauncher(), loader_name="synthetic_images",
        loader_config={"dataset": "cifar", "class_lengths": (0, 0, 64),
                       "minibatch_size": 16, "seed": 5},
        layers=LAYERS, decision_config={"max_epochs": None})
    wf.decision.fail_iterations = None
    wf.initialize(device=Device(backend="cpu"))
    wf.run_steps(2)
    return wf


def _python_forward(wf, x):
    wf.loader.minibatch_data.devmem.copy_(torch.from_numpy(x))
    for f in wf.forwards:
        if hasattr(f, "forward_mode"):
            f.forward_mode = True
        f.run()
    return wf.forwards[-1].output.devmem.float().numpy()


def test_memory_optimizer_bindings():
    h, pos = rt.optimize_memory([(i, i + 2, 1) for i in range(6)])
    assert h == 2
    assert all(p in (0, 1) for p in pos)
    nodes = [(0, 3, 3), (1, 2, 2), (2, 5, 1), (3, 6, 2), (0, 6, 1),
             (4, 6, 3)]
    h, pos = rt.optimize_memory(nodes)
    for i, a in enumerate(nodes):
        for j, b in enumerate(nodes[:i]):
            if a[0] < b[1] and b[0] < a[1]:
                assert pos[i] + a[2] <= pos[j] or pos[j] + b[2] <= pos[i]
    assert h <= 6 + 2


def test_cpp_selftests():
    rt.build_runtime()
    r = subprocess.run([rt.TEST_BIN], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_cpp_selftests_under_host_sanitizers(kind):
    """ASan+UBSan and TSan builds of the C++ self-tests (memory optimizer,
    JSON / npy parsers, unit factory, thread-pool engine) must run clean."""
    exe, env = rt.build_sanitized_tests(kind)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr[-4000:] + r.stdout
    assert "OK 0" in r.stdout
    assert "runtime error" not in r.stderr  # UBSan reports


@pytest.mark.parametrize("fmt", ["zip", "tgz"])
def test_native_forward_matches_python(tmp_path, fmt):
    wf = _trained_workflow()
    pkg = str(tmp_path / ("pkg." + ("zip" if fmt == "zip" else "tar.gz")))
    wf.package_export(pkg, archive_format=fmt)
    x = numpy.random.RandomState(0).uniform(
        -1, 1, tuple(wf.loader.minibatch_data.shape)).astype(numpy.float32)
    ref = _python_forward(wf, x)
    nw = rt.NativeWorkflow(pkg)
    assert nw.unit_classes[0] == "ConvStrictRELU"
    assert "LRNormalizerForward" in nw.unit_classes
    nw.initialize(x.shape, gpu=False)
    y = nw.run(x)
    assert y.shape == ref.shape
    numpy.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5)
    # arena reuse: far less than the sum of all unit outputs
    assert 0 < nw.arena_bytes


def test_cli(tmp_path):
    wf = _trained_workflow()
    pkg = str(tmp_path / "pkg.zip")
    wf.package_export(pkg)
    x = numpy.random.RandomState(1).uniform(
        -1, 1, tuple(wf.loader.minibatch_data.shape)).astype(numpy.float32)
    ref = _python_forward(wf, x)
    numpy.save(tmp_path / "x.npy", x)
    numpy.save(tmp_path / "ref.npy", ref)
    r = subprocess.run([rt.CLI, pkg, str(tmp_path / "x.npy"),
                        str(tmp_path / "y.npy")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    y = numpy.load(tmp_path / "y.npy")
    numpy.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5)
    r = subprocess.run([rt.TEST_BIN, pkg, str(tmp_path / "x.npy"),
                        str(tmp_path / "ref.npy")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    c = json.loads(zipfile.ZipFile(pkg).read("contents.json"))
    assert len(c["units"]) == len(LAYERS)


@pytest.mark.gpu
def test_native_forward_gpu_matches_cpu(tmp_path):
    """The HIP path (bf16 activations through libhvk) vs the float32 CPU
    path of the same package."""
    wf = _trained_workflow()
    pkg = str(tmp_path / "pkg.zip")
    wf.package_export(pkg)
    x = numpy.random.RandomState(2).uniform(
        -1, 1, tuple(wf.loader.minibatch_data.shape)).astype(numpy.float32)
    cpu = rt.NativeWorkflow(pkg)
    cpu.initialize(x.shape, gpu=False)
    ref = cpu.run(x)
    gpu = rt.NativeWorkflow(pkg)
    gpu._gpu = True
    gpu.initialize(x.shape, gpu=True)
    y = gpu.run(x)
    numpy.testing.assert_allclose(y, ref, atol=3e-2)
    assert numpy.argmax(y, 1).tolist() == numpy.argmax(ref, 1).tolist() or \
        numpy.mean(numpy.argmax(y, 1) == numpy.argmax(ref, 1)) > 0.9


# The reference's own fixtures (libVeles/tests/workflow_files, exported by
# the reference from its MNIST workflow): the runtime must load both archive
# formats and compute the forward the packaged arrays define.
REF_FIX = "/root/reference/libVeles/tests/workflow_files"


def _numpy_forward_from_package(pkg, x):
    """All2AllTanh (1.7159 * tanh(0.6666 v)) -> All2AllSoftmax from the
    package's own .npy arrays (loaded with allow_pickle=False)."""
    import io
    import tarfile
    if pkg.endswith(".zip"):
        z = zipfile.ZipFile(pkg)
        read = z.read
    else:
        t = tarfile.open(pkg)
        read = lambda n: t.extractfile(n).read()  # noqa: E731
    c = json.loads(read("contents.json"))
    arrays = {}
    for u in c["units"]:
        for k, v in u["data"].items():
            if isinstance(v, str) and v.startswith("@"):
                arrays[v] = numpy.load(io.BytesIO(read(v[1:] + ".npy")),
                                       allow_pickle=False)
    h = x.reshape(len(x), -1).astype(numpy.float64)
    for u in c["units"]:
        w = arrays[u["data"]["weights"]].astype(numpy.float64)
        b = arrays[u["data"]["bias"]].astype(numpy.float64)
        v = h @ w.T + b
        if u["class"]["name"] == "All2AllTanh":
            h = 1.7159 * numpy.tanh(0.6666 * v)
        else:
            e = numpy.exp(v - v.max(1, keepdims=True))
            h = e / e.sum(1, keepdims=True)
    return h.astype(numpy.float32)


@pytest.mark.skipif(not __import__("os").path.isdir(REF_FIX),
                    reason="reference fixtures absent")
@pytest.mark.parametrize("name", ["mnist.zip", "mnist.tar.gz"])
@pytest.mark.parametrize("threads", [0, 3])
def test_reference_fixture_packages(tmp_path, name, threads):
    pkg = REF_FIX + "/" + name
    x = numpy.random.RandomState(7).uniform(0, 1, (5, 784)).astype(
        numpy.float32)
    ref = _numpy_forward_from_package(pkg, x)
    nw = rt.NativeWorkflow(pkg)
    assert nw.unit_classes == ["All2AllTanh", "All2AllSoftmax"]
    nw.set_engine(threads)
    nw.initialize(x.shape, gpu=False)
    y = nw.run(x)
    assert y.shape == (5, 10)
    numpy.testing.assert_allclose(y, ref, rtol=1e-5, atol=2e-6)
    # the same through the C++ test binary and the CLI
    numpy.save(tmp_path / "x.npy", x)
    numpy.save(tmp_path / "ref.npy", ref)
    r = subprocess.run([rt.TEST_BIN, pkg, str(tmp_path / "x.npy"),
                        str(tmp_path / "ref.npy")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    r = subprocess.run([rt.CLI, pkg, str(tmp_path / "x.npy"),
                        str(tmp_path / "y.npy"), "--threads", "2",
                        "--repeat", "3"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    numpy.testing.assert_allclose(numpy.load(tmp_path / "y.npy"), ref,
                                  rtol=1e-5, atol=2e-6)


@pytest.mark.gpu
def test_native_branch_streams_and_graph_on_gpu():
    """Branches of a DAG on their own HIP streams joined by events, pooled
    host enqueue, and a captured + replayed hipGraph of the pass
    (veles_rt_tests --gpu-branch)."""
    rt.build_runtime()
    r = subprocess.run([rt.TEST_BIN, "--gpu-branch"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "OK 0" in r.stdout


@pytest.mark.gpu
def test_native_reference_fixture_gpu_graph(tmp_path):
    pkg = REF_FIX + "/mnist.zip"
    if not __import__("os").path.exists(pkg):
        pytest.skip("reference fixtures absent")
    x = numpy.random.RandomState(8).uniform(0, 1, (64, 784)).astype(
        numpy.float32)
    ref = _numpy_forward_from_package(pkg, x)
    nw = rt.NativeWorkflow(pkg)
    nw._gpu = True
    nw.enable_graph(True)
    nw.initialize(x.shape, gpu=True)
    for _ in range(3):
        y = nw.run(x)
        numpy.testing.assert_allclose(y, ref, atol=2e-2)
    assert nw.graph_active
