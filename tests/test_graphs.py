"""GraphSegment dispatch (veles_amd/graphs.py) on the CPU: a host-side
recorder stands in for HIP-graph capture - while "capturing", launches are
recorded instead of executed, and replay() executes the recording - so the
warmup / capture / replay / invalidation / failure state machine is pinned
without a GPU (the real capture is covered by tests/test_graphs_gpu.py)."""
import pytest
import torch

from veles_amd.graphs import GraphSegment
from veles_amd.memory import Array

_ACTIVE = []


def launch(fn):
    if _ACTIVE:
        _ACTIVE[-1].ops.append(fn)
    else:
        fn()


class FakeGraph(object):
    def __init__(self):
        self.ops = []

    def replay(self):
        for fn in self.ops:
            fn()


class _Ctx(object):
    def __init__(self, g):
        self.g = g

    def __enter__(self):
        _ACTIVE.append(self.g)

    def __exit__(self, *exc):
        _ACTIVE.remove(self.g)


class Recording(GraphSegment):
    @staticmethod
    def new_graph():
        g = FakeGraph()
        return g, _Ctx(g)


class U(object):
    """A unit whose run() does host work (log) + 'device' work (count)."""

    def __init__(self, name, log, dev, fail_in_capture=False):
        self.name = name
        self.log = log
        self.dev = dev
        self.fail_in_capture = fail_in_capture
        self.output = Array()

    def run(self):
        if self.fail_in_capture and _ACTIVE:
            raise RuntimeError("operation not permitted when capturing")
        self.log.append(self.name)
        launch(lambda: self.dev.__setitem__(self.name,
                                            self.dev.get(self.name, 0) + 1))


def _pass(seg):
    for u in seg.units:
        seg.run_unit(u)


def _make(warmup=2, **kw):
    log, dev = [], {}
    units = [U("a", log, dev), U("b", log, dev, **kw), U("c", log, dev)]
    key = [("train", 8)]
    hooks = {"pre": 0, "replay": 0}
    inp = Array()
    inp.devmem = torch.zeros(2)
    seg = Recording("t", units, lambda: key[0], lambda: [inp], warmup=warmup,
                    pre_hooks=[lambda: hooks.__setitem__("pre",
                                                         hooks["pre"] + 1)],
                    replay_hooks=[lambda: hooks.__setitem__(
                        "replay", hooks["replay"] + 1)])
    return seg, log, dev, key, hooks, inp


def test_warmup_capture_replay():
    seg, log, dev, key, hooks, _ = _make()
    for _ in range(2):
        _pass(seg)
    assert log == list("abcabc") and dev == {"a": 2, "b": 2, "c": 2}
    assert seg.captures == 0
    _pass(seg)  # captured: host code runs, the device work runs ONCE
    assert log == list("abc" * 3)
    assert dev == {"a": 3, "b": 3, "c": 3}
    assert seg.captures == 1 and hooks["replay"] == 0
    for _ in range(4):
        _pass(seg)  # replays: no host code, device work every pass
    assert log == list("abc" * 3)
    assert dev == {"a": 7, "b": 7, "c": 7}
    assert seg.replays == 4 and hooks["replay"] == 4
    assert hooks["pre"] == 7  # every eligible pass


def test_new_key_warms_up_and_captures_separately():
    seg, log, dev, key, hooks, _ = _make(warmup=1)
    for _ in range(3):
        _pass(seg)
    assert seg.captures == 1 and seg.replays == 1
    key[0] = ("valid", 8)
    _pass(seg)  # eager warmup of the new key
    assert seg.captures == 1 and log[-3:] == list("abc")
    _pass(seg)
    assert seg.captures == 2 and set(seg.graphs) == {("train", 8),
                                                     ("valid", 8)}
    key[0] = ("train", 8)
    n = len(log)
    _pass(seg)
    assert len(log) == n and seg.replays == 2
    assert dev["a"] == 6


def test_key_none_runs_eagerly():
    seg, log, dev, key, hooks, _ = _make(warmup=0)
    key[0] = None
    for _ in range(3):
        _pass(seg)
    assert seg.captures == 0 and log == list("abc" * 3)
    assert hooks["pre"] == 0


def test_moved_input_drops_the_graph():
    seg, log, dev, key, hooks, inp = _make(warmup=1)
    for _ in range(3):
        _pass(seg)
    assert seg.replays == 1
    inp.devmem = torch.ones(2)  # the loader swapped its buffer
    _pass(seg)  # graph dropped, eager warmup again
    assert seg.replays == 1 and log[-3:] == list("abc")
    _pass(seg)
    assert seg.captures == 2
    _pass(seg)
    assert seg.replays == 2
    assert dev["a"] == 6


def test_failed_capture_reruns_eagerly_and_pins_the_key():
    seg, log, dev, key, hooks, _ = _make(warmup=1, fail_in_capture=True)
    _pass(seg)
    _pass(seg)  # capture attempt: b fails -> a, b re-run eagerly, c eager
    assert seg.failures == 1 and seg.captures == 0
    assert dev == {"a": 2, "b": 2, "c": 2}
    assert key[0] in seg.eager_keys and not _ACTIVE
    _pass(seg)
    assert dev == {"a": 3, "b": 3, "c": 3} and seg.replays == 0


def test_replay_reattaches_recorded_tensors():
    seg, log, dev, key, hooks, _ = _make(warmup=1)
    b = seg.units[1]
    t_train, t_valid = torch.zeros(3), torch.zeros(4)
    orig = U.run

    def run_alias(self):
        orig(self)
        if self.name == "b":
            self.output.devmem = t_train if key[0][0] == "train" \
                else t_valid
    U.run = run_alias
    try:
        for _ in range(2):
            _pass(seg)  # train: warmup + capture
        key[0] = ("valid", 8)
        for _ in range(2):
            _pass(seg)
        assert b.output.devmem is t_valid
        key[0] = ("train", 8)
        _pass(seg)  # replay restores what the train capture left
        assert b.output.devmem is t_train
    finally:
        U.run = orig


def test_unsafe_unit_keeps_segment_eager():
    log, dev = [], {}
    u = U("x", log, dev)
    u.graph_safe = False
    seg = Recording("t", [U("a", log, dev), u], lambda: 1, warmup=0)
    for _ in range(3):
        _pass(seg)
    assert seg.captures == 0 and log == list("ax" * 3)


def test_install_is_noop_on_cpu():
    from veles_amd.graphs import install_step_graphs

    class WF(object):
        device = None
    assert install_step_graphs(WF()) == []


@pytest.mark.parametrize("seed", [0, 1, 12345, 2 ** 31 - 1, 2 ** 32 - 1])
def test_seed_advance_reference(seed):
    from veles_amd import ops
    t = torch.tensor([seed - (1 << 32) if seed >= (1 << 31) else seed],
                     dtype=torch.int32)
    ops.seed_advance(t)
    assert int(t[0]) & 0xFFFFFFFF == ops.seed_advance_ref(seed)
    x = torch.randn(1000)
    y1 = ops.dropout(x, 0.3, None, seed_dev=t)
    y2 = ops.dropout(x, 0.3, int(t[0]) & 0xFFFFFFFF)
    assert torch.equal(y1, y2)


def test_stochastic_pool_reference_draws():
    """CPU reference of hvk_stochastic_pool: drawn values sit at the drawn
    offsets, zero-probability elements are never drawn unless the window
    is all non-positive, test mode is the probability-weighted average."""
    from veles_amd import ops
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 6, 6, 4, generator=g)
    y, am = ops.stochastic_pool(x, 2, 2, (2, 2), False, True, seed=7)
    assert torch.equal(y.view(-1), x.view(-1)[am.view(-1).long()])
    win = x.unfold(1, 2, 2).unfold(2, 2, 2)  # N, 3, 3, C, 2, 2
    anypos = (win > 0).flatten(-2).any(-1)
    assert bool(((y > 0) | ~anypos).all())
    yt, _ = ops.stochastic_pool(x, 2, 2, (2, 2), False, False)
    w = win.clamp(min=0).flatten(-2)
    p = w / w.sum(-1, keepdim=True).clamp(min=1e-30)
    p = torch.where(w.sum(-1, keepdim=True) > 0, p, torch.full_like(p, .25))
    ref = (p * win.flatten(-2)).sum(-1)
    assert torch.allclose(yt, ref, atol=1e-5)
    # a different seed draws differently somewhere
    y2, am2 = ops.stochastic_pool(x, 2, 2, (2, 2), False, True, seed=8)
    assert not torch.equal(am, am2)


def test_gradient_buckets_keep_a_small_tail():
    """Buckets follow the backward order (the flat buffer is in reverse
    registration order); the last bucket - the one no backward work can
    hide - holds only the layers finishing last (<= tail_bucket_mb)."""
    import numpy
    from veles_amd.models.params import ParameterStore

    class Owner(object):
        pass
    st = ParameterStore(None)
    sizes = [("conv1", 34848), ("conv2", 307200), ("conv3", 884736),
             ("conv4", 663552), ("conv5", 442368), ("fc6", 37748736),
             ("fc7", 16777216), ("fc8", 4096000)]
    for name, n in sizes:
        o = Owner()
        o.name = name
        st.register(o, "weights", numpy.zeros(n, numpy.float32))
    st.finalize()
    names = [[p.owner.name for p in b] for b in st.buckets]
    assert names[0] == ["fc8", "fc7"] and names[1] == ["fc6"]
    assert names[-1] == ["conv2", "conv1"]  # 1.3 MB tail
    assert sum(p.size for p in st.buckets[-1]) * 4 <= 2 << 20
    assert [p for b in st.buckets for p in b] == sorted(
        st.params, key=lambda p: p.offset)


# -------------------------------------------------- validated capture
class _Val(object):
    """Validator double: device state = the units' counter dict."""

    def __init__(self, dev, ok=True):
        self.dev = dev
        self.ok = ok
        self.calls = []

    def wanted(self):
        return True

    def save(self):
        return dict(self.dev)

    def restore(self, snap):
        self.dev.clear()
        self.dev.update(snap)

    def result(self):
        return dict(self.dev)

    def compare(self, snap, got, ref):
        self.calls.append((snap, got, ref))
        return self.ok and got == ref

    def agree(self, ok):
        return ok


@pytest.mark.parametrize("ok", [True, False])
def test_validated_capture_keeps_or_pins(ok):
    """The first captured pass is compared with an eager re-run of the same
    pass from the same state: kept on a match, pinned eager on a mismatch;
    the device state after the pass is the eager pass's either way (one
    pass worth of work, not two)."""
    log, dev = [], {}
    units = [U("a", log, dev), U("b", log, dev)]
    key = [("train", 8)]
    v = _Val(dev, ok)
    seg = Recording("t", units, lambda: key[0], warmup=1, validator=v)
    _pass(seg)                      # eager warmup
    assert dev == {"a": 1, "b": 1}
    _pass(seg)                      # capture + replay, then the eager check
    assert seg.validations == [ok] and len(v.calls) == 1
    snap, got, ref = v.calls[0]
    assert snap == {"a": 1, "b": 1} and got == ref == {"a": 2, "b": 2}
    assert dev == {"a": 2, "b": 2}
    _pass(seg)
    assert dev == {"a": 3, "b": 3}
    if ok:
        assert seg.replays == 1 and key[0] not in seg.eager_keys
    else:
        assert seg.replays == 0 and key[0] in seg.eager_keys


def _validate_rank(rank, port, fail_rank, q):
    import os
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2",
                       "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    if fail_rank is not None:
        os.environ["VELES_AMD_DP_VALIDATE_FAIL_RANK"] = str(fail_rank)
    import torch
    from veles_amd.models.params import CaptureValidator
    from veles_amd.parallel.dp import DataParallel
    dp = DataParallel(backend="gloo", timeout_s=60)

    class Store(object):
        pass
    st = Store()
    st.dp = dp
    st.master = torch.zeros(8)
    st.params = []
    val = CaptureValidator(st)
    log, dev = [], {}
    units = [U("a", log, dev), U("b", log, dev)]
    seg = Recording("t", units, lambda: "k", warmup=1, validator=val)
    val.wanted = lambda: True
    val.save = lambda: {"master": st.master.clone()}
    val.restore = lambda snap: None
    for _ in range(3):
        _pass(seg)
    q.put((rank, seg.validations, "k" in seg.eager_keys, seg.replays))
    dp.shutdown()


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_validated_capture_agrees_over_gloo(fail_rank):
    """Two gloo ranks: a mismatch forced on rank 1 alone
    (VELES_AMD_DP_VALIDATE_FAIL_RANK) pins the key to eager mode on BOTH
    ranks; with no mismatch both keep their graph."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_validate_rank, args=(r, port, fail_rank, q))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert [p.exitcode for p in ps] == [0, 0]
    for rank, vals, pinned, replays in res:
        if fail_rank is None:
            assert vals == [True] and not pinned and replays == 1
        else:
            assert vals == [False] and pinned and replays == 0


def test_capture_validator_compares_updates_per_tensor():
    """A wrong update of one small tensor is caught although the weights
    themselves differ by ~1e-4 of their size (the comparison is on the
    updates, tensor by tensor)."""
    from veles_amd.models.params import CaptureValidator

    class P(object):
        def __init__(self, name, offset, size):
            self.owner, self.name = None, name
            self.offset, self.size = offset, size

    class Store(object):
        dp = None
        params = [P("big", 0, 1000), P("small", 1000, 10)]
    v = CaptureValidator(Store())
    before = torch.ones(1010)
    upd = torch.randn(1010) * 1e-4
    ref = before + upd
    assert v.compare({"master": before}, ref.clone(), ref)
    got = ref.clone()
    got[1000:] = before[1000:] - upd[1000:]    # the small tensor's sign flipped
    assert not v.compare({"master": before}, got, ref)
    noisy = ref + torch.randn(1010) * 1e-9       # f32-atomic noise level
    assert v.compare({"master": before}, noisy, ref)
