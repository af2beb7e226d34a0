"""Scratch buffers and process-group state that concurrent fan-out branches
or later workflows must not share:

* ``ops._workspace`` keys carry the branch stream while a branch runs
  (units._Branches), so two branches doing split-K GEMMs / dgrads of the
  same shape get separate workspaces;
* ``_Branches.join_all`` makes the current stream wait on every branch
  stream forked since the last call (dead-end branches included) and is
  called when the outermost scheduler drain ends;
* ``DataParallel.shutdown`` drops itself from the fp8 registries."""
import torch

from veles_amd import ops
from veles_amd.units import _Branches, _Scheduler


class _FakeStream(object):
    def __init__(self, sid):
        self.cuda_stream = sid
        self.waited = []


def test_workspace_per_branch():
    a = ops._workspace(("t_ws", 16), (16,), torch.float32,
                       torch.device("cpu"))
    s1, s2 = _FakeStream(1), _FakeStream(2)
    try:
        _Branches._tls.br = (s1, None, None)
        b1 = ops._workspace(("t_ws", 16), (16,), torch.float32,
                            torch.device("cpu"))
        _Branches._tls.br = (s2, None, None)
        b2 = ops._workspace(("t_ws", 16), (16,), torch.float32,
                            torch.device("cpu"))
        _Branches._tls.br = (s1, None, None)
        b1b = ops._workspace(("t_ws", 16), (16,), torch.float32,
                             torch.device("cpu"))
    finally:
        _Branches._tls.br = None
    assert b1 is b1b
    assert len({id(a), id(b1), id(b2)}) == 3
    assert ops._workspace(("t_ws", 16), (16,), torch.float32,
                          torch.device("cpu")) is a


def test_join_all_waits_on_every_forked_stream(monkeypatch):
    class Cur(object):
        cuda_stream = 0
        waited = []

        def wait_stream(self, st):
            self.waited.append(st.cuda_stream)
    cur = Cur()
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a: cur)
    f = _Branches._forked()
    f.clear()
    # two branches of a fork; one joins at a multi-parent unit, the other
    # is a dead end - both are waited for once the outermost drain ends
    f[1] = _FakeStream(11)
    f[2] = _FakeStream(12)
    with _Scheduler():
        with _Scheduler():
            pass
        assert cur.waited == []      # an inner drain does not join
    assert sorted(cur.waited) == [11, 12]
    assert not _Branches._forked()
    _Branches.join_all()             # nothing forked since: no waits
    assert sorted(cur.waited) == [11, 12]


def test_fp8_registry_forgets_dp():
    from veles_amd.ops import fp8
    r = fp8.registry("cpu")

    class DP(object):
        multi = True
    dp = DP()
    r.dp = dp
    fp8.release_dp(dp)
    assert r.dp is None
