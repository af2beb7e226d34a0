"""Command-line flags with reference semantics (veles/cmdline.py:158-230,
__main__.py:372-378 / 628-656, launcher.py:688-690, pickle2.py:66-111,
thread_pool.py:139-142): --dry-run stops BEFORE the named stage,
--visualize initialises without running, --debug-pickle names the
unpicklable attribute, --pdb-on-finish opens the debugger, -b daemonizes,
--manhole serves a console on SIGUSR2."""
import os
import pickle
import signal
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WF = '''
import os
from veles_amd.units import TrivialUnit
from veles_amd.workflow import Workflow

def mark(s):
    with open(os.environ["VT_LOG"], "a") as f:
        f.write(s + "\\n")

class Step(TrivialUnit):
    def run(self):
        mark("run")

class W(Workflow):
    def __init__(self, launcher, **kw):
        super().__init__(launcher, **kw)
        self.step = Step(self)
        self.step.link_from(self.start_point)
        self.end_point.link_from(self.step)
        mark("create")

    def initialize(self, **kw):
        mark("init")
        return super().initialize(**kw)

def run(load, main):
    load(W)
    main()
'''


@pytest.fixture
def wf_file(tmp_path, monkeypatch):
    p = tmp_path / "flagwf.py"
    p.write_text(WF)
    log = tmp_path / "marks.log"
    monkeypatch.setenv("VT_LOG", str(log))
    return str(p), log


def _marks(log):
    return log.read_text().split() if log.exists() else []


def _main(*argv):
    from veles_amd.__main__ import Main
    m = Main(list(argv))
    assert m.run() == 0
    return m


@pytest.mark.parametrize("stage,expect,stopped", [
    ("load", [], "load"), ("init", ["create"], "initialize"),
    ("exec", ["create", "init"], "run"),
    ("no", ["create", "init", "run"], None)])
def test_dry_run_stops_before_the_stage(wf_file, stage, expect, stopped):
    path, log = wf_file
    m = _main(path, "", "-a", "cpu", "--dry-run", stage)
    assert _marks(log) == expect
    assert m.stopped_before == stopped


def test_visualize_initializes_without_running(wf_file, tmp_path):
    path, log = wf_file
    dot = str(tmp_path / "g.dot")
    m = _main(path, "", "-a", "cpu", "--visualize", "--workflow-graph", dot)
    assert _marks(log) == ["create", "init"]
    assert dot in m.visualized and os.path.getsize(dot) > 0
    assert "digraph" in open(dot).read()


class _Holder(object):
    def __init__(self):
        self.ok = [1, 2]
        self.inner = {"deep": [3, lambda x: x]}


def test_debug_pickle_names_the_attribute():
    from veles_amd.utils import pickle2
    pickle2.setup_pickle_debug(interactive=False)
    try:
        with pytest.raises(pickle.PicklingError) as ei:
            pickle.dumps(_Holder())
        assert "obj.inner.deep.1" in str(ei.value)
        assert pickle.loads(pickle.dumps([1, 2])) == [1, 2]
    finally:
        pickle2.teardown_pickle_debug()
    with pytest.raises(Exception) as ei:
        pickle.dumps(_Holder())
    assert "obj.inner" not in str(ei.value)


def test_debug_pickle_flag_installs_it(wf_file, monkeypatch):
    from veles_amd.utils import pickle2
    path, _ = wf_file
    try:
        _main(path, "", "-a", "cpu", "--debug-pickle", "--dry-run", "load")
        assert pickle2._saved is not None
    finally:
        pickle2.teardown_pickle_debug()


def test_pdb_on_finish(wf_file, monkeypatch):
    import pdb
    path, log = wf_file
    calls = []
    monkeypatch.setattr(pdb, "set_trace", lambda *a, **k: calls.append(1))
    monkeypatch.setattr(sys.stdin, "isatty", lambda: True, raising=False)
    _main(path, "", "-a", "cpu", "--pdb-on-finish")
    assert _marks(log) == ["create", "init", "run"] and calls == [1]


def test_background_daemonizes(wf_file, tmp_path):
    path, log = wf_file
    out = tmp_path / "daemon.log"
    env = dict(os.environ, PYTHONPATH=REPO)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "veles_amd", path, "", "-a",
                        "cpu", "-b", "-f", str(out)], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # the foreground process returned; the daemon finishes the run
    for _ in range(240):
        if "run" in _marks(log):
            break
        time.sleep(0.5)
    assert _marks(log) == ["create", "init", "run"], (
        _marks(log), out.read_text() if out.exists() else "")
    assert time.time() - t0 < 150


def test_manhole_serves_a_console_on_sigusr2(tmp_path):
    from veles_amd.dummy import DummyWorkflow
    from veles_amd.interaction import install_manhole
    wf = DummyWorkflow()
    path = str(tmp_path / "mh.sock")
    old = signal.getsignal(signal.SIGUSR2)
    try:
        assert install_manhole(wf, path) == path
        os.kill(os.getpid(), signal.SIGUSR2)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        for _ in range(100):
            try:
                s.connect(path)
                break
            except OSError:
                time.sleep(0.05)
        # owner-only socket whatever the umask
        assert os.stat(path).st_mode & 0o077 == 0
        f = s.makefile("rw")
        assert f.read(4) == ">>> "
        f.write("print(len(units) >= 2, type(workflow).__name__)\n")
        f.flush()
        line = f.readline()
        assert "True DummyWorkflow" in line
        s.close()
    finally:
        signal.signal(signal.SIGUSR2, old)


def test_manhole_flag(wf_file):
    path, _ = wf_file
    old = signal.getsignal(signal.SIGUSR2)
    try:
        m = _main(path, "", "-a", "cpu", "--manhole", "--dry-run", "exec")
        assert m.manhole_path.endswith("manhole.sock")
        # a private directory, not a predictable name in shared /tmp
        assert os.stat(os.path.dirname(m.manhole_path)).st_mode & 0o077 == 0
        assert signal.getsignal(signal.SIGUSR2) is not old
    finally:
        signal.signal(signal.SIGUSR2, old)
