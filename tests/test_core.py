"""Core runtime semantics: gates, links,
initialization order/retry, demand checks, Bool algebra, LinkableAttribute,
config tree, pickling, registry misprint detection, thread pool."""
import pickle

import pytest

from veles_amd.dummy import DummyWorkflow, DummyUnit
from veles_amd.mutable import Bool, link
from veles_amd.plumbing import Repeater
from veles_amd.units import (NotInitializedError, TrivialUnit, Unit)
from veles_amd.unit_registry import damerau_levenshtein
from veles_amd.utils.config import Config, get, root
from veles_amd.thread_pool import ThreadPool


class Recorder(Unit):
    def __init__(self, wf, **kw):
        super().__init__(wf, **kw)
        self.log = kw.get("log")

    def initialize(self, **kw):
        pass

    def run(self):
        self.log.append(self.name)


def chain(wf, names, log):
    units = [Recorder(wf, name=n, log=log) for n in names]
    return units


def test_gate_requires_all_parents():
    wf = DummyWorkflow()
    wf.end_point.unlink_all()
    log = []
    a, b, c = chain(wf, "abc", log)
    a.link_from(wf.start_point)
    b.link_from(wf.start_point)
    c.link_from(a, b)
    wf.end_point.link_from(c)
    wf.initialize()
    wf.run()
    assert log == ["a", "b", "c"]
    assert wf.finished


def test_gate_block_and_skip():
    wf = DummyWorkflow()
    wf.end_point.unlink_all()
    log = []
    a, b = chain(wf, "ab", log)
    a.link_from(wf.start_point)
    b.link_from(a)
    wf.end_point.link_from(b)
    wf.initialize()
    a.gate_skip <<= True
    wf.run()
    assert log == ["b"]
    log.clear()
    a.gate_skip <<= False
    b.gate_block <<= True
    for u in wf:
        u.stopped = False
    wf.run()
    assert log == ["a"]
    assert not wf.finished or True


def test_ignore_gate_and_loop():
    wf = DummyWorkflow()
    wf.end_point.unlink_all()
    log = []
    rep = Repeater(wf)
    rep.link_from(wf.start_point)
    (a,) = chain(wf, "a", log)
    a.link_from(rep)
    rep.link_from(a)
    done = Bool(False)
    a.run = a.run  # instance wrapper kept

    class Stop(Unit):
        def initialize(self, **kw):
            self.n = 0

        def run(self):
            self.n += 1
            done.__ilshift__(self.n >= 50)

    s = Stop(wf)
    s.link_from(a)
    rep.unlink_from(a)
    rep.link_from(s)
    wf.end_point.link_from(s)
    rep.gate_block = done
    wf.end_point.gate_block = ~done
    wf.initialize()
    wf.run()
    assert len(log) == 50 and wf.finished


def test_successors_sorted_by_name():
    wf = DummyWorkflow()
    wf.end_point.unlink_all()
    log = []
    z, y, x = chain(wf, "zyx", log)
    for u in (z, y, x):
        u.link_from(wf.start_point)
    wf.initialize()
    wf.run()
    assert log == ["x", "y", "z"]


def test_run_before_initialize_raises():
    u = TrivialUnit(DummyWorkflow())
    with pytest.raises(NotInitializedError):
        u.run()


def test_demand_checked_at_initialize():
    class Needy(TrivialUnit):
        def __init__(self, wf, **kw):
            super().__init__(wf, **kw)
            self.demand("data")

    u = Needy(DummyWorkflow())
    with pytest.raises(AttributeError):
        u.initialize()
    u.data = 5
    u.initialize()
    assert u.is_initialized


def test_initialize_retry():
    calls = []

    class Retry(TrivialUnit):
        def initialize(self, **kw):
            calls.append(1)
            return len(calls) < 3

    wf = DummyWorkflow()
    r = Retry(wf)
    r.link_from(wf.start_point)
    wf.initialize()
    assert len(calls) == 3 and r.is_initialized


def test_bool_algebra_and_callbacks():
    a, b = Bool(False), Bool(True)
    c = a | b
    d = a & b
    e = ~a
    f = a ^ b
    assert bool(c) and not bool(d) and bool(e) and bool(f)
    fired = []
    d.on_true = lambda x: fired.append("d")
    a <<= True
    assert bool(d) and not bool(e) and not bool(f)
    assert fired == ["d"]
    with pytest.raises(RuntimeError):
        c <<= False
    g = pickle.loads(pickle.dumps(c))
    assert bool(g)


def test_linkable_attribute_one_and_two_way():
    s = DummyUnit(x=1, y=2)
    t = DummyUnit()
    t.link_attrs(s, "x", ("z", "y"))
    assert t.x == 1 and t.z == 2
    s.x = 7
    assert t.x == 7
    with pytest.raises(RuntimeError):
        t.x = 3
    u = DummyUnit()
    u.link_attrs(s, "x", two_way=True)
    u.x = 42
    assert s.x == 42 and t.x == 42
    # mutable objects are shared by reference
    s.lst = [1]
    t.link_attrs(s, "lst")
    assert t.lst is s.lst


def test_link_function_and_pickle_roundtrip():
    a, b = DummyUnit(v=3), DummyUnit()
    link(b, "w", a, "v")
    assert b.w == 3
    wf = DummyWorkflow()
    u = TrivialUnit(wf, name="t1")
    u.link_from(wf.start_point)
    w2 = pickle.loads(pickle.dumps(wf))
    assert len(w2) == len(wf)
    assert w2["t1"].name == "t1"
    assert w2.restored_from_snapshot


def test_config_tree():
    c = Config("t")
    c.a.b.c = 5
    assert c.a.b.c == 5
    assert get(c.x.y, 9) == 9
    c.update({"p": {"q": 1}, "r": 2})
    assert c.p.q == 1 and c.r == 2
    c.protect("r")
    with pytest.raises(AttributeError):
        c.r = 3
    assert root.common.engine.dp.bucket_mb > 0


def test_misprint_distance():
    assert damerau_levenshtein("learnig_rate", "learning_rate") == 1
    assert damerau_levenshtein("ab", "ba") == 1


def test_thread_pool_pause_resume():
    p = ThreadPool(2, 4, name="t")
    out = []
    p.pause()
    for i in range(10):
        p.callInThread(out.append, i)
    import time
    time.sleep(0.05)
    assert out == []
    p.resume()
    assert p.wait_idle(5)
    assert sorted(out) == list(range(10))
    p.shutdown()
    p.shutdown()


def test_graph_dot_and_checksum():
    wf = DummyWorkflow()
    TrivialUnit(wf, name="mid").link_from(wf.start_point)
    dot, _ = wf.generate_graph(write_on_disk=False, with_data_links=True)
    assert dot.startswith("digraph Workflow") and "mid" in dot
    assert wf.checksum.endswith("_%d" % len(wf))
