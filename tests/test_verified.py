"""Interface verification (reference veles/verified.py, zope verifyObject
/ verifyClass)."""
import pytest

from veles_amd.dummy import DummyWorkflow
from veles_amd.units import IUnit, Unit
from veles_amd.verified import (BrokenImplementation, verify_class,
                                verify_object)


class IThing(object):
    __attributes__ = ("size",)

    def go(self, a, b=1):
        raise NotImplementedError


class Good(IThing):
    size = 3

    def go(self, a, b=1, *args, **kwargs):
        return a


class Missing(IThing):
    size = 1


class BadSig(IThing):
    size = 1

    def go(self, x, y, z):
        return x


class NoAttr(IThing):
    def go(self, a, b=2):
        return a


def test_verify_class_and_object():
    assert verify_class(IThing, Good)
    assert verify_object(IThing, Good())
    with pytest.raises(BrokenImplementation):
        verify_class(IThing, Missing)
    with pytest.raises(BrokenImplementation):
        verify_class(IThing, BadSig)
    with pytest.raises(BrokenImplementation):
        verify_object(IThing, NoAttr())
    with pytest.raises(BrokenImplementation):
        verify_class(IThing, object)


def test_units_are_verified_on_initialize():
    class NoRun(Unit):  # run() needs an argument nobody passes
        def initialize(self, **kwargs):
            pass

        def run(self, minibatch):
            pass

    class Fine(Unit):
        def initialize(self, **kwargs):
            pass

        def run(self):
            pass

    wf = DummyWorkflow()
    Fine(wf).do_initialize()
    with pytest.raises(BrokenImplementation):
        NoRun(wf).do_initialize()

    class Opted(NoRun):
        DISABLE_INTERFACE_VERIFICATION = True
    Opted(wf).do_initialize()


def test_every_registered_unit_implements_iunit():
    import veles_amd
    bad = []
    for cls in veles_amd.__units__:
        if getattr(cls, "hide_from_registry", False) or \
                getattr(cls, "DISABLE_INTERFACE_VERIFICATION", False):
            continue
        try:
            verify_class(IUnit, cls)
        except BrokenImplementation as e:
            bad.append(str(e))
    assert not bad, bad
