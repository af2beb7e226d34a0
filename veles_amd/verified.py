"""Interface verification for units (reference veles/verified.py:45-66 and
zope_verify_fix.py, which call zope.interface's ``verifyObject`` /
``verifyClass``).

Interfaces here are plain classes whose methods raise
``NotImplementedError`` (``IUnit``, ``IDistributable``, ``ILoader``,
``IResultProvider``, ...), mixed into the implementations.  A class
implements an interface when

* it derives from it (zope's ``providedBy``),
* every public method of the interface is overridden by a class in the MRO
  other than the interface itself (a bare stub would raise at run time),
* each override accepts the interface's positional parameters: its own
  required parameters are among them, or it takes ``*args`` / ``**kwargs``,
* the attributes the interface lists in ``__attributes__`` exist on the
  object (``verify_object`` only).

``Unit.do_initialize`` verifies ``IUnit`` once per class unless the class
sets ``DISABLE_INTERFACE_VERIFICATION`` (as in the reference).
"""
from __future__ import annotations

import inspect

__all__ = ["verify_class", "verify_object", "Verified",
           "BrokenImplementation"]


class BrokenImplementation(NotImplementedError):
    pass


def _iface_methods(iface):
    out = {}
    for base in reversed(iface.__mro__):
        if base is object:
            continue
        for name, v in vars(base).items():
            if name.startswith("_") or not callable(v):
                continue
            out[name] = base
    return out


def _positional(fn):
    try:
        sig = inspect.signature(fn)
    except (TypeError, ValueError):
        return None
    return sig


def _compatible(impl, spec):
    si, ss = _positional(impl), _positional(spec)
    if si is None or ss is None:
        return True
    kinds = {p.kind for p in si.parameters.values()}
    if inspect.Parameter.VAR_POSITIONAL in kinds and \
            inspect.Parameter.VAR_KEYWORD in kinds:
        return True
    spec_names = set(ss.parameters)
    var_kw = inspect.Parameter.VAR_KEYWORD in kinds
    for p in si.parameters.values():
        if p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
            continue
        if p.default is p.empty and p.name not in spec_names:
            return False
    # the interface's explicit parameters must be accepted
    for p in ss.parameters.values():
        if p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD):
            continue
        if p.name not in si.parameters and not var_kw and \
                inspect.Parameter.VAR_POSITIONAL not in kinds:
            return False
    return True


def verify_class(iface, cls):
    if not (isinstance(cls, type) and issubclass(cls, iface)):
        raise BrokenImplementation("%s does not implement %s" %
                                   (cls.__name__, iface.__name__))
    for name, owner in _iface_methods(iface).items():
        impl_owner = next((k for k in cls.__mro__ if name in vars(k)), None)
        if impl_owner is None or impl_owner is owner or \
                (isinstance(impl_owner, type) and issubclass(iface,
                                                             impl_owner)):
            raise BrokenImplementation(
                "%s does not implement %s.%s" % (cls.__name__,
                                                 iface.__name__, name))
        if not _compatible(vars(impl_owner)[name], vars(owner)[name]):
            raise BrokenImplementation(
                "%s.%s has a signature incompatible with %s.%s" % (
                    cls.__name__, name, iface.__name__, name))
    return True


def verify_object(iface, obj):
    verify_class(iface, type(obj))
    for attr in getattr(iface, "__attributes__", ()):
        if not hasattr(obj, attr):
            raise BrokenImplementation("%r lacks attribute %s required by %s"
                                       % (obj, attr, iface.__name__))
    return True


class Verified(object):
    """Mixin: ``self.verify_interface(IFoo)`` (reference ``Verified``)."""

    DISABLE_INTERFACE_VERIFICATION = False
    _verified_classes = set()

    def verify_interface(self, iface):
        cls = type(self)
        if getattr(cls, "DISABLE_INTERFACE_VERIFICATION", False):
            return
        key = (cls, iface)
        if key in Verified._verified_classes:
            return
        verify_object(iface, self)
        Verified._verified_classes.add(key)
