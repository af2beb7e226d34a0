"""Mutable composable booleans (gates) and live attribute links.

Behavioural spec (reference: veles/mutable.py:44-216 ``Bool``, :219-350
``LinkableAttribute``, :353-357 ``link``):

* ``Bool``: ``a <<= x`` assigns (x: bool, Bool or a zero-arg callable);
  ``~a``, ``a | b``, ``a & b``, ``a ^ b`` build LIVE derived expressions which
  cannot be assigned to; ``on_true`` / ``on_false`` callbacks fire when an
  assignment changes what an expression evaluates to.
* Derived expressions are stored as data (operator name + operands), not as
  closures, so gates pickle with the workflow snapshot.
* ``LinkableAttribute``: ``b.x`` reads ``a.y`` live.  Assigning ``b.x`` raises
  unless the link is ``two_way`` (then it writes through to ``a.y``).
"""
from __future__ import annotations

import weakref

__all__ = ["Bool", "LinkableAttribute", "link", "unlink"]

_OPS = {
    "not": lambda vals: not vals[0],
    "or": lambda vals: vals[0] or vals[1],
    "and": lambda vals: vals[0] and vals[1],
    "xor": lambda vals: vals[0] != vals[1],
}


class Bool(object):
    """A mutable boolean value or a live boolean expression."""

    __slots__ = ("_value", "_op", "_args", "on_true", "on_false",
                 "_dependents", "_last", "__weakref__")

    def __init__(self, value=False):
        self._op = None
        self._args = ()
        self.on_true = None
        self.on_false = None
        self._dependents = weakref.WeakSet()
        if isinstance(value, Bool):
            # copy semantics: a new leaf holding the current value... unless
            # it is derived, in which case mirror the expression.
            if value._op is not None:
                self._op = value._op
                self._args = value._args
                for a in self._args:
                    a._dependents.add(self)
                self._value = None
            else:
                self._value = value._value
        else:
            self._check(value)
            self._value = value
        self._last = None

    @staticmethod
    def _check(value):
        if not (isinstance(value, bool) or callable(value)):
            raise TypeError("Value must be a boolean value or a function")

    @staticmethod
    def _derived(op, *args):
        b = Bool.__new__(Bool)
        b._value = None
        b._op = op
        b._args = tuple(args)
        b.on_true = None
        b.on_false = None
        b._dependents = weakref.WeakSet()
        b._last = None
        for a in args:
            a._dependents.add(b)
        return b

    @property
    def derived(self):
        return self._op is not None

    def __bool__(self):
        if self._op is not None:
            return bool(_OPS[self._op]([bool(a) for a in self._args]))
        v = self._value
        return bool(v()) if callable(v) else v

    def __int__(self):
        return int(bool(self))

    def __repr__(self):
        return repr(bool(self))

    __str__ = __repr__

    def __ilshift__(self, value):
        if self._op is not None:
            raise RuntimeError("Derived expressions cannot be assigned to.")
        if isinstance(value, Bool) or type(value).__module__ == "numpy":
            value = bool(value)
        self._check(value)
        self._value = value
        self.touch()
        return self

    def touch(self):
        """Fire callbacks on this node and on every expression built on it."""
        seen = set()
        stack = [self]
        while stack:
            node = stack.pop()
            if id(node) in seen:
                continue
            seen.add(id(node))
            v = bool(node)
            cb = node.on_true if v else node.on_false
            if cb is not None:
                cb(node)
            stack.extend(list(node._dependents))

    @staticmethod
    def _wrap(value):
        if isinstance(value, Bool):
            return value
        if isinstance(value, bool):
            return Bool(value)
        raise TypeError("Bool operations require Bool or bool operands")

    def __invert__(self):
        return Bool._derived("not", self)

    def __or__(self, other):
        return Bool._derived("or", self, Bool._wrap(other))

    __ror__ = __or__

    def __and__(self, other):
        return Bool._derived("and", self, Bool._wrap(other))

    __rand__ = __and__

    def __xor__(self, other):
        return Bool._derived("xor", self, Bool._wrap(other))

    __rxor__ = __xor__

    def __call__(self, other):
        """``a(b)``: become a copy of b's current value (leaf)."""
        self <<= bool(other)
        return self

    # -- pickling: keep the expression graph, drop callbacks ---------------
    def __getstate__(self):
        value = self._value
        if callable(value):
            try:
                import pickle
                pickle.dumps(value)
            except Exception:
                value = bool(value())
        return {"v": value, "op": self._op, "args": self._args,
                "on_true": _picklable_or_none(self.on_true),
                "on_false": _picklable_or_none(self.on_false)}

    def __setstate__(self, state):
        self._value = state["v"]
        self._op = state["op"]
        self._args = tuple(state["args"])
        self.on_true = state.get("on_true")
        self.on_false = state.get("on_false")
        self._dependents = weakref.WeakSet()
        self._last = None
        for a in self._args:
            a._dependents.add(self)


def _picklable_or_none(fn):
    if fn is None:
        return None
    try:
        import pickle
        pickle.dumps(fn)
        return fn
    except Exception:
        return None


class LinkableAttribute(object):
    """Class-level data descriptor implementing per-instance attribute links.

    An instance that has a link for ``name`` stores the pointer
    ``(src_obj, src_attr, two_way, assignment_guard)`` under
    ``obj.__dict__["_lnk_" + name]``; instances without a link keep the plain
    value in ``obj.__dict__[name]``.
    """

    def __init__(self, name):
        self.name = name
        self.key = "_lnk_" + name

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        d = obj.__dict__
        ptr = d.get(self.key)
        if ptr is not None:
            return getattr(ptr[0], ptr[1])
        try:
            return d[self.name]
        except KeyError:
            raise AttributeError(self.name) from None

    def __set__(self, obj, value):
        d = obj.__dict__
        ptr = d.get(self.key)
        if ptr is not None:
            src, attr, two_way, guard = ptr
            if two_way:
                setattr(src, attr, value)
                return
            if guard:
                raise RuntimeError(
                    "Attempted to set the value of linked property '%s' in "
                    "object %s and two_way is switched off." % (self.name, obj))
            # unguarded: assignment breaks the link
            del d[self.key]
        d[self.name] = value

    def __delete__(self, obj):
        d = obj.__dict__
        if self.key in d:
            del d[self.key]
        elif self.name in d:
            del d[self.name]
        else:
            raise AttributeError(self.name)

    @staticmethod
    def install(obj, name):
        cls = type(obj)
        existing = cls.__dict__.get(name)
        if isinstance(existing, LinkableAttribute):
            return existing
        # a property/other descriptor defined on the class cannot be linked
        for klass in cls.__mro__:
            if name in klass.__dict__:
                attr = klass.__dict__[name]
                if isinstance(attr, LinkableAttribute):
                    return attr
                if hasattr(attr, "__get__") and not callable(attr):
                    raise TypeError(
                        "Cannot link %s.%s: it is a descriptor" %
                        (cls.__name__, name))
                break
        desc = LinkableAttribute(name)
        setattr(cls, name, desc)
        return desc


def link(obj_dst, name_dst, obj_src, name_src, two_way=False,
         assignment_guard=True):
    """Make ``obj_dst.name_dst`` read ``obj_src.name_src`` live."""
    if obj_dst is obj_src and name_dst == name_src:
        raise ValueError("Attempted to link an attribute to itself")
    desc = LinkableAttribute.install(obj_dst, name_dst)
    obj_dst.__dict__.pop(desc.name, None)
    obj_dst.__dict__[desc.key] = (obj_src, name_src, two_way,
                                  assignment_guard)


def unlink(obj, name):
    """Remove a link, keeping the current value as a plain attribute."""
    key = "_lnk_" + name
    ptr = obj.__dict__.get(key)
    if ptr is None:
        return
    value = getattr(ptr[0], ptr[1])
    del obj.__dict__[key]
    obj.__dict__[name] = value


def is_linked(obj, name):
    return ("_lnk_" + name) in obj.__dict__
