"""The ctypes signature table (veles_amd/ops/_lib.py) must match the C ABI
declared in csrc/kernels/*.hip (HVK_API functions): a wrong argument count
or kind only shows up on a GPU box otherwise."""
import glob
import os
import re

from veles_amd.ops import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _decls():
    """name -> (return type, argument declarations)"""
    out = {}
    for f in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")):
        src = open(f).read()
        for m in re.finditer(r"HVK_API\s+(int|void\s*\*|long\s+long|void)\s*"
                             r"(hvk_\w+)\s*"
                             r"\(([^)]*)\)", src):
            out[m.group(2)] = (m.group(1).replace(" ", ""),
                               [a.strip() for a in m.group(3).split(",")
                                if a.strip()])
    return out


def _kind(arg):
    a = re.sub(r"\s+", " ", arg)
    if "*" in a or a.startswith("hipStream_t"):
        return _lib.P
    if a.startswith(("long long", "int64_t", "size_t")):
        return _lib.L
    if a.startswith("float"):
        return _lib.F
    if a.startswith("double"):
        return _lib.D
    if a.startswith(("unsigned", "uint32_t")):
        return _lib.U
    return _lib.I


def test_every_binding_matches_its_declaration():
    decls = _decls()
    assert len(decls) >= 20
    for name, sig in _lib._SIGS.items():
        assert name in decls, "%s is bound but not declared" % name
        ret, args = decls[name]
        # a pointer result read back as a C int would be truncated
        assert (ret == "void*") == (name in _lib._PTR_RET), \
            "%s returns %s" % (name, ret)
        # a 64-bit result read back as a C int would be truncated too
        assert (ret == "longlong") == (name in _lib._LL_RET), \
            "%s returns %s" % (name, ret)
        want = [_kind(a) for a in args]
        assert len(sig) == len(want), "%s: %d args bound, %d declared" % (
            name, len(sig), len(want))
        for i, (got, exp) in enumerate(zip(sig, want)):
            # ints and unsigned ints are interchangeable at this ABI level
            if {got, exp} <= {_lib.I, _lib.U}:
                continue
            assert got == exp, "%s arg %d: %s vs %s (%s)" % (
                name, i, got, exp, args[i])
