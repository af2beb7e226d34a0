"""Build an A/B copy of libhvk.so with ONE kernel source taken from another
git revision (the other objects as built now), for HVK_LIBRARY runs:

    python tools/build_ab_lib.py pool_lrn HEAD~3 abl/libhvk_lrn_old.so

Extra HVK_API symbols the working tree binds but the old source lacks get
no-op stubs (``--stub name`` ...), e.g. a newer A/B selector."""
import argparse
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))
from veles_amd.ops import build as b  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel", help="csrc/kernels/<kernel>.hip")
    ap.add_argument("rev", help="git revision of the old source")
    ap.add_argument("out", help="output .so")
    ap.add_argument("--stub", action="append", default=[],
                    help="void hvk_...(int) symbol to stub")
    a = ap.parse_args()
    b.build(verbose=False)
    tmp = tempfile.mkdtemp()
    src = os.path.join(tmp, a.kernel + ".hip")
    with open(src, "w") as f:
        f.write(subprocess.check_output(
            ["git", "show", "%s:csrc/kernels/%s.hip" % (a.rev, a.kernel)],
            cwd=b.REPO, text=True))
    old_obj = os.path.join(tmp, a.kernel + ".o")
    subprocess.check_call([b.HIPCC] + b.FLAGS + ["-I", b.KDIR, "-c", src,
                                                 "-o", old_obj])
    objs = []
    for s in sorted(os.listdir(b.KDIR)):
        if not s.endswith(".hip"):
            continue
        name = s[:-4]
        if name == a.kernel:
            objs.append(old_obj)
        else:
            objs.append(os.path.join(b.BUILD, "%s-%s.o" % (
                name, b._hash(os.path.join(b.KDIR, s), b.FLAGS))))
    if a.stub:
        stub = os.path.join(tmp, "stub.cpp")
        with open(stub, "w") as f:
            for n in a.stub:
                f.write('extern "C" __attribute__((visibility("default"))) '
                        'void %s(int) {}\n' % n)
        subprocess.check_call(["g++", "-O2", "-fPIC", "-c", stub, "-o",
                               stub + ".o"])
        objs.append(stub + ".o")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    subprocess.check_call([b.HIPCC, "-shared", "-fPIC",
                           "--offload-arch=" + b.ARCH, "-o", a.out] + objs)
    print("built", a.out)


if __name__ == "__main__":
    main()
