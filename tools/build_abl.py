"""Diagnostic builds of libhvk.so with the T4 loop's ablation switches
(csrc/kernels/gemm_t4.h, HVK_T4_ABL: 1 no main-loop DMA, 2 no epilogue,
4 no main-loop waits / barriers, 8 main-loop DMA of cache-resident sources;
results are wrong by design).  Each build
lands in build/abl/libhvk_abl<N>.so and is selected at run time with
HVK_LIBRARY=<path> (veles_amd/ops/_lib.py), e.g. by
tools/bench_gemm_ab.py under ``gpu_job.sh benv:HVK_LIBRARY=...``.

    python tools/build_abl.py 1 2 4
    python tools/build_abl.py hc     # conv_hc.hip: build/hcabl/libhvk_hcabl.so
    python tools/build_abl.py halo 1 4   # wgrad_halo.hip: build/haloabl/"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                ".."))
from veles_amd.ops import build as B  # noqa: E402


def build_hc():
    """The conv_hc.hip ablation instantiations (-DHVK_HC_ABL, selected at
    run time by hvk_hc_ablation) in build/hcabl/libhvk_hcabl.so: the
    production library carries none of them."""
    B.FLAGS = list(B.FLAGS) + ["-DHVK_HC_ABL"]
    B.BUILD = os.path.join(B.REPO, "build", "hcabl", "obj")
    B.LIB = os.path.join(B.REPO, "build", "hcabl", "libhvk_hcabl.so")
    B.build(verbose=True)


def main(levels):
    base_flags = list(B.FLAGS)
    for n in levels:
        B.FLAGS = base_flags + ["-DHVK_T4_ABL=%d" % n]
        B.BUILD = os.path.join(B.REPO, "build", "abl", "obj%d" % n)
        B.LIB = os.path.join(B.REPO, "build", "abl", "libhvk_abl%d.so" % n)
        B.build(verbose=True)


def build_halo(levels):
    """The halo weight-gradient ablations (wgrad_halo.hip HVK_HALO_ABL: 1 no
    window DMA, 2 no epilogue stores, 4 no MFMAs): build/haloabl/
    libhvk_halo<N>.so each."""
    base_flags = list(B.FLAGS)
    for n in levels:
        B.FLAGS = base_flags + ["-DHVK_HALO_ABL=%d" % n]
        B.BUILD = os.path.join(B.REPO, "build", "haloabl", "obj%d" % n)
        B.LIB = os.path.join(B.REPO, "build", "haloabl",
                             "libhvk_halo%d.so" % n)
        B.build(verbose=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["hc"]:
        build_hc()
    elif sys.argv[1:2] == ["halo"]:
        build_halo([int(a) for a in sys.argv[2:]] or [1, 2, 4])
    else:
        main([int(a) for a in sys.argv[1:]] or [1, 2, 4])
