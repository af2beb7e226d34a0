"""Ablation of the channel-chunked halo conv kernels (conv_hc.hip): times the
diagnostic instantiations against the production kernel, interleaved in one
process.  They exist only in the -DHVK_HC_ABL build
(``python tools/build_abl.py hc``; run with
HVK_LIBRARY=build/hcabl/libhvk_hcabl.so).  conv_hc32 (configurations 21 /
22): 1 no DMA after the first stage, 2 the DMA at the first k-step, 4 no
MFMAs, 8 no stage-end DMA wait, 16 the DMA over every k-step, 32 no
epilogue stores, 64 no epilogue; conv_hc_kernel (configuration 5): its own
table.

    HVK_LIBRARY=build/hcabl/libhvk_hcabl.so \
        python tools/ablate_conv_hc.py [batch] [rounds] [ablations] [filter]"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
import veles_amd.ops as ops  # noqa: E402
from veles_amd.ops import _lib  # noqa: E402

sys.path.insert(0, "tools")
from bench_conv_hc_ab import case, timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lib = _lib.lib()
    ops.set_conv_hc(True, -1)
    cases = [("conv3_fwd v21", ("fwd", B, 13, 13, 256, 384, 3, 1, 1, 1)),
             ("conv4_fwd v22", ("fwd", B, 13, 13, 384, 384, 3, 1, 1, 2)),
             ("conv5_dgrad v22", ("dgrad", B, 13, 13, 384, 256, 3, 1, 1, 2)),
             ("conv1_fwd v22", ("fwd", B, 227, 227, 3, 96, 11, 4, 0, 1)),
             ("conv2_fwd v11", ("fwd", B, 27, 27, 96, 256, 5, 1, 2, 2)),
             ("conv2_dgrad v5", ("dgrad", B, 27, 27, 96, 256, 5, 1, 2, 2))]
    abls = [int(a) for a in sys.argv[3].split(",")] \
        if len(sys.argv) > 3 else [0, 1, 2, 4, 8, 16, 32, 9]
    if len(sys.argv) > 4:   # case-name filter (the bits differ per kernel)
        cases = [c for c in cases if sys.argv[4] in c[0]]
    try:
        for name, shp in cases:
            fl, fn = case(*shp)
            res = {a: [] for a in abls}
            for _ in range(rounds):
                for a in abls:
                    lib.hvk_hc_ablation(a)
                    res[a].append(timeit(fn) * 1e3)
            med = {a: statistics.median(v) for a, v in res.items()}
            print("%-15s " % name + "  ".join(
                "abl%d %.3f ms (%.0f TF)" % (a, med[a], fl / med[a] / 1e9)
                for a in abls), flush=True)
            del fn
            torch.cuda.empty_cache()
    finally:
        lib.hvk_hc_ablation(0)
        ops.set_conv_hc(True, -2)


if __name__ == "__main__":
    main()
