"""The AlexNet loader gather with the conv1 space-to-depth transform
(hvk_fill_minibatch_s2d: uint8 227x227x3 -> normalised bf16 57x57x48) at
batch B: HIP-event time and HBM rate (also a rocprofv3 / PMC probe).

    python tools/probe_fill_s2d.py [batch] [reps] [variant ...]

Variants (hvk_set_gemm_variant): -1 the default (four images per block),
61 one image per block, 60 the per-chunk kernel; every variant's output is
checked bit-identical to the first's."""
import sys

import torch

sys.path.insert(0, ".")
from veles_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    n_img, H, W, C, s, K = 2 * B, 227, 227, 3, 4, 11
    g = torch.Generator(device="cuda").manual_seed(0)
    src = torch.randint(0, 256, (n_img, H, W, C), generator=g, device="cuda",
                        dtype=torch.uint8)
    shuffled = torch.randperm(n_img, device="cuda").to(torch.int32)
    mean = torch.rand(H * W * C) * 255
    disp = torch.rand(H * W * C) * 60 + 1
    pad = (0, 0, 0, 0)
    mean2 = ops.s2d_affine(mean, (H, W, C), s, K, K, pad, 0.0).cuda()
    rdisp2 = ops.s2d_affine(1.0 / disp, (H, W, C), s, K, K, pad, 1.0).cuda()
    H2, W2, C2 = ops.s2d_geometry(src.shape, s, K, K, pad)
    dst = torch.empty(B, H2, W2, C2, dtype=torch.bfloat16, device="cuda")
    f = lambda: ops.fill_minibatch_s2d(src, shuffled, 0, B, dst, s, K, K,  # noqa
                                       pad, mean2, rdisp2)
    variants = [int(v) for v in sys.argv[3:]] or [-1]
    lib = ops._lib.lib()
    ref = None
    for v in variants:
        lib.hvk_set_gemm_variant(v)
        # a long warmup: the first variant timed after 3 calls read ~8 %
        # slow (clocks still ramping), profiles/r6/fill_s2d_staging_r6ii.log
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        if ref is None:
            ref = dst.clone()
        same = torch.equal(dst, ref)
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        for _ in range(reps):
            f()
        b.record()
        b.synchronize()
        us = a.elapsed_time(b) / reps * 1e3
        mb = (B * H * W * C + dst.numel() * 2) / 1e6
        print("fill_s2d b%d variant %d: %.1f us, %.0f MB -> %.2f TB/s, "
              "bit-identical %s" % (B, v, us, mb, mb / us, same))
    lib.hvk_set_gemm_variant(-1)

if __name__ == "__main__":
    main()
