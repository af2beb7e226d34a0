"""ctypes binding of the in-tree HIP kernel library ``libhvk.so``.

The kernels take raw device pointers and the current HIP stream, so they are
stream-ordered with PyTorch's own work and capture into HIP graphs.  On a GPU
box the library is REQUIRED: ``require_library()`` raises instead of silently
falling back to PyTorch (the CPU path is only the numerics reference).
"""
from __future__ import annotations

import ctypes
import os
import threading

from veles_amd.error import KernelLibraryMissing

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HVK_LIBRARY", os.path.join(_HERE, "libhvk.so"))

_lib = None
_lock = threading.Lock()

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double
U = ctypes.c_uint

_SIGS = {
    "hvk_gemm": [I, I, I, I, I, P, I, P, I, P, I, I, I, F, F, P, I, I, P, I, I,
                 I, P, P],
    "hvk_gemm_splitk": [I, I, I, I, I, P, I, P, I, P, I, I, F, P, I, P, I, I,
                        I, P, I, P],
    "hvk_conv_fwd": [P, P, P, P] + [I] * 15 + [P],
    "hvk_conv_dgrad_t": [P, P, P] + [I] * 14 + [P, I, P],
    # (X, Wt, bias, Y, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, act, s)
    "hvk_conv_fwd_halo": [P, P, P, P] + [I] * 13 + [P],
    "hvk_conv_fwd_halo_q8": [P, P, P, P] + [I] * 13 + [P, P, P, F, I, I, P],
    "hvk_conv_fwd_q8": [P, P, P, P] + [I] * 15 + [P, P, P, F, I, I, P],
    # (dY, Wt, dX, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, aux,
    #  aux_act, s)
    "hvk_conv_dgrad_halo": [P, P, P] + [I] * 12 + [P, I, P],
    "hvk_conv_wgrad": [P, P, P] + [I] * 15 + [P, P],
    "hvk_conv_fwd_run": [P, P, P, P] + [I] * 14 + [P],
    "hvk_conv_fwd_direct": [P, P, P, P] + [I] * 14 + [P],
    "hvk_conv_wgrad_run": [P, P, P, P] + [I] * 14 + [P],
    "hvk_im2col": [P, P] + [I] * 13 + [P],
    "hvk_fill_minibatch": [P, I, P, I, I, I, L, P, P, P, I, P, P, P, P],
    "hvk_fill_minibatch_s2d": [P, L, P, I, I, I, I, I, I, I, I, I, I, I, P,
                               P, P, P, P, P, P],
    "hvk_image_batch": [P, L, I, I, I, P, P, I, I, I, I, P, P, P, P, P, P],
    "hvk_mean_disp_normalize": [P, I, P, P, P, I, L, L, P],
    "hvk_softmax_ce": [P, I, I, I, P, F, P, I, P, P, P, P, P],
    "hvk_mse": [P, I, P, I, I, I, F, P, I, P, P, I, P],
    "hvk_sgd": [P, P, P, P, P, I, L, F, P],
    "hvk_sgd4": [P, P, P, P, P, I, L, F, L, P],
    "hvk_sgd4_grid": [P, P, P, P, P, I, L, F, L, I, P],
    "hvk_col_sum": [P, I, I, I, P, F, P],
    "hvk_row_sum": [P, I, I, I, P, F, P],
    "hvk_act_fwd": [P, I, P, I, L, I, P],
    "hvk_act_bwd": [P, I, P, I, P, I, L, I, P],
    "hvk_dropout": [P, I, P, I, L, U, F, P, P],
    "hvk_dropout_dev": [P, I, P, I, L, P, F, P, P],
    "hvk_dropout_dev_at": [P, I, P, I, L, P, F, L, P],
    "hvk_seed_advance": [P, P],
    "hvk_trace_marker": [I, P],
    "hvk_xact": [P, I, P, I, P, I, L, I, F, L, I, P],
    "hvk_gather": [P, I, P, P, I, L, P],
    "hvk_xorshift1024star": [P, I, I, P, P],
    "hvk_xorshift128plus": [P, I, P, P],
    "hvk_u64_to_uniform": [P, P, L, F, F, P],
    "hvk_join": [P, P, I, I, P, I, P],
    "hvk_cast": [P, I, P, I, L, F, P],
    "hvk_solver": [P, P, P, P, P, P, I, L, F, L, P],
    "hvk_space_to_depth": [P, P] + [I] * 9 + [P],
    "hvk_s2d_weights": [P, P] + [I] * 5 + [P],
    "hvk_s2d_grad_fold": [P, P] + [I] * 6 + [P],
    "hvk_pool_fwd": [P, P, P] + [I] * 13 + [P],
    "hvk_pool_bwd": [P, P, P] + [I] * 13 + [P, I, P],
    "hvk_lrn_fwd": [P, P, L, I, I, F, F, F, P],
    "hvk_lrn_bwd": [P, P, P, L, I, I, F, F, F, P, I, P],
    "hvk_lrn_pool_fwd": [P, P, P] + [I] * 9 + [F, F, F, P],
    "hvk_lrn_pool_bwd": [P, P, P, P] + [I] * 9 + [F, F, F, P, I, P],
    "hvk_pool2_fwd": [P, P] + [I] * 5 + [P],
    # + (q8, q8_st, q8_shard, q8_fmax, q8_fmt, hist): fused fp8 copy
    "hvk_pool2_fwd_q8": [P, P] + [I] * 5 + [P, P, P, F, I, I, P],
    "hvk_stochastic_pool": [P, P, P] + [I] * 12 + [P, P],
    "hvk_pool2_bwd": [P, P, P] + [I] * 5 + [P, I, P],
    "hvk_pool2_bwd_q8": [P, P, P] + [I] * 5 + [P, I, P, P, P, F, I, I, P],
    "hvk_lrn_pool_fwd_u8": [P, P, P] + [I] * 7 + [F, F, F, P],
    "hvk_lrn_pool_bwd_u8": [P, P, P, P] + [I] * 7 + [F, F, F, P, I, P],
    # exact-precision GEMMs (csrc/kernels/gemm_f32.hip)
    "hvk_gemm_f32": [I, I, I, I, I, P, I, P, I, P, I, F, F, I, P],
    "hvk_gemm_f64": [I, I, I, I, I, P, I, P, I, P, I, D, D, I, P],
    # fp8 (csrc/kernels/gemm_fp8.hip)
    "hvk_fp8_quant": [P, I, L, P, I, P, I, F, I, P],
    "hvk_fp8_amax": [P, I, L, P, I, P],
    "hvk_fp8_roll": [P, I, I, I, I, P, P],
    "hvk_fp8_roll_dev": [P, I, I, P, P, P],
    "hvk_gemm_fp8": [I, I, I, P, I, I, P, I, I, P, I, P, I, P, I, I, P, P, I,
                     F, F, P],
    "hvk_conv_fwd_fp8": [P, P, P, P] + [I] * 17 + [P, P, I, F, F,
                                                  P, P, P, F, I, P],
    "hvk_conv_dgrad_fp8": [P, P, P] + [I] * 14 + [P, I, I, I, P, P, I, F, F,
                           P, P, P, F, I, P],
    "hvk_conv_wgrad_fp8": [P, P, P, P] + [I] * 17 + [P, P, I, F, F, P],
    # halo weight gradient (csrc/kernels/wgrad_halo.hip): (X, dY, dW,
    # dbias, ws, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, splits, s)
    "hvk_conv_wgrad_halo": [P, P, P, P, P] + [I] * 13 + [P],
    "hvk_conv_wgrad_halo_splits": [I] * 13,
    "hvk_conv_wgrad_halo_fp8": [P, P, P, P, P] + [I] * 15 + [P, P, I, F, F,
                                                            P],
    # channel-chunked halo convs (csrc/kernels/conv_hc.hip)
    "hvk_conv_fwd_hc": [P, P, P, P] + [I] * 13 + [P, P],
    "hvk_conv_dgrad_hc": [P, P, P] + [I] * 12 + [P, I, P, P],
    "hvk_conv_dgrad_hc_w": [P, P, P] + [I] * 12 + [P, I, P, P],
    "hvk_conv_hc_wpack_bytes": [I] * 14,
    "hvk_hc_variant": [I],
    "hvk_hc_pitch_pad": [I],
    "hvk_hc32": [I],
    "hvk_halo_pitch_pad": [I],
    "hvk_hc32_ts": [I],
    # out = in^T and the column sums of in (csrc/kernels/elementwise.hip)
    "hvk_transpose_colsum": [P, I, I, P, P, I, P, P],
    "hvk_hc_last_variant": [],
    "hvk_set_pool_bwd_variant": [I],
    "hvk_hc_ablation": [I],
    "hvk_take_last_error": [],
    "hvk_end_stream_capture": [P],
    "hvk_stream_create": [],
}
_OPTIONAL = {}
# functions returning a pointer / a 64-bit int (every other one returns int)
_PTR_RET = {"hvk_stream_create"}
_LL_RET = {"hvk_conv_wgrad_halo", "hvk_conv_wgrad_halo_fp8",
           "hvk_conv_hc_wpack_bytes"}


def _load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            return None
        lib = ctypes.CDLL(LIB_PATH)
        for name, sig in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise KernelLibraryMissing("%s lacks %s - rebuild with python "
                                           "-m veles_amd.ops.build" %
                                           (LIB_PATH, name))
            fn.argtypes = sig
            fn.restype = ctypes.c_void_p if name in _PTR_RET else \
                ctypes.c_longlong if name in _LL_RET else ctypes.c_int
        # A/B schedule selectors for whole-run experiments (bench.py under
        # an environment setting; tests and tools call the setters directly)
        for env, fn in (("VELES_AMD_GEMM_VARIANT", "hvk_set_gemm_variant"),
                        ("VELES_AMD_FP8_VARIANT", "hvk_set_fp8_variant")):
            v = os.environ.get(env)
            if v is not None and hasattr(lib, fn):
                getattr(lib, fn)(ctypes.c_int(int(v)))
        _lib = lib
        return lib


def available():
    return _load() is not None


def require_library():
    lib = _load()
    if lib is None:
        raise KernelLibraryMissing(
            "HIP kernel library %s is missing; build it with `python -m "
            "veles_amd.ops.build` (gfx950)" % LIB_PATH)
    return lib


def lib():
    return require_library()


def check(rc, name):
    if rc != 0:
        raise RuntimeError("%s failed with HIP error %d%s" % (
            name, rc, _capture_context() if 900 <= rc < 910 else ""))


def _capture_context():
    """stream-capture errors: which stream the launch went to and whether
    a capture is in progress on it (diagnostics for the error message)"""
    try:
        import torch
        from veles_amd import graphs
        st = torch.cuda.current_stream()
        side = graphs._HipCapture._stream
        return (" (current stream %#x%s, capturing %s, open graph segment %s,"
                " capture side stream %s)" % (
                    st.cuda_stream,
                    " = default" if st == torch.cuda.default_stream() else "",
                    torch.cuda.is_current_stream_capturing(),
                    getattr(graphs._open_segment, "name", None),
                    None if side is None else "%#x" % side.cuda_stream))
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return " (%s)" % e
