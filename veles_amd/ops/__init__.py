"""Functional ops: hand-written HIP kernels on the GPU, PyTorch-fp32 references
on the CPU.

One code path for units: every op takes torch tensors; CUDA (HIP) tensors go
to ``libhvk.so`` (csrc/kernels, gfx950 MFMA / vectorised kernels) on the
current stream, CPU tensors are evaluated by the float32 reference below -
the numerics oracle of every kernel test (the reference's "numpy backend",
veles/backends.py:917-948).  There is no silent fallback: a GPU tensor with a
missing library raises ``KernelLibraryMissing``.

Layout conventions (docs/OPS.md): activations NHWC, conv weights
[OC][KH][KW][C/groups], fully-connected weights [out][in] (reference export
fixture libVeles/tests/workflow_files/contents.json), padding (left, top,
right, bottom), sliding (x, y).
"""
from __future__ import annotations

import os
import struct

import torch
import torch.nn.functional as F

from veles_amd.ops import _lib
from veles_amd.ops._lib import available, require_library  # noqa: F401

__all__ = ["ACT", "gemm", "linear_fwd", "conv_out_size", "conv_fwd",
           "conv_dgrad", "conv_wgrad", "col_sum", "row_sum", "act_fwd",
           "act_bwd", "pool_fwd", "pool_bwd", "lrn_fwd", "lrn_bwd",
           "softmax_ce", "mse", "sgd_update", "dropout", "xorshift1024star",
           "xorshift128plus", "join", "cast", "fill_minibatch",
           "mean_disp_normalize", "act_code"]

DT = {torch.float32: 0, torch.bfloat16: 1, torch.uint8: 2, torch.int32: 3,
      torch.float16: 4}
ACT = {"linear": 0, None: 0, "tanh": 1, "relu": 2, "strict_relu": 3,
       "str": 3, "sigmoid": 4}


def act_code(act):
    if isinstance(act, int):
        return act
    return ACT[act]


def _p(t):
    return None if t is None else t.data_ptr()


def _s(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _lib_call(name, *args):
    fn = getattr(_lib.lib(), name)
    _lib.check(fn(*args), name)


def _gpu(t):
    return t is not None and t.is_cuda


# The LDS-DMA loaders address an operand through 32-bit buffer offsets
# (csrc/kernels/conv_geom.h kBufMaxBytes); a larger operand drops the kernel
# to its per-lane-address loader (VGG-16 b512 conv1_2: 3.3 GB activations,
# forward 3.1 ms on that path).  Convolutions over larger batches therefore
# run in image chunks that keep every operand under the limit.
_BUF_MAX = (1 << 31) - 64


def _image_chunks(N, *tensors):
    """Equal image ranges [(n0, n1)] whose slices of ``tensors`` (leading
    dimension = images) each stay under ``_BUF_MAX`` bytes."""
    per = max([t.numel() // max(t.shape[0], 1) * t.element_size()
               for t in tensors if t is not None] + [1])
    if N * per < _BUF_MAX or N < 2:
        return [(0, N)]
    n = max(1, (_BUF_MAX - 1) // per)
    k = -(-N // n)
    step = -(-N // k)
    return [(i, min(N, i + step)) for i in range(0, N, step)]


# --------------------------------------------------------------- activations
def act_fwd_ref(x, act):
    act = act_code(act)
    if act == 1:
        return 1.7159 * torch.tanh(0.6666 * x)
    if act == 2:
        return torch.where(x > 15, x, torch.log1p(torch.exp(x.clamp(max=15))))
    if act == 3:
        return torch.clamp(x, min=0)
    if act == 4:
        return torch.sigmoid(x)
    return x


def act_bwd_ref(y, act):
    act = act_code(act)
    if act == 1:
        return 0.6666 * 1.7159 - (0.6666 / 1.7159) * y * y
    if act == 2:
        return 1 - torch.exp(-y)
    if act == 3:
        return (y > 0).to(y.dtype)
    if act == 4:
        return y * (1 - y)
    return torch.ones_like(y)


def act_fwd(x, act, out=None):
    act = act_code(act)
    if _gpu(x):
        out = torch.empty_like(x) if out is None else out
        _lib_call("hvk_act_fwd", _p(x), DT[x.dtype], _p(out), DT[out.dtype],
                  x.numel(), act, _s(x))
        return out
    r = act_fwd_ref(x.float(), act).to(x.dtype)
    if out is None:
        return r
    out.copy_(r)
    return out


XACT = {"log": 1, "tanhlog": 2, "sincos": 3, "mul": 4}


def xact_ref(x, kind, p=0.0, bwd=False, err=None):
    """float32 reference of hvk_xact: activations whose derivative is a
    function of the input x (log = asinh, tanhlog, sincos, mul)."""
    kind = XACT.get(kind, kind)
    x = x.float()
    if kind == 1:
        d = torch.rsqrt(x * x + 1) if bwd else torch.log(
            x + torch.sqrt(x * x + 1))
    elif kind == 2:
        a = x.abs()
        t = torch.tanh(torch.tensor(0.6666 * p))
        edge, slope = 1.7159 * t, 1.7159 * 0.6666 * (1 - t * t)
        th = torch.tanh(0.6666 * x)
        if bwd:
            d = torch.where(a <= p, 1.7159 * 0.6666 * (1 - th * th),
                            slope * p / a.clamp(min=p))
        else:
            d = torch.where(a <= p, 1.7159 * th, torch.sign(x) * (
                edge + slope * p * torch.log(a.clamp(min=p) / p)))
    elif kind == 3:
        flat = x.reshape(x.shape[0] if x.dim() > 1 else 1, -1)
        odd = (torch.arange(flat.shape[1], device=x.device) % 2 == 1)
        if bwd:
            d = torch.where(odd, -torch.sin(flat), torch.cos(flat))
        else:
            d = torch.where(odd, torch.cos(flat), torch.sin(flat))
        d = d.view(x.shape)
    elif kind == 4:
        d = torch.full_like(x, p) if bwd else x * p
    else:
        raise ValueError("unknown activation %r" % kind)
    return err.float() * d if bwd else d


def xact(x, kind, p=0.0, out=None, err=None):
    """y = f(x) (err None) or y = err * f'(x) for the input-derivative
    activations (``XACT``); ``hvk_xact`` on the GPU."""
    kind = XACT.get(kind, kind)
    bwd = err is not None
    if out is None:
        out = torch.empty_like(err if bwd else x)
    if _gpu(x):
        rowlen = x[0].numel() if x.dim() > 1 else x.numel()
        _lib_call("hvk_xact", _p(x), DT[x.dtype], _p(err),
                  DT[err.dtype] if bwd else 0, _p(out), DT[out.dtype],
                  x.numel(), int(kind), float(p), max(1, int(rowlen)),
                  int(bwd), _s(x))
        return out
    out.copy_(xact_ref(x, kind, p, bwd, err).to(out.dtype))
    return out


def gather(x, idx, out=None):
    """out[i] = x.flat[idx.flat[i]] (int32 indices; negative -> 0)."""
    if out is None:
        out = torch.empty(idx.shape, dtype=x.dtype, device=x.device)
    if _gpu(x):
        _lib_call("hvk_gather", _p(x), DT[x.dtype], _p(idx), _p(out),
                  DT[out.dtype], idx.numel(), _s(x))
        return out
    i = idx.reshape(-1).long()
    v = x.reshape(-1)[i.clamp(min=0)]
    v = torch.where(i >= 0, v, torch.zeros_like(v))
    out.copy_(v.view(out.shape))
    return out


def act_bwd(dy, y, act, out=None):
    """dx = dy * f'(y) (derivative expressed through the output y)."""
    act = act_code(act)
    if _gpu(dy):
        out = torch.empty_like(dy) if out is None else out
        _lib_call("hvk_act_bwd", _p(dy), DT[dy.dtype], _p(y), DT[y.dtype],
                  _p(out), DT[out.dtype], dy.numel(), act, _s(dy))
        return out
    r = (dy.float() * act_bwd_ref(y.float(), act)).to(dy.dtype)
    if out is None:
        return r
    out.copy_(r)
    return out


# --------------------------------------------------------------------- GEMM
def gemm(a, b, *, trans_a=False, trans_b=False, out=None, out_dtype=None,
         alpha=1.0, beta=0.0, bias=None, bias_mode="col", act=0, aux=None,
         aux_act=0, accumulate=False, splits=1, bias_grad=None,
         precision_level=None):
    """out[M][N] = act(alpha*op(a)@op(b) + beta*out + bias) * f'_aux(aux).

    ``accumulate``: out (float32) += alpha*op(a)@op(b) (+bias) - split-K
    partial sums are reduced with float atomics on the GPU.
    ``bias_grad`` (float32 [M], accumulate only): += alpha * row sums of
    op(a), computed by the same kernel (a ones column appended to op(b)).
    ``accumulate="overwrite"``: out (and bias_grad) := the product instead
    of +=, written without reading out - a weight gradient that is the
    step's only contribution (no zeroing pass needed before it).

    float32 / float64 GPU operands run the exact-precision MFMA SGEMM /
    DGEMM (csrc/kernels/gemm_f32.hip; alpha / beta / accumulate only) with
    the reference's ``precision_level`` 0 (plain), 1 (Kahan) or 2 (TwoSum
    multi-partial); default ``root.common.engine.precision_level``.
    """
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    if K != Kb:
        raise ValueError("gemm: inner dimensions differ (%d vs %d)" % (K, Kb))
    act = act_code(act)
    aux_act = act_code(aux_act)
    bm = {"col": 1, "row": 2}[bias_mode]
    dev = a.device
    if out is None:
        out_dtype = out_dtype or (torch.float32 if accumulate else a.dtype)
        out = (torch.zeros if accumulate else torch.empty)(
            M, N, dtype=out_dtype, device=dev)
    overwrite = accumulate == "overwrite"
    if _gpu(a) and a.dtype in (torch.float32, torch.float64):
        return _gemm_fx(a, b, trans_a, trans_b, out, M, N, K, alpha, beta,
                        accumulate and not overwrite, precision_level, bias,
                        act, aux, bias_grad)
    if _gpu(a):
        if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
            raise TypeError("GPU gemm operands must be bfloat16 (or float32 "
                            "/ float64 for the exact-precision GEMM)")
        for t in (a, b, out):
            if t.stride(-1) != 1:
                raise ValueError("gemm operands must be row-major")
        if accumulate and out.dtype != torch.float32:
            raise TypeError("accumulate requires a float32 output")
        res = out
        pad = None
        if not accumulate and beta == 0.0 and bias_grad is None:
            pad = _dma_padded(a, b, trans_a, trans_b, M, N, K, bias, aux,
                              bm)
        if pad is not None:
            # odd M / N / K: zero-padded operands take the LDS-DMA loaders
            a, b, Mp, Np, Kp = pad
            out = torch.empty(Mp, Np, dtype=out.dtype, device=dev)
            M, N, K = Mp, Np, Kp
        # rows off the 16-B grid would drop the whole GEMM to the per-element
        # loaders (3001^3: 76 vs ~800 TF): re-stride such operands first
        a, b = _row_aligned(a), _row_aligned(b)
        if not accumulate and beta == 0.0 and out.dim() == 2 and \
                (out.stride(0) % 8 or out.data_ptr() % 16):
            # and a write-only output into an aligned buffer (vector
            # epilogue stores), copied out after
            out = torch.empty(M, -(-N // 8) * 8, dtype=out.dtype,
                              device=dev)[:, :N]
        atomic = 2 if overwrite else (1 if accumulate else 0)
        if splits > 1 and not accumulate:
            raise ValueError("split-K requires accumulate=True")
        if deterministic():
            splits = 1
        elif accumulate and splits == 1:
            # a weight gradient with a handful of output tiles and a long K
            # (CIFAR quick fc2: 10 x 64 over a 4096 batch, ONE workgroup
            # for 0.27 ms): split K over f32 atomics; an overwrite is then a
            # zero fill + atomic accumulate
            sp = _wgrad_gemm_splits(M, N + (bias_grad is not None), K)
            if sp > 1:
                if overwrite:
                    out.zero_()
                    if bias_grad is not None:
                        bias_grad.zero_()
                atomic, splits = 1, sp
        if bias_grad is not None and (trans_b or not accumulate):
            raise ValueError("bias_grad needs accumulate=True, trans_b=False")
        sk = 0 if accumulate or beta != 0.0 else \
            _splitk_for(a, b, trans_a, trans_b, out, M, N, K, bias, aux)
        if sk > 1:
            # a persistent f32 workspace of sk slices per size: each K split
            # stores its partial product to its own slice, the finishing
            # pass sums them in order (no atomics, nothing to zero)
            ws = _workspace(("splitk_ws", M * N * sk), (M * N * sk,),
                            torch.float32, dev)
            _lib_call("hvk_gemm_splitk", int(trans_a), int(trans_b), M, N, K,
                      _p(a), a.stride(0), _p(b), b.stride(0), _p(out),
                      out.stride(0), int(out.dtype == torch.float32),
                      float(alpha), _p(bias), act, _p(aux),
                      0 if aux is None else aux.stride(0), aux_act, sk,
                      _p(ws), 1, _s(a))
        else:
            _lib_call("hvk_gemm", int(trans_a), int(trans_b), M, N, K, _p(a),
                      a.stride(0), _p(b), b.stride(0), _p(out),
                      out.stride(0), int(out.dtype == torch.float32), atomic,
                      float(alpha), float(beta), _p(bias), bm, act, _p(aux),
                      0 if aux is None else aux.stride(0), aux_act,
                      int(splits), _p(bias_grad), _s(a))
        if res is not out:
            res.copy_(out[:res.shape[0], :res.shape[1]])
        return res
    A = a.float().t() if trans_a else a.float()
    B = b.float().t() if trans_b else b.float()
    r = alpha * (A @ B)
    if bias is not None:
        r = r + (bias.float().view(1, -1) if bm == 1 else
                 bias.float().view(-1, 1))
    if overwrite:
        out.copy_(r.to(out.dtype))
        if bias_grad is not None:
            bias_grad.copy_(alpha * A.sum(1))
        return out
    if accumulate:
        out += r.to(out.dtype)
        if bias_grad is not None:
            bias_grad += alpha * A.sum(1)
        return out
    if beta != 0.0:
        r = r + beta * out.float()
    r = act_fwd_ref(r, act)
    if aux is not None:
        r = r * act_bwd_ref(aux.float(), aux_act)
    out.copy_(r.to(out.dtype))
    return out


_DMA_PAD_MIN = 1 << 24   # M*N*K above which padding pays for its copies

# Deterministic mode (engine.deterministic / VELES_AMD_DETERMINISTIC=1):
# no f32-atomic reductions in the gradient path - GEMM weight gradients
# and GEMM-path conv weight gradients unsplit (one tile sums its whole K),
# column sums through torch's fixed-order reduction; the halo weight
# gradient and the workspace split-K GEMM are deterministic already.
# Two runs of the same step are then bit-identical (exact-resume tests);
# it costs the split-K parallelism of small weight gradients.
_DETERMINISTIC = os.environ.get("VELES_AMD_DETERMINISTIC", "0") != "0"


def set_deterministic(on):
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)


def deterministic():
    from veles_amd.utils.config import root, get
    return _DETERMINISTIC or bool(get(root.common.engine.deterministic,
                                      False))


def _dma_padded(a, b, trans_a, trans_b, M, N, K, bias, aux, bias_mode=1):
    """Zero-padded copies of a large GEMM's operands when an odd dimension
    keeps them off the LDS-DMA loaders (a K-major operand needs K % 8 == 0,
    an MN-major one M / N % 8 == 0; csrc/kernels/gemm.hip ``dma_ok``): K
    pads with zeros (adds nothing), M / N pads are sliced off the output.
    None when nothing needs padding, the GEMM is small, or a bias / aux
    operand would have to be padded too."""
    r8 = lambda v: -(-v // 8) * 8  # noqa: E731
    ka, kb = not trans_a, bool(trans_b)
    Kp = r8(K) if (ka or kb) and K % 8 else K
    Mp = r8(M) if not ka and M % 8 else M
    Np = r8(N) if not kb and N % 8 else N
    if (Mp, Np, Kp) == (M, N, K) or M * N * K < _DMA_PAD_MIN:
        return None
    # a per-column (1) / per-row (2) bias would be read past its end
    if bias is not None and (Np != N if bias_mode == 1 else Mp != M):
        return None
    if aux is not None and (Mp, Np) != (M, N):
        return None

    def padded(t, rows, cols):
        if tuple(t.shape) == (rows, cols):
            return t
        z = torch.zeros(rows, cols, dtype=t.dtype, device=t.device)
        z[:t.shape[0], :t.shape[1]].copy_(t)
        return z
    a2 = padded(a, M, Kp) if ka else padded(a, Kp, Mp)
    b2 = padded(b, Np, Kp) if kb else padded(b, Kp, Np)
    return a2, b2, Mp, Np, Kp


def _row_aligned(t):
    """``t`` itself when its rows start on 16-B boundaries, else a copy in a
    buffer whose row pitch is padded to a multiple of 8 elements (the view
    keeps the logical shape; the LDS-DMA loaders never read the pad)."""
    if t.dim() != 2 or (t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0):
        return t
    R, C = t.shape
    buf = torch.empty(R, -(-C // 8) * 8, dtype=t.dtype, device=t.device)
    v = buf[:, :C]
    v.copy_(t)
    return v


_SPLITK_ENV = os.environ.get("HVK_SPLITK")


def _wgrad_gemm_splits(M, N, K):
    """K splits for an accumulating GEMM under 64 output tiles with K >= 2048
    (~256 workgroups, >= 256 of K each); 1 = leave it whole.  The large FC
    weight gradients (AlexNet fc6: 2304 tiles) keep their single-pass
    read-modify-write.  HVK_SPLITK=0 disables."""
    if _SPLITK_ENV == "0" or K < 2048:
        return 1
    tiles = -(-M // 128) * -(-N // 128)
    if tiles >= 64:
        return 1
    return max(1, min(-(-256 // tiles), K // 256))


def _splitk_aligned(N, out, bias, aux):
    """Operands hvk_gemm_splitk takes (16-B rows for the finishing pass)."""
    return not (N % 8 or out.stride(0) % 8 or out.data_ptr() % 16 or
                (bias is not None and bias.data_ptr() % 16) or
                (aux is not None and (aux.stride(0) % 8 or
                                      aux.data_ptr() % 16)))


def auto_splitk(M, N, K, out, bias=None, aux=None):
    """K splits for a GEMM whose 128 x 128 output tiles cannot fill the
    MI355X's 256 CUs twice over (the FC layers at batch 512): enough splits
    for ~512 workgroups, each keeping >= 1024 of K.  0 = no split (shape or
    alignment not taken by hvk_gemm_splitk).  HVK_SPLITK=0 disables."""
    if _SPLITK_ENV == "0":
        return 0
    tiles = -(-M // 128) * -(-N // 128)
    if tiles >= 256 or K < 2048 or not _splitk_aligned(N, out, bias, aux):
        return 0
    sk = min(-(-512 // tiles), K // 1024)
    return sk if sk > 1 else 0


# the autotuner's replay forces a split count (ops/autotune.py)
_splitk_forced = None


def _splitk_for(a, b, trans_a, trans_b, out, M, N, K, bias, aux):
    """auto_splitk, overridden per shape by the device tuning table."""
    if _splitk_forced is not None:
        return _splitk_forced if _splitk_aligned(N, out, bias, aux) else 0
    sk = auto_splitk(M, N, K, out, bias, aux)
    # the table may also split a GEMM with 256..511 tiles (one 128 x 128
    # tile per CU: AlexNet b1024 fc6 forward runs 2 splits 7 % faster,
    # profiles/splitk_sweep_fc_r3.log)
    if _SPLITK_ENV == "0" or -(-M // 128) * -(-N // 128) >= 512 or \
            K < 1024 or not _splitk_aligned(N, out, bias, aux):
        return sk
    from veles_amd.ops import autotune
    autotune.log_call("splitk", (M, N, K), {
        "a": tuple(a.shape), "b": tuple(b.shape), "out": tuple(out.shape),
        "trans_a": trans_a, "trans_b": trans_b, "default": sk})
    t = autotune.lookup("splitk", M, N, K)
    return sk if t is None else (t if t > 1 else 0)


def _precision_level(level):
    if level is not None:
        return int(level)
    from veles_amd.utils.config import root, get
    return int(get(root.common.engine.precision_level, 0))


def _gemm_fx(a, b, ta, tb, out, M, N, K, alpha, beta, accumulate, level,
             bias, act, aux, bias_grad):
    if bias is not None or act_code(act) or aux is not None or \
            bias_grad is not None:
        raise ValueError("the float32/float64 GEMM takes alpha/beta only")
    if b.dtype != a.dtype or out.dtype != a.dtype:
        raise TypeError("gemm: mixed %s / %s / %s operands" %
                        (a.dtype, b.dtype, out.dtype))
    for t in (a, b, out):
        if t.stride(-1) != 1:
            raise ValueError("gemm operands must be row-major")
    name = "hvk_gemm_f32" if a.dtype == torch.float32 else "hvk_gemm_f64"
    _lib_call(name, int(ta), int(tb), M, N, K, _p(a), a.stride(0), _p(b),
              b.stride(0), _p(out), out.stride(0), float(alpha),
              1.0 if accumulate else float(beta), _precision_level(level),
              _s(a))
    return out


def linear_fwd(x, w, bias=None, act=0, out=None):
    """y[B][out] = act(x[B][in] @ w[out][in]^T + bias)."""
    return gemm(x, w, trans_b=True, bias=bias, act=act, out=out)


# --------------------------------------------------------------- convolution
def conv_out_size(h, w, kh, kw, sliding, padding):
    sx, sy = sliding
    pl, pt, pr, pb = padding
    return (h + pt + pb - kh) // sy + 1, (w + pl + pr - kw) // sx + 1


def _nchw(x):
    return x.permute(0, 3, 1, 2).float()


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


_WS = {}


def _branch_key():
    """The branch stream's id while a fan-out branch runs (units._Branches):
    concurrent branches must not share scratch buffers."""
    from veles_amd.units import _Branches
    br = _Branches.current()
    return None if br is None else id(br[0])


def _workspace(key, shape, dtype, device, zero=False):
    bk = _branch_key()
    if bk is not None:
        key = (key, "branch", bk)
    t = _WS.get(key)
    if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype or \
            t.device != device:
        t = (torch.zeros if zero else torch.empty)(shape, dtype=dtype,
                                                   device=device)
        _WS[key] = t
    return t


_GROWN = {}
_RETIRED = []


def _grow_ws(name, n, dtype, device):
    """A scratch buffer of at least n elements shared by every call with this
    name (per device and fan-out branch), grown geometrically.  A buffer it
    outgrows stays allocated: a HIP graph captured earlier may still write
    into it on replay."""
    key = (name, str(device), dtype, _branch_key())
    t = _GROWN.get(key)
    if t is None or t.numel() < n:
        if t is not None:
            _RETIRED.append(t)
        size = max(n, 0 if t is None else t.numel() * 3 // 2)
        t = _GROWN[key] = torch.empty(size, dtype=dtype, device=device)
    return t[:n]


def needs_im2col(C, groups):
    """Small-channel convs (C/groups % 8 != 0, e.g. RGB input) run as an
    explicit bf16 im2col + dense MFMA GEMM instead of per-element gathers."""
    return groups == 1 and C % 8 != 0


# Small-channel (3 <= C < 8, e.g. RGB at stride 1) convs: zero-pad the
# channels to 8 and run the implicit-GEMM path instead of the packed
# (kw, c)-run kernels.  VGG-16 conv1_1 (b128, 224^2): weight gradient 0.82 ->
# 0.32 ms (+0.05 ms for the pad, shared with the forward), forward 1.41 ->
# 1.26 ms (tools/bench_c3_pad.py).  HVK_C3_PAD=0 keeps the run kernels.
_C_PAD8 = os.environ.get("HVK_C3_PAD", "1") != "0"
_DIRECT = os.environ.get("HVK_CONV_DIRECT", "1") != "0"
_C_PAD_MIN = int(os.environ.get("HVK_C3_PAD_MIN", "3"))


def pad8_ok(C, groups):
    """Channels padded to the next multiple of 8 (3 -> 8, LeNet's 20 -> 24)."""
    return _C_PAD8 and groups == 1 and C >= _C_PAD_MIN and C % 8 != 0


def _cpad(C):
    return -(-C // 8) * 8


class PaddedImage(object):
    """The channel-padded image of a small-channel conv input, kept by the
    forward pass for the weight-gradient GEMM."""

    def __init__(self, x, C):
        self.x = x
        self.C = C


def _pad_channels(x):
    """x [N,H,W,C] -> [N,H,W,Cp] (Cp = C rounded up to 8), the padding
    channels zero (a persistent buffer per input tensor: the pad stays zero,
    only x's channels are copied)."""
    N, H, W, C = x.shape
    buf = _workspace(("cpad8", x.data_ptr(), N, H, W, C),
                     (N, H, W, _cpad(C)), x.dtype, x.device, zero=True)
    buf[..., :C].copy_(x)
    return buf


def _pad_weights(w, key):
    OC, KH, KW, C = w.shape
    wp = _workspace((key, id(w)), (OC, KH, KW, _cpad(C)), w.dtype,
                    w.device, zero=True)
    wp[..., :C].copy_(w)
    return wp


class S2DImage(object):
    """The space-to-depth image of a strided small-channel conv input: kept
    by the forward pass for the weight-gradient GEMM, or served directly by
    the loader's fused gather (``fill_minibatch_s2d``) as the conv input.
    ``shape`` is the NHWC shape of the image it stands for."""
    __slots__ = ("x", "s", "shape")

    def __init__(self, x, s, shape=None):
        self.x = x
        self.s = s
        self.shape = tuple(shape) if shape is not None else None


_S2D = os.environ.get("HVK_S2D", "1") != "0"   # A/B knob


def s2d_factor(C, groups, sliding, KH, KW):
    """Stride s when a conv is better run as space-to-depth (C -> s*s*C
    channels, stride 1, ceil(K/s) taps): small C, equal strides, s*s*C a
    multiple of 8 (the aligned LDS-DMA loaders), kernel at least s wide."""
    sx, sy = sliding
    if groups != 1 or C % 8 == 0 or sx != sy or sx < 2 or not _S2D:
        return 0
    if (sx * sx * C) % 8 or KH < sx or KW < sx:
        return 0
    return sx


def _s2d_geometry(H, W, KH, KW, s, padding):
    OH, OW = conv_out_size(H, W, KH, KW, (s, s), padding)
    KH2, KW2 = -(-KH // s), -(-KW // s)
    return OH, OW, KH2, KW2, OH - 1 + KH2, OW - 1 + KW2


def s2d_geometry(shape, s, KH, KW, padding):
    """(H2, W2, C2) of the space-to-depth image of an NHWC ``shape``."""
    _, H, W, C = shape
    _, _, _, _, H2, W2 = _s2d_geometry(H, W, KH, KW, s, padding)
    return H2, W2, s * s * C


def space_to_depth_ref(x, s, KH, KW, padding):
    """Torch reference of hvk_space_to_depth: x [N,H,W,C] ->
    [N,H2,W2,s*s*C], y[n,Y,X,dy,dx,c] = x[n, s*Y+dy-pt, s*X+dx-pl, c] (0
    outside the image)."""
    N, H, W, C = x.shape
    _, _, _, _, H2, W2 = _s2d_geometry(H, W, KH, KW, s, padding)
    pl, pt = padding[0], padding[1]
    xp = F.pad(x.permute(0, 3, 1, 2), (pl, s * W2 - W - pl, pt,
                                       s * H2 - H - pt))
    xp = xp.permute(0, 2, 3, 1)   # [N, s*H2, s*W2, C]
    return xp.reshape(N, H2, s, W2, s, C).permute(0, 1, 3, 2, 4, 5) \
        .reshape(N, H2, W2, s * s * C).contiguous()


def s2d_affine(vec, sample_shape, s, KH, KW, padding, fill):
    """A per-feature vector over an [H,W,C] sample laid out in space-to-depth
    order (``fill`` where the s2d image has no input pixel): the mean /
    rdisp of ``fill_minibatch_s2d``."""
    H, W, C = sample_shape
    y = space_to_depth_ref(vec.reshape(1, H, W, C).float(), s, KH, KW,
                           padding)
    if fill:   # exact values inside, ``fill`` where no input pixel is
        inb = space_to_depth_ref(torch.ones(1, H, W, C), s, KH, KW, padding)
        y = torch.where(inb > 0, y, torch.full_like(y, float(fill)))
    return y.reshape(-1).contiguous()


def fill_minibatch_s2d(src, shuffled, start, count, dst, s, KH, KW, padding,
                       mean2, rdisp2, labels=None, labels_out=None,
                       idx_out=None):
    """fill_minibatch fused with the first conv's space-to-depth transform:
    dst [n,H2,W2,s*s*C] = s2d((src[shuffled[start+i]] - mean) * rdisp),
    with ``mean2`` / ``rdisp2`` from ``s2d_affine``.  Same labels / indices
    outputs as fill_minibatch."""
    N, H, W, C = src.shape
    max_mb = dst.shape[0]
    H2, W2, C2 = s2d_geometry(src.shape, s, KH, KW, padding)
    if _gpu(dst):
        _lib_call("hvk_fill_minibatch_s2d", _p(src), src.numel(),
                  _p(shuffled), int(start), int(count), max_mb, H, W, C, s,
                  padding[1], padding[0], H2, W2, _p(mean2), _p(rdisp2),
                  _p(dst), _p(labels), _p(labels_out), _p(idx_out), _s(dst))
        return dst
    idx = shuffled[start:start + count].long()
    v = src.reshape(N, -1)[idx].float()
    v = space_to_depth_ref(v.reshape(-1, H, W, C), s, KH, KW, padding)
    v = (v.reshape(len(idx), -1) - mean2.reshape(1, -1)) * \
        rdisp2.reshape(1, -1)
    # no input pixel: 0 in the normalised image (the conv's zero padding)
    inb = space_to_depth_ref(torch.ones(1, H, W, C), s, KH, KW,
                             padding).reshape(1, -1)
    v = v * inb
    d = dst.view(max_mb, -1)
    d[:count] = v.to(dst.dtype)
    d[count:] = 0
    if labels_out is not None:
        labels_out[:count] = labels[idx] if labels is not None else -1
        labels_out[count:] = -1
    if idx_out is not None:
        idx_out[:count] = idx.to(idx_out.dtype)
        idx_out[count:] = -1
    return dst


def space_to_depth(x, s, KH, KW, padding):
    N, H, W, C = x.shape
    _, _, KH2, KW2, H2, W2 = _s2d_geometry(H, W, KH, KW, s, padding)
    y = torch.empty(N, H2, W2, s * s * C, dtype=x.dtype, device=x.device)
    _lib_call("hvk_space_to_depth", _p(x), _p(y), N, H, W, C, s, padding[1],
              padding[0], H2, W2, _s(x))
    return y


def _s2d_weights(w, s):
    """[OC][KH][KW][C] -> the space-to-depth weights [OC][KH2][KW2][s*s*C]
    (taps past KH / KW zero) in one kernel."""
    OC, KH, KW, C = w.shape
    KH2, KW2 = -(-KH // s), -(-KW // s)
    w2 = _workspace(("s2dw", id(w)), (OC, KH2, KW2, s * s * C), w.dtype,
                    w.device)
    if _gpu(w) and w.dtype == torch.bfloat16 and w.is_contiguous():
        _lib_call("hvk_s2d_weights", _p(w), _p(w2), OC, KH, KW, C, s, _s(w))
        return w2
    wp = torch.zeros(OC, KH2 * s, KW2 * s, C, dtype=w.dtype, device=w.device)
    wp[:, :KH, :KW].copy_(w)   # taps past KH/KW stay zero
    w2.copy_(wp.view(OC, KH2, s, KW2, s, C).permute(0, 1, 3, 2, 4, 5)
             .reshape(OC, KH2, KW2, s * s * C))
    return w2


def im2col(x, KH, KW, sliding, padding, out=None):
    N, H, W, C = x.shape
    sx, sy = sliding
    pl, pt, pr, pb = padding
    OH, OW = conv_out_size(H, W, KH, KW, sliding, padding)
    K = KH * KW * C
    Kp = (K + 7) // 8 * 8
    M = N * OH * OW
    if out is None:
        out = torch.empty(M, Kp, dtype=x.dtype, device=x.device)
    if _gpu(x):
        _lib_call("hvk_im2col", _p(x), _p(out), N, H, W, C, KH, KW, sy, sx,
                  pt, pl, OH, OW, Kp, _s(x))
        return out
    xp = F.pad(_nchw(x), (pl, pr, pt, pb))
    cols = F.unfold(xp, (KH, KW), stride=(sy, sx))  # [N, C*KH*KW, L]
    cols = cols.view(N, C, KH, KW, -1).permute(0, 4, 2, 3, 1).reshape(M, K)
    out.zero_()
    out[:, :K] = cols.to(out.dtype)
    return out


# stride-1 convolutions with the input tile held in LDS
# (csrc/kernels/conv_halo.hip); False (VELES_AMD_HALO=0) runs every conv on
# the implicit GEMM
_HALO = os.environ.get("VELES_AMD_HALO", "1") != "0"
# the backward-data halo kernel measured slower than the implicit GEMM on
# every AlexNet shape (profiles/r3_experiments.md §9): off unless asked for
_HALO_DGRAD = os.environ.get("VELES_AMD_HALO_DGRAD", "0") != "0"


# channel-chunked halo convs (csrc/kernels/conv_hc.hip): stride-1 3 x 3 and
# 5 x 5 forward / backward-data with a per-chunk input window shared by
# every tap; on by default for the shapes where it measured faster
# (conv_hc.hip hc_plan, profiles/r5/ab_conv_hc_*.log)
_CONV_HC = os.environ.get("VELES_AMD_CONV_HC", "1") != "0"


def set_conv_hc(on, variant=None):
    """A/B knob of the channel-chunked halo conv kernels; ``variant``: -2
    the automatic shape policy (default), -1 every supported shape, > 0 one
    forced configuration of conv_hc.hip's table."""
    global _CONV_HC
    _CONV_HC = bool(on)
    if variant is not None and _lib.available():
        _lib.lib().hvk_hc_variant(int(variant))


def _hc_wpack(dgrad, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, out,
              aux, device):
    """The stage-major filter-bank workspace a conv_hc32 launch packs its
    weights into (csrc/kernels/conv_hc.hip hc32_pack_kernel), or None when
    the call does not take conv_hc32.  One buffer per device and fan-out
    branch, shared by the layers: each launch packs right before its conv
    on the same stream."""
    al = out.data_ptr() % 16 == 0 and (aux is None or aux.data_ptr() % 16 == 0)
    need = int(_lib.lib().hvk_conv_hc_wpack_bytes(
        dgrad, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, int(al)))
    if need <= 0:
        return None
    return _grow_ws("hc32_wpack", need // 2, torch.bfloat16, device)


def set_conv_hc32(on):
    """A/B knob of conv_hc.hip's 32x32x16-MFMA configurations (one tap per
    k-step; default on): off leaves the 16x16x32 two-taps-per-step kernel."""
    if _lib.available():
        _lib.lib().hvk_hc32(int(bool(on)))


def conv_hc_last_variant():
    """conv_hc.hip configuration of the last halo conv launch (tests)."""
    return int(_lib.lib().hvk_hc_last_variant())


def set_conv_halo(on, dgrad=None):
    """Enable / disable the LDS-halo stride-1 conv kernels (A/B runs);
    ``dgrad`` sets the backward-data kernel separately (default: same as
    ``on`` when given, else unchanged)."""
    global _HALO, _HALO_DGRAD
    _HALO = bool(on)
    if dgrad is not None:
        _HALO_DGRAD = bool(dgrad)


def _conv_fwd_call(x, w, bias, out, N, H, W, C, OC, KH, KW, sy, sx, pt, pl,
                   OH, OW, groups, act, stream, q8=None):
    """``q8``: the kernel arguments of a fused fp8 copy of ``out``
    (``fp8._q8_args`` + history length) or None.  Returns whether the fp8
    copy was written (the fused epilogue needs aligned rows and bias)."""
    chunks = _image_chunks(N, x)
    if len(chunks) > 1:
        fused = True
        for n0, n1 in chunks:
            qc = None
            if q8 is not None:
                qc = list(q8)
                qc[0] += n0 * OH * OW * OC     # one byte per element
            fused = _conv_fwd_call(
                x[n0:n1], w, bias, out[n0:n1], n1 - n0, H, W, C, OC, KH, KW,
                sy, sx, pt, pl, OH, OW, groups, act, stream, q8=qc) and fused
        return fused
    sfx = "" if q8 is None else "_q8"
    extra = [] if q8 is None else list(q8)
    if _CONV_HC and q8 is None and sy == 1 and sx == 1 and \
            out.is_contiguous() and x.dtype == torch.bfloat16:
        wp = _hc_wpack(0, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
                       out, None, x.device)
        rc = _lib.lib().hvk_conv_fwd_hc(
            _p(x), _p(w), _p(bias), _p(out), N, H, W, C, OC, KH, KW, pt, pl,
            OH, OW, groups, act, _p(wp), stream)
        if rc == 0:
            return False
        if rc != -2:
            _lib.check(rc, "hvk_conv_fwd_hc")
    if _HALO and sy == 1 and sx == 1 and out.is_contiguous():
        rc = getattr(_lib.lib(), "hvk_conv_fwd_halo" + sfx)(
            _p(x), _p(w), _p(bias), _p(out), N, H, W, C, OC, KH, KW, pt, pl,
            OH, OW, groups, act, *extra, stream)
        if rc == 0:
            return True
        if rc == -3 and q8 is not None:
            # the fused output needs the vector epilogue (aligned rows,
            # bias): unfused call, the caller quantizes separately
            return _conv_fwd_call(x, w, bias, out, N, H, W, C, OC, KH, KW,
                                  sy, sx, pt, pl, OH, OW, groups, act, stream)
        if rc != -2:
            _lib.check(rc, "hvk_conv_fwd_halo" + sfx)
    rc = getattr(_lib.lib(), "hvk_conv_fwd" + sfx)(
        _p(x), _p(w), _p(bias), _p(out), N, H, W, C, OC, KH, KW, sy, sx, pt,
        pl, OH, OW, groups, act, *extra, stream)
    if rc == -3 and q8 is not None:
        _conv_fwd_call(x, w, bias, out, N, H, W, C, OC, KH, KW, sy, sx, pt,
                       pl, OH, OW, groups, act, stream)
        return False
    _lib.check(rc, "hvk_conv_fwd" + sfx)
    return q8 is not None


def conv_fwd(x, w, bias=None, sliding=(1, 1), padding=(0, 0, 0, 0),
             groups=1, act=0, out=None, col_out=None, q8=None,
             q8_scaler=None):
    """x [N,H,W,C], w [OC,KH,KW,C/g] -> y [N,OH,OW,OC].

    ``col_out``: a dict that receives the im2col matrix when the explicit
    path is used (the weight-gradient GEMM reuses it).  ``q8`` /
    ``q8_scaler``: also write the fp8 copy of y that the fp8 layer reading
    it takes (``ops.fp8.conv_fwd`` semantics) - from the GEMM / halo
    epilogue where the kernel path has one, else by a separate quantize
    pass."""
    if q8 is None:
        return _conv_fwd(x, w, bias, sliding, padding, groups, act, out,
                         col_out, None)
    from veles_amd.ops import fp8
    if not _gpu(x):
        y = _conv_fwd(x, w, bias, sliding, padding, groups, act, out,
                      col_out, None)
        fp8._q8_ref(y, q8, q8_scaler)
        return y
    fq = [fp8._q8_args(q8, q8_scaler) + [fp8.HIST], False]
    y = _conv_fwd(x, w, bias, sliding, padding, groups, act, out, col_out,
                  fq)
    if not fq[1]:   # a kernel path without the fused output: separate pass
        fp8.quantize(y, q8_scaler, out=q8)
    return y


def _conv_fwd(x, w, bias, sliding, padding, groups, act, out, col_out, fq):
    """conv_fwd; ``fq`` = [q8 kernel arguments, fused flag] or None: the
    fused-epilogue calls pass the arguments and set the flag."""
    pre = x if isinstance(x, S2DImage) else None   # loader-made s2d input
    N, H, W, C = x.shape
    OC, KH, KW, Cg = w.shape
    if Cg * groups != C or OC % groups:
        raise ValueError("conv_fwd: bad grouping %s %s g=%d" %
                         (tuple(x.shape), tuple(w.shape), groups))
    sx, sy = sliding
    pl, pt, pr, pb = padding
    OH, OW = conv_out_size(H, W, KH, KW, sliding, padding)
    act = act_code(act)
    if pre is not None:
        if pre.s != s2d_factor(C, groups, sliding, KH, KW):
            raise ValueError("conv_fwd: s2d input of factor %d does not fit "
                             "this conv" % pre.s)
        x = pre.x
    if out is None:
        out = torch.empty(N, OH, OW, OC, dtype=x.dtype, device=x.device)
    elif tuple(out.shape) != (N, OH, OW, OC):
        raise ValueError("conv_fwd: out %s, expected %s" % (
            tuple(out.shape), (N, OH, OW, OC)))
    if _gpu(x):
        def call(*a):
            q = None
            if fq is not None and out.dtype == torch.bfloat16 and \
                    out.is_contiguous() and (OC // groups) % 8 == 0:
                q = fq[0]
            fused = _conv_fwd_call(*a, q8=q)
            if q is not None:
                fq[1] = fused
        s2 = s2d_factor(C, groups, sliding, KH, KW)
        if s2:
            # strided RGB conv as a stride-1 conv on the space-to-depth image
            _, _, KH2, KW2, H2, W2 = _s2d_geometry(H, W, KH, KW, s2, padding)
            x2 = pre.x if pre is not None else \
                space_to_depth(x, s2, KH, KW, padding)
            w2 = _s2d_weights(w, s2)
            C2 = s2 * s2 * C
            call(x2, w2, bias, out, N, H2, W2, C2, OC, KH2, KW2, 1, 1, 0, 0,
                 OH, OW, 1, act, _s(x))
            if col_out is not None:
                col_out["col"] = S2DImage(x2, s2, (N, H, W, C))
            return out
        if pad8_ok(C, groups):
            xp = _pad_channels(x)
            wp8 = _pad_weights(w, "wpad8")
            call(xp, wp8, bias, out, N, H, W, _cpad(C), OC, KH, KW, sy, sx,
                 pt, pl, OH, OW, 1, act, _s(x))
            if col_out is not None:
                col_out["col"] = PaddedImage(xp, C)
            return out
        if _DIRECT and groups == 1 and C < 3 and KH * KW * C <= 64 and \
                OC <= 64 and out.is_contiguous() and \
                _lib.lib().hvk_conv_fwd_direct(
                    _p(x), _p(w), _p(bias), _p(out), N, H, W, C, OC, KH, KW,
                    sy, sx, pt, pl, OH, OW, act, _s(x)) == 0:
            # a reduction this short (LeNet conv1: 25 taps) is latency bound
            # on the GEMM tile: direct per-pixel kernel
            return out
        if needs_im2col(C, groups):
            # packed (kw, c) runs: no im2col pass (csrc/kernels/gemm.hip)
            run = KW * C
            runp = (run + 7) // 8 * 8
            wp = _workspace(("wrun", id(w)), (OC, KH, runp), w.dtype,
                            w.device)
            if runp != run:
                wp[:, :, run:].zero_()
            wp[:, :, :run].copy_(w.reshape(OC, KH, run))
            _lib_call("hvk_conv_fwd_run", _p(x), _p(wp), _p(bias), _p(out),
                      N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW, act,
                      _s(x))
            return out
        call(x, w, bias, out, N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW,
             groups, act, _s(x))
        return out
    xp = F.pad(_nchw(x), (pl, pr, pt, pb))
    y = F.conv2d(xp, w.permute(0, 3, 1, 2).float(),
                 None if bias is None else bias.float(), stride=(sy, sx),
                 groups=groups)
    y = act_fwd_ref(y, act)
    out.copy_(_nhwc(y).to(out.dtype))
    return out


def _dgrad_hc_fwd_w(dy, w, out, aux, N, H, W, C, OC, KH, KW, sy, sx, pt, pl,
                    OH, OW, groups, aux_act):
    """Backward-data on conv_hc32 from the forward-layout weights: its
    filter-bank pack reads them directly, so the [g][c][kh][kw][oc]
    permutation pass is skipped.  False when that path does not apply (the
    caller permutes and dispatches as before)."""
    if not (_CONV_HC and sx == 1 and sy == 1 and out.is_contiguous() and
            dy.dtype == torch.bfloat16 and w.is_contiguous() and
            (aux is None or aux.is_contiguous())):
        return False
    chunks = list(_image_chunks(N, dy))
    if len(chunks) != 1:
        return False
    wp = _hc_wpack(1, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups, out,
                   aux, dy.device)
    if wp is None:
        return False
    rc = _lib.lib().hvk_conv_dgrad_hc_w(
        _p(dy), _p(w), _p(out), N, H, W, C, OC, KH, KW, pt, pl, OH, OW,
        groups, _p(aux), aux_act, _p(wp), _s(dy))
    if rc in (-2, -3):
        return False
    _lib.check(rc, "hvk_conv_dgrad_hc_w")
    return True


def _dgrad_call(dy, wt, out, aux, N, H, W, C, OC, KH, KW, sy, sx, pt, pl,
                OH, OW, groups, aux_act):
    if _CONV_HC and sx == 1 and sy == 1 and out.is_contiguous() and \
            dy.dtype == torch.bfloat16 and \
            (aux is None or aux.is_contiguous()):
        wp = _hc_wpack(1, N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
                       out, aux, dy.device)
        rc = _lib.lib().hvk_conv_dgrad_hc(
            _p(dy), _p(wt), _p(out), N, H, W, C, OC, KH, KW, pt, pl, OH, OW,
            groups, _p(aux), aux_act, _p(wp), _s(dy))
        if rc == 0:
            return
        if rc != -2:
            _lib.check(rc, "hvk_conv_dgrad_hc")
    if _HALO_DGRAD and sx == 1 and sy == 1 and out.is_contiguous():
        rc = _lib.lib().hvk_conv_dgrad_halo(
            _p(dy), _p(wt), _p(out), N, H, W, C, OC, KH, KW, pt, pl, OH,
            OW, groups, _p(aux), aux_act, _s(dy))
        if rc == 0:
            return
        if rc != -2:
            _lib.check(rc, "hvk_conv_dgrad_halo")
    _lib_call("hvk_conv_dgrad_t", _p(dy), _p(wt), _p(out), N, H, W, C,
              OC, KH, KW, sy, sx, pt, pl, OH, OW, groups, _p(aux),
              aux_act, _s(dy))


def conv_dgrad(dy, w, x_shape, sliding=(1, 1), padding=(0, 0, 0, 0),
               groups=1, aux=None, aux_act=0, out=None):
    """dx [N,H,W,C] = conv^T(dy, w) [* f'(aux)]."""
    N, H, W, C = x_shape
    _, OH, OW, OC = dy.shape
    _, KH, KW, Cg = w.shape
    sx, sy = sliding
    pl, pt, pr, pb = padding
    aux_act = act_code(aux_act)
    # the kernels index dy, w, aux and out with this geometry: a mismatch
    # would read or write out of bounds on the device
    if (Cg * groups != C or OC % groups or dy.shape[0] != N or
            w.shape[0] != OC or
            (OH, OW) != conv_out_size(H, W, KH, KW, sliding, padding) or
            (out is not None and tuple(out.shape) != (N, H, W, C)) or
            (aux is not None and tuple(aux.shape) != (N, H, W, C))):
        raise ValueError(
            "conv_dgrad geometry: x %s, dy %s, w %s, sliding %s, padding %s, "
            "groups %d" % (tuple(x_shape), tuple(dy.shape), tuple(w.shape),
                           sliding, padding, groups))
    if out is None:
        out = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
    if _gpu(dy):
        # weights permuted to [g][c][kh][kw][oc]: a dense K-major B operand
        OCg, Cg = OC // groups, C // groups
        if groups == 1 and OC % 8:
            # an output-channel count off the 16-byte grid (LeNet's 50)
            # would force the per-element A loader (5x slower): zero-pad
            # dy's and the weights' channel dimension to a multiple of 8
            OCp = -(-OC // 8) * 8
            wt = _workspace(("dgrad_wtp", id(w)), (1, C, KH, KW, OCp),
                            w.dtype, w.device, zero=True)
            wt[..., :OC].copy_(w.view(1, OC, KH, KW, C).permute(
                0, 4, 2, 3, 1))
            dyp = _workspace(("dgrad_dyp", N, OH, OW, OCp), (N, OH, OW, OCp),
                             dy.dtype, dy.device, zero=True)
            dyp[..., :OC].copy_(dy)
            dy, OC = dyp, OCp
        else:
            if _dgrad_hc_fwd_w(dy, w, out, aux, N, H, W, C, OC, KH, KW, sy,
                               sx, pt, pl, OH, OW, groups, aux_act):
                return out
            wt = _workspace(("dgrad_wt", id(w)), (groups, Cg, KH, KW, OCg),
                            w.dtype, w.device)
            wt.copy_(w.view(groups, OCg, KH, KW, Cg).permute(0, 4, 2, 3, 1))
        for n0, n1 in _image_chunks(N, dy):
            _dgrad_call(dy[n0:n1], wt, out[n0:n1],
                        None if aux is None else aux[n0:n1], n1 - n0, H, W,
                        C, OC, KH, KW, sy, sx, pt, pl, OH, OW, groups, aux_act)
        return out
    Hp, Wp = H + pt + pb, W + pl + pr
    dxp = torch.nn.grad.conv2d_input((N, C, Hp, Wp),
                                     w.permute(0, 3, 1, 2).float(),
                                     _nchw(dy), stride=(sy, sx), groups=groups)
    dx = dxp[:, :, pt:pt + H, pl:pl + W]
    if aux is not None:
        dx = dx * act_bwd_ref(_nchw(aux), aux_act)
    out.copy_(_nhwc(dx).to(out.dtype))
    return out


def conv_wgrad(x, dy, dw, sliding=(1, 1), padding=(0, 0, 0, 0), groups=1,
               splits=None, col=None, dbias=None):
    """dw (float32 [OC,KH,KW,C/g]) += sum over pixels of dy (x) im2col(x);
    ``dbias`` (float32 [OC]) += sum over pixels of dy, fused into the same
    GEMM.  ``col``: an explicit im2col matrix to use instead (optional)."""
    if isinstance(x, S2DImage):   # loader-made s2d input (conv_fwd)
        col, x = x, x.x
        N, H, W, C = col.shape
    else:
        N, H, W, C = x.shape
    _, OH, OW, OC = dy.shape
    _, KH, KW, Cg = dw.shape
    sx, sy = sliding
    pl, pt, pr, pb = padding
    if dw.dtype != torch.float32:
        raise TypeError("conv_wgrad accumulates into float32")
    # the kernels index x, dy and dw with this geometry: a mismatch would
    # read out of bounds on the device
    if (Cg * groups != C or OC % groups or dy.shape[0] != N or
            OH != (H + pt + pb - KH) // sy + 1 or
            OW != (W + pl + pr - KW) // sx + 1):
        raise ValueError(
            "conv_wgrad geometry: x %s, dy %s, dw %s, sliding %s, padding "
            "%s, groups %d" % ((N, H, W, C), tuple(dy.shape), tuple(dw.shape),
                               sliding, padding, groups))
    if _gpu(x):
        xt = col.x if isinstance(col, (S2DImage, PaddedImage)) else x
        chunks = _image_chunks(N, xt, dy)
        if len(chunks) > 1:
            # a sum over pixels: the image chunks accumulate into dw / dbias
            for n0, n1 in chunks:
                c = col
                if isinstance(col, S2DImage):
                    c = S2DImage(col.x[n0:n1], col.s, (n1 - n0,) +
                                 tuple(col.shape[1:]))
                elif isinstance(col, PaddedImage):
                    c = PaddedImage(col.x[n0:n1], col.C)
                elif col is not None:
                    c = col[n0 * OH * OW:n1 * OH * OW]
                if isinstance(col, S2DImage) and col.x is x:
                    xc = c            # the loader-made s2d input itself
                else:
                    xc = x[n0:n1]
                conv_wgrad(xc, dy[n0:n1], dw, sliding, padding, groups,
                           None, c, dbias)
            return dw
        s2 = s2d_factor(C, groups, sliding, KH, KW)
        if s2:
            x2 = col.x if isinstance(col, S2DImage) else \
                space_to_depth(x, s2, KH, KW, padding)
            H2, W2, C2 = x2.shape[1], x2.shape[2], x2.shape[3]
            KH2, KW2 = -(-KH // s2), -(-KW // s2)
            # self-clearing workspace: zeroed once, cleared again by the fold
            dw2 = _workspace(("s2dg", dw.data_ptr()), (OC, KH2, KW2, C2),
                             torch.float32, dw.device, zero=True)
            if not _halo_wgrad(x2, dy, dw2, dbias, N, H2, W2, C2, OC, KH2,
                               KW2, 0, 0, OH, OW, 1, splits):
                # logged with the logical image shape: the autotuner
                # replays the call on a plain image (the s2d data has C2
                # channels)
                sp = splits or _wgrad_splits_for(
                    (N, H, W, C), dy, dw, sliding, padding, groups,
                    (N * OH * OW, OC, KH2 * KW2 * C2 + 1, 1))
                _lib_call("hvk_conv_wgrad", _p(x2), _p(dy), _p(dw2), N, H2,
                          W2, C2, OC, KH2, KW2, 1, 1, 0, 0, OH, OW, 1,
                          int(sp), _p(dbias), _s(x))
            if dw.is_contiguous():
                _lib_call("hvk_s2d_grad_fold", _p(dw2), _p(dw), OC, KH, KW, C,
                          s2, 1, _s(x))
                return dw
            full = dw2.view(OC, KH2, KW2, s2, s2, C).permute(
                0, 1, 3, 2, 4, 5).reshape(OC, KH2 * s2, KW2 * s2, C)
            dw += full[:, :KH, :KW]
            dw2.zero_()
            return dw
        if pad8_ok(C, groups):
            xp = col.x if isinstance(col, PaddedImage) and \
                col.x.shape[:3] == x.shape[:3] else _pad_channels(x)
            # self-clearing padded gradient: zeroed once, cleared after the fold
            Cp = _cpad(C)
            dwp = _workspace(("wgpad8", dw.data_ptr()), (OC, KH, KW, Cp),
                             torch.float32, dw.device, zero=True)
            sp = splits or _wgrad_splits_for(
                xp, dy, dwp, sliding, padding, 1,
                (N * OH * OW, OC, KH * KW * Cp + 1, 1))
            _lib_call("hvk_conv_wgrad", _p(xp), _p(dy), _p(dwp), N, H, W, Cp,
                      OC, KH, KW, sy, sx, pt, pl, OH, OW, 1, int(sp),
                      _p(dbias), _s(x))
            dw += dwp[..., :C]
            dwp.zero_()
            return dw
        if isinstance(col, (S2DImage, PaddedImage)):
            col = None
        if col is not None:
            K = KH * KW * Cg
            M = N * OH * OW
            sp = splits or wgrad_splits(M, OC, K, 1)
            gemm(dy.reshape(M, OC), col[:, :K], trans_a=True,
                 out=dw.view(OC, K), accumulate=True, splits=sp,
                 bias_grad=dbias)
            return dw
        if needs_im2col(C, groups):
            runp = (KW * C + 7) // 8 * 8
            sp = splits or _wgrad_splits_for(
                x, dy, dw, sliding, padding, groups,
                (N * OH * OW, OC, KH * runp + 1, 1))
            _lib_call("hvk_conv_wgrad_run", _p(x), _p(dy), _p(dw), _p(dbias),
                      N, H, W, C, OC, KH, KW, sy, sx, pt, pl, OH, OW,
                      int(sp), _s(x))
            return dw
        if (sy, sx) == (1, 1) and _halo_wgrad(x, dy, dw, dbias, N, H, W, C,
                                               OC, KH, KW, pt, pl, OH, OW,
                                               groups, splits):
            return dw
        if splits is None:
            splits = _wgrad_splits_for(
                x, dy, dw, sliding, padding, groups,
                (N * OH * OW, OC // groups, KH * KW * Cg + 1, groups))
        _lib_call("hvk_conv_wgrad", _p(x), _p(dy), _p(dw), N, H, W, C, OC, KH,
                  KW, sy, sx, pt, pl, OH, OW, groups, int(splits), _p(dbias),
                  _s(x))
        return dw
    xp = F.pad(_nchw(x), (pl, pr, pt, pb))
    g = torch.nn.grad.conv2d_weight(xp, (OC, Cg, KH, KW), _nchw(dy),
                                    stride=(sy, sx), groups=groups)
    dw += g.permute(0, 2, 3, 1)
    if dbias is not None:
        dbias += dy.float().reshape(-1, OC).sum(0)
    return dw


_HALO_WGRAD = os.environ.get("VELES_AMD_HALO_WGRAD", "1") != "0"


def set_halo_wgrad(on):
    """A/B knob of the halo weight-gradient kernel (env
    VELES_AMD_HALO_WGRAD)."""
    global _HALO_WGRAD
    _HALO_WGRAD = bool(on)


def _halo_wgrad(x, dy, dw, dbias, N, H, W, C, OC, KH, KW, pt, pl, OH, OW,
                groups, splits=None):
    """Stride-1 weight gradient on the halo kernel (csrc/kernels/
    wgrad_halo.hip) when the shape takes it: the input window of each
    64-pixel step is staged once and read by every tap; split over pixels
    into workspace slices that a finishing pass adds into dw / dbias in
    split order (deterministic).  ``splits``: the caller's pixel split
    count (None: the kernel's plan).  False: the caller uses
    hvk_conv_wgrad."""
    # the LDS-DMA loads need 16-B aligned X / dY: refuse misaligned views
    # here (the launch would fail after a plan-only call that said yes)
    if not _HALO_WGRAD or x.dtype != torch.bfloat16 or \
            dy.dtype != torch.bfloat16 or not dw.is_contiguous() or \
            not x.is_contiguous() or not dy.is_contiguous() or \
            x.data_ptr() % 16 or dy.data_ptr() % 16:
        return False
    from veles_amd.ops import _lib
    fn = _lib.lib().hvk_conv_wgrad_halo
    geo = (N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
           int(splits) if splits else 0)
    need = fn(_p(x), _p(dy), _p(dw), _p(dbias), None, *geo, _s(x))
    if need < 0:
        return False
    ws = _grow_ws("wgrad_halo_ws", int(need), torch.float32, x.device)
    rc = fn(_p(x), _p(dy), _p(dw), _p(dbias), _p(ws), *geo, _s(x))
    _lib.check(int(rc), "hvk_conv_wgrad_halo")
    return True


# 512 blocks (2 per CU) measured best on AlexNet b512 (72.7k img/s vs 71.6k
# at 2048 and 69.0k at 4096: fewer splits = fewer f32 atomics)
_WGRAD_BLOCKS = int(os.environ.get("HVK_WGRAD_BLOCKS", "512"))


def _wgrad_splits_for(x, dy, dw, sliding, padding, groups, shape):
    """wgrad_splits, overridden per shape by the device tuning table (the
    call's geometry is logged for the autotuner, ops/autotune.py)."""
    from veles_amd.ops import autotune
    default = wgrad_splits(*shape)
    autotune.log_call("wgrad", shape, {
        "x": tuple(x if isinstance(x, tuple) else x.shape), "dy": tuple(dy.shape), "dw": tuple(dw.shape),
        "sliding": tuple(sliding), "padding": tuple(padding),
        "groups": groups, "default": default})
    t = autotune.lookup("wgrad", *shape)
    if deterministic():
        return 1
    return default if t is None else max(1, t)


def wgrad_splits(P, M, N, groups, target_blocks=None):
    """Pixel (K) splits of a weight-gradient GEMM: enough blocks to fill the
    256 CUs, few enough that the f32 atomic reduction stays small (1 in
    deterministic mode: no atomics)."""
    if deterministic():
        return 1
    target_blocks = target_blocks or _WGRAD_BLOCKS
    tiles = ((M + 127) // 128) * ((N + 127) // 128) * groups
    splits = max(1, min(target_blocks // max(tiles, 1), P // 256))
    return splits


# ------------------------------------------------------------- reductions
def col_sum(x2d, out=None, scale=1.0, accumulate=False):
    """out[c] (+)= scale * sum_r x[r][c]  (float32 out)."""
    R, C = x2d.shape
    if out is None:
        out = torch.zeros(C, dtype=torch.float32, device=x2d.device)
    elif not accumulate:
        out.zero_()
    if _gpu(x2d) and not deterministic():
        _lib_call("hvk_col_sum", _p(x2d), DT[x2d.dtype], R, C, _p(out),
                  float(scale), _s(x2d))
        return out
    out += scale * x2d.float().sum(0)
    return out


def transpose_colsum(x2d, out=None, colsum=None, accumulate=False, ws=None):
    """out[C][R] = x[R][C]^T (bf16) and colsum[c] (+)= sum_r x[r][c] (float32,
    summed per 64-row slab, then the slabs in order: deterministic).  One
    pass over x: the FC weight gradient's dY^T plus its bias gradient.
    GPU: R and C multiples of 64; ws, float32 of (R / 64) * C, is the slab
    workspace (allocated when None)."""
    R, C = x2d.shape
    if out is None:
        out = torch.empty(C, R, dtype=x2d.dtype, device=x2d.device)
    if _gpu(x2d):
        if x2d.dtype != torch.bfloat16 or R % 64 or C % 64 or \
                not x2d.is_contiguous() or not out.is_contiguous():
            raise ValueError("transpose_colsum: contiguous bf16 with R, C "
                             "multiples of 64")
        if ws is None:
            ws = torch.empty(R // 64 * C, dtype=torch.float32,
                             device=x2d.device)
        _lib_call("hvk_transpose_colsum", _p(x2d), R, C, _p(out),
                  _p(colsum) if colsum is not None else None,
                  int(bool(accumulate)), _p(ws), _s(x2d))
        return out
    out.copy_(x2d.t())
    if colsum is not None:
        sums = x2d.float().sum(0)
        if accumulate:
            colsum += sums
        else:
            colsum.copy_(sums)
    return out


def row_sum(x2d, out=None, scale=1.0):
    R, C = x2d.shape
    if out is None:
        out = torch.empty(R, dtype=torch.float32, device=x2d.device)
    if _gpu(x2d):
        _lib_call("hvk_row_sum", _p(x2d), DT[x2d.dtype], R, C, _p(out),
                  float(scale), _s(x2d))
        return out
    out.copy_(scale * x2d.float().sum(1))
    return out


# ----------------------------------------------------------------- pooling
POOL = {"max": 0, "avg": 1, "maxabs": 2}


def pool_out_size(h, w, ky, kx, sy, sx):
    """Znicz pooling geometry: partial windows at the far edge are kept
    (ceil), never a window that starts outside the input."""
    return (h - ky + sy - 1) // sy + 1 if h > ky else 1, \
        (w - kx + sx - 1) // sx + 1 if w > kx else 1


def _pool_ref(x, ky, kx, sy, sx, mode, OH, OW):
    N, H, W, C = x.shape
    xf = x.float()
    neg = float("-inf")
    Hp, Wp = (OH - 1) * sy + ky, (OW - 1) * sx + kx
    pad = torch.full((N, Hp, Wp, C), float("nan"))
    pad[:, :H, :W, :] = xf
    idx = torch.arange(N * H * W * C).view(N, H, W, C)
    pidx = torch.full((N, Hp, Wp, C), -1, dtype=torch.long)
    pidx[:, :H, :W, :] = idx
    best = torch.full((N, OH, OW, C), neg)
    bkey = torch.full((N, OH, OW, C), neg)
    bidx = torch.full((N, OH, OW, C), -1, dtype=torch.long)
    s = torch.zeros(N, OH, OW, C)
    cnt = torch.zeros(N, OH, OW, C)
    for dy in range(ky):
        for dx in range(kx):
            v = pad[:, dy:dy + (OH - 1) * sy + 1:sy, dx:dx + (OW - 1) * sx + 1:sx, :]
            vi = pidx[:, dy:dy + (OH - 1) * sy + 1:sy, dx:dx + (OW - 1) * sx + 1:sx, :]
            valid = ~torch.isnan(v)
            if mode == 1:
                s += torch.where(valid, v, torch.zeros_like(v))
                cnt += valid.float()
            else:
                key = v.abs() if mode == 2 else v
                better = valid & ((bidx < 0) | (key > bkey))
                best = torch.where(better, v, best)
                bkey = torch.where(better, key, bkey)
                bidx = torch.where(better, vi, bidx)
    if mode == 1:
        return s / cnt.clamp(min=1), None
    return best, bidx.to(torch.int32)


def pool_fwd(x, ky, kx, sliding=None, mode="max", out=None, argmax=None):
    """NHWC pooling; returns (y, argmax) - argmax is the flat input index of
    the chosen element (None for avg)."""
    sx, sy = sliding or (kx, ky)
    N, H, W, C = x.shape
    OH, OW = pool_out_size(H, W, ky, kx, sy, sx)
    m = POOL[mode]
    if out is None:
        out = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
    if m != 1 and argmax is None:
        argmax = torch.empty(N, OH, OW, C, dtype=torch.int32, device=x.device)
    if _gpu(x):
        _lib_call("hvk_pool_fwd", _p(x), _p(out), _p(argmax), N, H, W, C, OH,
                  OW, ky, kx, sy, sx, 0, 0, m, _s(x))
        return out, argmax
    y, idx = _pool_ref(x.cpu(), ky, kx, sy, sx, m, OH, OW)
    out.copy_(y.to(out.dtype))
    if idx is not None:
        argmax.copy_(idx)
    return out, argmax


def stochastic_pool_u(n, seed, device="cpu"):
    """The uniforms hvk_stochastic_pool draws: (hash32(o, seed) >> 8) / 2^24
    for output element o."""
    o = torch.arange(n, dtype=torch.int64, device=device)
    return (_hash32(o, int(seed) & 0xFFFFFFFF) >> 8).float() / 16777216.0


def stochastic_pool(x, ky, kx, sliding=None, use_abs=False, train=True,
                    seed=0, seed_dev=None, out=None, argmax=None):
    """Stochastic pooling (NHWC): train - draw a window element with
    probability max(x, 0) / sum (|x| for use_abs; uniform when the sum is 0);
    test - the probability-weighted average.  Returns (y, argmax) with the
    flat input offset of the drawn (most probable) element.  GPU:
    ``hvk_stochastic_pool`` with the seed in device memory (``seed_dev``,
    int32 [1]); the CPU reference draws the same uniforms."""
    sx, sy = sliding or (kx, ky)
    N, H, W, C = x.shape
    OH, OW = pool_out_size(H, W, ky, kx, sy, sx)
    if out is None:
        out = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
    if argmax is None:
        argmax = torch.empty(N, OH, OW, C, dtype=torch.int32, device=x.device)
    if _gpu(x):
        if seed_dev is None:
            seed_dev = torch.tensor([int(seed) & 0x7FFFFFFF],
                                    dtype=torch.int32, device=x.device)
        _lib_call("hvk_stochastic_pool", _p(x), _p(out), _p(argmax), N, H, W,
                  C, OH, OW, ky, kx, sy, sx, int(bool(use_abs)),
                  int(bool(train)), _p(seed_dev), _s(x))
        return out, argmax
    if seed_dev is not None:
        seed = int(seed_dev.reshape(-1)[0]) & 0xFFFFFFFF
    xf = x.float().cpu()
    Hp, Wp = (OH - 1) * sy + ky, (OW - 1) * sx + kx
    pad = torch.zeros(N, Hp, Wp, C)
    pad[:, :H, :W] = xf
    ok = torch.zeros(N, Hp, Wp, C, dtype=torch.bool)
    ok[:, :H, :W] = True
    idx = torch.full((N, Hp, Wp, C), -1, dtype=torch.long)
    idx[:, :H, :W] = torch.arange(N * H * W * C).view(N, H, W, C)
    vals, oks, ids = [], [], []
    for dy in range(ky):
        for dx in range(kx):
            sl = (slice(None), slice(dy, dy + (OH - 1) * sy + 1, sy),
                  slice(dx, dx + (OW - 1) * sx + 1, sx))
            vals.append(pad[sl])
            oks.append(ok[sl])
            ids.append(idx[sl])
    w = [(v.abs() if use_abs else v.clamp(min=0)) * o
         for v, o in zip(vals, oks)]
    tot = torch.zeros_like(vals[0])
    cnt = torch.zeros_like(vals[0])
    for wi, o in zip(w, oks):  # sequential, as the kernel sums
        tot = tot + wi
        cnt = cnt + o.float()
    inv = torch.where(tot > 0, 1.0 / tot.clamp(min=1e-38),
                      torch.zeros_like(tot))
    uni = 1.0 / cnt
    prs = [torch.where(tot > 0, wi * inv, uni) * o for wi, o in zip(w, oks)]
    y = torch.zeros_like(tot)
    pick = torch.full(tot.shape, -1, dtype=torch.long)
    if train:
        u = stochastic_pool_u(tot.numel(), seed).view(tot.shape)
        cum = torch.zeros_like(tot)
        taken = torch.zeros(tot.shape, dtype=torch.bool)
        for v, pr, o, i in zip(vals, prs, oks, ids):
            cum = cum + pr
            hit = o & ~taken & (cum >= u)
            fall = o & ~taken & ~hit
            y = torch.where(hit | fall, v, y)
            pick = torch.where(hit | fall, i, pick)
            taken = taken | hit
    else:
        best = torch.full(tot.shape, -1.0)
        for v, pr, o, i in zip(vals, prs, oks, ids):
            y = y + pr * v
            better = o & (pr > best)
            best = torch.where(better, pr, best)
            pick = torch.where(better, i, pick)
    out.copy_(y.to(out.dtype))
    argmax.copy_(pick.to(torch.int32))
    return out, argmax


def pool_bwd(dy, argmax, x_shape, ky, kx, sliding=None, mode="max",
             aux=None, aux_act=0, out=None):
    sx, sy = sliding or (kx, ky)
    N, H, W, C = x_shape
    _, OH, OW, _ = dy.shape
    m = POOL[mode]
    aux_act = act_code(aux_act)
    if out is None:
        out = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
    if _gpu(dy):
        _lib_call("hvk_pool_bwd", _p(dy), _p(argmax), _p(out), N, H, W, C, OH,
                  OW, ky, kx, sy, sx, 0, 0, m, _p(aux), aux_act, _s(dy))
        return out
    g = dy.float()
    dx = torch.zeros(N * H * W * C)
    if m == 1:
        dx = dx.view(N, H, W, C)
        cnt = torch.zeros(N, OH, OW, C)
        for oh in range(OH):
            h0, h1 = oh * sy, min(oh * sy + ky, H)
            for ow in range(OW):
                w0, w1 = ow * sx, min(ow * sx + kx, W)
                c = (h1 - h0) * (w1 - w0)
                dx[:, h0:h1, w0:w1, :] += (g[:, oh, ow, :] / c)[:, None, None, :]
    else:
        dx.index_add_(0, argmax.long().reshape(-1), g.reshape(-1))
        dx = dx.view(N, H, W, C)
    if aux is not None:
        dx = dx * act_bwd_ref(aux.float(), aux_act)
    out.copy_(dx.to(out.dtype))
    return out


def pool2_ok(x_shape, ky, kx, sliding):
    """Geometry of the argmax-free 2 x 2 / stride-2 pooling kernels."""
    if len(x_shape) != 4:
        return False
    N, H, W, C = x_shape
    return ky == 2 and kx == 2 and tuple(sliding) == (2, 2) and \
        C % 8 == 0 and H % 2 == 0 and W % 2 == 0


def _q8_pool_args(q8, qs):
    from veles_amd.ops import fp8 as _f8
    if q8 is None:
        return [None, None, None, 1.0, 0, _f8.HIST]
    return [q8.data_ptr(), qs.state.data_ptr(), qs.shard.data_ptr(),
            float(qs.fmax_eff), qs.fmt, _f8.HIST]


# The pooling and LRN-pool kernels index with 32-bit element offsets (they
# refuse tensors of 2^31 elements or more): larger batches run in image
# chunks (every image is independent in these ops; NHWC slices along N stay
# contiguous and 16-B aligned for C % 8 == 0)
_CHUNK_ELEMS = 1 << 31


def _n_chunks(N, per_image):
    """[(n0, n1)] image ranges of under _CHUNK_ELEMS elements each, or
    None when the whole batch fits."""
    if N * per_image < _CHUNK_ELEMS:
        return None
    step = max(1, (_CHUNK_ELEMS - 1) // max(per_image, 1))
    return [(n0, min(N, n0 + step)) for n0 in range(0, N, step)]


def _sl(t, n0, n1):
    return None if t is None else t[n0:n1]


def _q8_sliceable(q8, N):
    """a fused fp8 copy splits with its result (the kernels only take the
    max of |result| into the scaler's shards: atomics, so chunks add up)"""
    return q8 is None or (q8.dim() == 4 and q8.shape[0] == N and
                          q8.is_contiguous())


def pool2_fwd(x, mode="max", out=None, q8=None, q8_scaler=None):
    """2 x 2 / stride-2 NHWC pooling that writes no argmax: ``pool2_bwd``
    recomputes the window's choice from x.  ``q8`` / ``q8_scaler``: also the
    fp8 copy of the result for the next fp8 layer (fused quantisation)."""
    N, H, W, C = x.shape
    m = POOL[mode]
    if out is None:
        out = torch.empty(N, H // 2, W // 2, C, dtype=x.dtype,
                          device=x.device)
    if _gpu(x):
        ch = _n_chunks(N, H * W * C) if _q8_sliceable(q8, N) else None
        if ch:
            for n0, n1 in ch:
                pool2_fwd(x[n0:n1], mode, out=out[n0:n1],
                          q8=_sl(q8, n0, n1), q8_scaler=q8_scaler)
            return out
        _lib_call("hvk_pool2_fwd_q8", _p(x), _p(out), N, H, W, C, m,
                  *_q8_pool_args(q8, q8_scaler), _s(x))
        return out
    y, _ = pool_fwd(x, 2, 2, (2, 2), mode, out=out)
    if q8 is not None:
        from veles_amd.ops import fp8 as _f8
        _f8._q8_ref(y, q8, q8_scaler)
    return y


def pool2_bwd(x, dy, mode="max", aux=None, aux_act=0, out=None, q8=None,
              q8_scaler=None):
    N, H, W, C = x.shape
    m = POOL[mode]
    aux_act = act_code(aux_act)
    if out is None:
        out = torch.empty_like(x, dtype=dy.dtype)
    if _gpu(x):
        ch = _n_chunks(N, H * W * C) if _q8_sliceable(q8, N) else None
        if ch:
            for n0, n1 in ch:
                pool2_bwd(x[n0:n1], dy[n0:n1], mode, aux=_sl(aux, n0, n1),
                          aux_act=aux_act, out=out[n0:n1],
                          q8=_sl(q8, n0, n1), q8_scaler=q8_scaler)
            return out
        _lib_call("hvk_pool2_bwd_q8", _p(x), _p(dy), _p(out), N, H, W, C, m,
                  _p(aux), aux_act, *_q8_pool_args(q8, q8_scaler), _s(x))
        return out
    if q8 is not None:
        dx = pool2_bwd(x, dy, mode, aux=aux, aux_act=aux_act, out=out)
        from veles_amd.ops import fp8 as _f8
        _f8._q8_ref(dx, q8, q8_scaler)
        return dx
    am = None
    if m != 1:
        _, am = pool_fwd(x, 2, 2, (2, 2), mode)
    return pool_bwd(dy, am, (N, H, W, C), 2, 2, (2, 2), mode, aux=aux,
                    aux_act=aux_act, out=out)


# --------------------------------------------------------------------- LRN
def _lrn_ref(x, n, alpha, beta, k):
    x2 = x * x
    half = n // 2
    xp = F.pad(x2, (half, half))
    s = sum(xp[..., i:i + x.shape[-1]] for i in range(2 * half + 1))
    return x * torch.pow(k + alpha * s, -beta)


def lrn_fwd(x, n=5, alpha=1e-4, beta=0.75, k=2.0, out=None):
    """Across-channel LRN on NHWC: y = x (k + alpha sum x^2)^-beta."""
    C = x.shape[-1]
    P = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    if _gpu(x):
        _lib_call("hvk_lrn_fwd", _p(x), _p(out), P, C, n, float(alpha),
                  float(beta), float(k), _s(x))
        return out
    out.copy_(_lrn_ref(x.float(), n, alpha, beta, k).to(out.dtype))
    return out


def lrn_bwd(x, dy, n=5, alpha=1e-4, beta=0.75, k=2.0, aux=None, aux_act=0,
            out=None):
    C = x.shape[-1]
    P = x.numel() // C
    aux_act = act_code(aux_act)
    if out is None:
        out = torch.empty_like(dy)
    if _gpu(x):
        _lib_call("hvk_lrn_bwd", _p(x), _p(dy), _p(out), P, C, n, float(alpha),
                  float(beta), float(k), _p(aux), aux_act, _s(x))
        return out
    xf = x.float().detach().requires_grad_(True)
    y = _lrn_ref(xf, n, alpha, beta, k)
    y.backward(dy.float())
    dx = xf.grad
    if aux is not None:
        dx = dx * act_bwd_ref(aux.float(), aux_act)
    out.copy_(dx.to(out.dtype))
    return out


# ------------------------------------------------------- fused LRN -> pool
def lrn_pool_fusable(C, n, ky, kx, sliding):
    """Shapes the fused LRN -> 3x3 max-pool kernels take."""
    sx, sy = sliding
    return C % 8 == 0 and n // 2 <= 4 and ky == 3 and kx == 3 and \
        sx >= 2 and sy >= 2


def window_index_to_offsets(am, x_shape, ky, kx, sliding):
    """A uint8 window-local argmax (0 .. ky*kx-1, row-major inside the pooling
    window) -> flat int32 offsets into the NHWC input, the format of
    ``pool_fwd``'s argmax (reference paths and tests)."""
    sx, sy = sliding
    N, H, W, C = x_shape
    _, OH, OW, _ = am.shape
    dev = am.device
    a = am.long()
    oh = torch.arange(OH, device=dev).view(1, OH, 1, 1)
    ow = torch.arange(OW, device=dev).view(1, 1, OW, 1)
    n = torch.arange(N, device=dev).view(N, 1, 1, 1)
    c = torch.arange(C, device=dev).view(1, 1, 1, C)
    h = oh * sy + a // kx
    w = ow * sx + a % kx
    return (((n * H + h) * W + w) * C + c).to(torch.int32)


def lrn_pool_fwd(x, n, alpha, beta, k, ky, kx, sliding, out=None,
                 argmax=None):
    """max_pool(lrn(x)) without materialising lrn(x); ``argmax`` indexes the
    (virtual) LRN output, i.e. x's geometry.  A uint8 ``argmax`` (GPU,
    stride 2) holds the window-local index instead: 1 byte per element
    (``window_index_to_offsets`` converts)."""
    sx, sy = sliding
    N, H, W, C = x.shape
    OH, OW = pool_out_size(H, W, ky, kx, sy, sx)
    if out is None:
        out = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
    if argmax is None:
        argmax = torch.empty(N, OH, OW, C, dtype=torch.int32, device=x.device)
    if _gpu(x):
        ch = _n_chunks(N, H * W * C) if argmax.dtype == torch.uint8 else None
        if ch:
            for n0, n1 in ch:
                lrn_pool_fwd(x[n0:n1], n, alpha, beta, k, ky, kx, sliding,
                             out=out[n0:n1], argmax=argmax[n0:n1])
            return out, argmax
        if argmax.dtype == torch.uint8:
            if (sx, sy) != (2, 2):
                raise ValueError("uint8 window-index argmax: stride 2 only")
            _lib_call("hvk_lrn_pool_fwd_u8", _p(x), _p(out), _p(argmax), N,
                      H, W, C, OH, OW, n, float(alpha), float(beta), float(k),
                      _s(x))
            return out, argmax
        _lib_call("hvk_lrn_pool_fwd", _p(x), _p(out), _p(argmax), N, H, W, C,
                  OH, OW, sy, sx, n, float(alpha), float(beta), float(k),
                  _s(x))
        return out, argmax
    y = lrn_fwd(x.float(), n, alpha, beta, k)
    if argmax.dtype == torch.uint8:
        yo, off = pool_fwd(y, ky, kx, sliding, "max", out=out)
        # window-local index of the chosen flat offset
        hw = (off.long() // C)
        h, w = (hw // W) % H, hw % W
        oh = torch.arange(OH).view(1, OH, 1, 1)
        ow = torch.arange(OW).view(1, 1, OW, 1)
        argmax.copy_(((h - oh * sy) * kx + (w - ow * sx)).to(torch.uint8))
        return yo, argmax
    return pool_fwd(y, ky, kx, sliding, "max", out=out, argmax=argmax)


def lrn_pool_bwd(x, dp, argmax, n, alpha, beta, k, ky, kx, sliding,
                 aux=None, aux_act=0, out=None):
    """lrn_bwd(x, pool_bwd(dp)) [* f'(aux)] without materialising the pool
    gradient."""
    sx, sy = sliding
    N, H, W, C = x.shape
    _, OH, OW, _ = dp.shape
    aux_act = act_code(aux_act)
    if out is None:
        out = torch.empty_like(x)
    if _gpu(x):
        ch = _n_chunks(N, H * W * C) if argmax.dtype == torch.uint8 else None
        if ch:
            for n0, n1 in ch:
                lrn_pool_bwd(x[n0:n1], dp[n0:n1], argmax[n0:n1], n, alpha,
                             beta, k, ky, kx, sliding, aux=_sl(aux, n0, n1),
                             aux_act=aux_act, out=out[n0:n1])
            return out
        if argmax.dtype == torch.uint8:
            _lib_call("hvk_lrn_pool_bwd_u8", _p(x), _p(dp), _p(argmax),
                      _p(out), N, H, W, C, OH, OW, n, float(alpha),
                      float(beta), float(k), _p(aux), aux_act, _s(x))
            return out
        _lib_call("hvk_lrn_pool_bwd", _p(x), _p(dp), _p(argmax), _p(out), N,
                  H, W, C, OH, OW, sy, sx, n, float(alpha), float(beta),
                  float(k), _p(aux), aux_act, _s(x))
        return out
    if argmax.dtype == torch.uint8:
        argmax = window_index_to_offsets(argmax, tuple(x.shape), ky, kx,
                                         sliding)
    g = pool_bwd(dp.float(), argmax, tuple(x.shape), ky, kx, sliding, "max")
    return lrn_bwd(x, g, n, alpha, beta, k, aux=aux, aux_act=aux_act,
                   out=out)


# --------------------------------------------------------------- evaluators
def softmax_ce(logits, labels, *, scale=None, err=None, probs=None,
               max_idx=None, metrics=None, confusion=None):
    """Fused softmax + cross-entropy gradient + error counting.

    err = (softmax(logits) - onehot(labels)) * scale (rows with label < 0 get
    0); metrics (float32[3]) += [n_err, sum CE loss, n_valid]."""
    B, C = logits.shape
    if scale is None:
        scale = 1.0 / B
    if _gpu(logits):
        _lib_call("hvk_softmax_ce", _p(logits), DT[logits.dtype], B, C,
                  _p(labels), float(scale), _p(err),
                  0 if err is None else DT[err.dtype], _p(probs), _p(max_idx),
                  _p(metrics), _p(confusion), _s(logits))
        return err
    lf = logits.float()
    p = torch.softmax(lf, 1)
    lab = labels.long() if labels is not None else torch.full(
        (B,), -1, dtype=torch.long)
    valid = lab >= 0
    if probs is not None:
        probs.copy_(p)
    if max_idx is not None:
        max_idx.copy_(lf.argmax(1).to(max_idx.dtype))
    if err is not None:
        oh = torch.zeros_like(p)
        oh[valid, lab[valid]] = 1.0
        e = (p - oh) * scale
        e[~valid] = 0
        err.copy_(e.to(err.dtype))
    if metrics is not None and valid.any():
        am = lf.argmax(1)
        pl = p[valid, lab[valid]].clamp(min=1e-30)
        metrics[0] += (am[valid] != lab[valid]).sum().float()
        metrics[1] += -torch.log(pl).sum()
        metrics[2] += valid.sum().float()
        if confusion is not None:
            for a, b in zip(am[valid].tolist(), lab[valid].tolist()):
                confusion[a, b] += 1
    return err


def mse(y, target, *, scale=1.0, err=None, mse_out=None, metrics=None,
        valid_rows=None):
    B = y.shape[0]
    D = y.numel() // B
    valid_rows = B if valid_rows is None else valid_rows
    if _gpu(y):
        _lib_call("hvk_mse", _p(y), DT[y.dtype], _p(target), DT[target.dtype],
                  B, D, float(scale), _p(err),
                  0 if err is None else DT[err.dtype], _p(mse_out),
                  _p(metrics), int(valid_rows), _s(y))
        return err
    d = y.float().reshape(B, D) - target.float().reshape(B, D)
    d[valid_rows:] = 0
    if err is not None:
        err.copy_((d * scale).reshape(err.shape).to(err.dtype))
    m = (d * d).mean(1)
    if mse_out is not None:
        mse_out.copy_(m)
    if metrics is not None:
        metrics[0] += m[:valid_rows].sum()
        metrics[1] += m[:valid_rows].sqrt().sum()
        metrics[2] += valid_rows
    return err


# --------------------------------------------------------------- optimizer
_SEG_CACHE = {}
_SEG_CACHE_MAX = 64


def _pack_sgd_segs(segs):
    return b"".join(struct.pack("<qqffff", int(b), int(e), float(lr),
                                float(d), float(l1), float(m))
                    for b, e, lr, d, l1, m in segs)


def _pack_solver_segs(segs):
    return b"".join(struct.pack(
        "<qqffffifff", int(b), int(e), float(lr), float(d), float(l1),
        float(m), int(mode), float(eps), float(rho), 0.0)
        for b, e, lr, d, l1, m, mode, eps, rho in segs)


def _segs_tensor(raw, device):
    """Device copy of a packed segment table, from a BOUNDED cache (one-off
    callers; a training loop whose learning rates move every step uses a
    :class:`SegmentTable` instead)."""
    key = (raw, str(device))
    t = _SEG_CACHE.get(key)
    if t is None:
        t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        if len(_SEG_CACHE) >= _SEG_CACHE_MAX:
            _SEG_CACHE.pop(next(iter(_SEG_CACHE)))
        _SEG_CACHE[key] = t
    return t


class SegmentTable(object):
    """One persistent device buffer holding a packed segment table, updated
    IN PLACE when the table changes (an LR policy such as ``exp`` changes it
    every step).  The device address never moves - a captured HIP graph of
    the train step keeps reading the current rates - and no device memory is
    allocated per step.  Host staging goes through two pinned buffers, each
    reused only after its previous stream-ordered copy has completed."""

    def __init__(self, device):
        self.device = device
        self.dev = None
        self._raw = None
        self._pinned = [None, None]
        self._events = [None, None]
        self._slot = 0

    def update(self, raw):
        if raw == self._raw and self.dev is not None:
            return self.dev
        n = len(raw)
        gpu = self.device.type == "cuda"
        if self.dev is None or self.dev.numel() < n:
            self.dev = torch.zeros(max(n, 64), dtype=torch.uint8,
                                   device=self.device)
            self._pinned = [None, None]
        if not gpu:
            self.dev[:n].copy_(torch.frombuffer(bytearray(raw),
                                                dtype=torch.uint8))
        else:
            i = self._slot
            self._slot ^= 1
            if self._events[i] is not None:
                self._events[i].synchronize()
            if self._pinned[i] is None or self._pinned[i].numel() < n:
                self._pinned[i] = torch.empty(self.dev.numel(),
                                              dtype=torch.uint8,
                                              pin_memory=True)
            self._pinned[i][:n].copy_(torch.frombuffer(bytearray(raw),
                                                       dtype=torch.uint8))
            self.dev[:n].copy_(self._pinned[i][:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[i] = ev
        self._raw = raw
        return self.dev


def _zero_from(zero_grad, n):
    """Offset from which an update clears the gradients: True -> 0 (all),
    False / None -> n (none), an int -> that offset (the split-K tail)."""
    if zero_grad is None or zero_grad is False:
        return n
    if zero_grad is True:
        return 0
    return max(0, min(int(zero_grad), n))


def sgd_update(w, grad, mom, segs, w_lp=None, gscale=1.0, zero_grad=False,
               table=None, max_blocks=None):
    """Fused multi-segment SGD (flat float32 buffers).

    segs: [(begin, end, lr, weights_decay, l1_vs_l2, gradient_moment)]
      g = grad*gscale + decay*((1-l1)*w + l1*sign(w));  v = moment*v - lr*g;
      w += v;  w_lp = bfloat16(w)
    zero_grad: True clears the whole gradient after reading it, an int
    offset clears only grad[offset:] (see :func:`_zero_from`).
    table: optional :class:`SegmentTable` the packed segments are kept in.
    max_blocks: cap on the GPU grid (a side-stream update next to compute)."""
    n = w.numel()
    zf = _zero_from(zero_grad, n)
    if _gpu(w):
        raw = _pack_sgd_segs(segs)
        st = table.update(raw) if table is not None else \
            _segs_tensor(raw, w.device)
        if mom is not None and max_blocks:
            fn = getattr(_lib.lib(), "hvk_sgd4_grid")
            if fn(_p(w), _p(grad), _p(mom), _p(w_lp), _p(st), len(segs), n,
                  float(gscale), zf, int(max_blocks), _s(w)) == 0:
                return w
        fn = getattr(_lib.lib(), "hvk_sgd4")
        if mom is not None and fn(_p(w), _p(grad), _p(mom), _p(w_lp),
                                  _p(st), len(segs), n, float(gscale),
                                  zf, _s(w)) == 0:
            return w
        _lib_call("hvk_sgd", _p(w), _p(grad), _p(mom), _p(w_lp), _p(st),
                  len(segs), n, float(gscale), _s(w))
        if zf < n:
            grad[zf:].zero_()
        return w
    for b, e, lr, d, l1, m in segs:
        ws = w[b:e]
        g = grad[b:e] * gscale
        if d:
            g = g + d * ((1 - l1) * ws + l1 * torch.sign(ws))
        v = -lr * g
        if mom is not None:
            v = v + m * mom[b:e]
            mom[b:e] = v
        ws += v
    if w_lp is not None:
        w_lp.copy_(w.to(w_lp.dtype))
    if zf < n:
        grad[zf:].zero_()
    return w


SOLVERS = {"momentum": 0, "adagrad": 1, "adadelta": 2, "rprop": 3}


def solver_update(w, grad, s1, s2, segs, w_lp=None, gscale=1.0,
                  zero_grad=False, table=None):
    """Fused multi-segment update with a solver per segment.

    segs: [(begin, end, lr, decay, l1_vs_l2, moment, mode, eps, rho)], modes
    in :data:`SOLVERS` (csrc/kernels/elementwise.hip ``solver_kernel``)."""
    n = w.numel()
    zf = _zero_from(zero_grad, n)
    if _gpu(w):
        raw = _pack_solver_segs(segs)
        st = table.update(raw) if table is not None else \
            _segs_tensor(raw, w.device)
        _lib_call("hvk_solver", _p(w), _p(grad), _p(s1), _p(s2), _p(w_lp),
                  _p(st), len(segs), n, float(gscale), zf, _s(w))
        return w
    for b, e, lr, d, l1, m, mode, eps, rho in segs:
        ws = w[b:e]
        g = grad[b:e] * gscale
        if d:
            g = g + d * ((1 - l1) * ws + l1 * torch.sign(ws))
        a = s1[b:e]
        if mode == 1:
            a += g * g
            ws -= lr * g / (a.sqrt() + eps)
        elif mode == 2:
            c = s2[b:e]
            a.mul_(rho).add_((1 - rho) * g * g)
            dd = g * (c + eps).sqrt() / (a + eps).sqrt()
            c.mul_(rho).add_((1 - rho) * dd * dd)
            ws -= lr * dd
        elif mode == 3:
            prev = s2[b:e]
            step = torch.where(a > 0, a, torch.full_like(a, lr))
            same = prev * g > 0
            flip = prev * g < 0
            step = torch.where(same, (step * 1.2).clamp(max=50.0), step)
            step = torch.where(flip, (step * 0.5).clamp(min=1e-6), step)
            g = torch.where(flip, torch.zeros_like(g), g)
            ws -= torch.sign(g) * step
            a.copy_(step)
            prev.copy_(g)
        else:
            a.mul_(m).sub_(lr * g)
            ws += a
    if w_lp is not None:
        w_lp.copy_(w.to(w_lp.dtype))
    if zf < n:
        grad[zf:].zero_()
    return w


# ---------------------------------------------------------------- dropout
def _hash32(i, seed):
    M = 0xFFFFFFFF
    x = i ^ ((seed * 0x9E3779B9) & M)
    x ^= x >> 16
    x = (x * 0x7feb352d) & M
    x ^= x >> 15
    x = (x * 0x846ca68b) & M
    x ^= x >> 16
    return x


def dropout_mask_ref(n, seed, p, base=0):
    i = (torch.arange(n, dtype=torch.int64) + int(base)) & 0xFFFFFFFF
    h = _hash32(i, int(seed) & 0xFFFFFFFF)
    thresh = min(0xFFFFFFFF, int(p * 4294967296.0))
    return h >= thresh


def dropout(x, p, seed, out=None, seed_dev=None, base=0):
    """y = x * keep / (1-p) with a counter-based mask (same seed -> same mask:
    the backward pass calls this on dy).  ``seed_dev``: a 1-element int32
    device tensor holding the seed instead (graph-safe, see
    :func:`seed_advance`); ``seed`` is then ignored.  ``base``: mask index
    of element 0 (a data-parallel rank's offset in the global minibatch)."""
    if out is None:
        out = torch.empty_like(x)
    if seed_dev is not None and not _gpu(x):
        seed = int(seed_dev.reshape(-1)[0]) & 0xFFFFFFFF
    if _gpu(x):
        if seed_dev is not None:
            if base:
                _lib_call("hvk_dropout_dev_at", _p(x), DT[x.dtype], _p(out),
                          DT[out.dtype], x.numel(), _p(seed_dev), float(p),
                          int(base), _s(x))
                return out
            _lib_call("hvk_dropout_dev", _p(x), DT[x.dtype], _p(out),
                      DT[out.dtype], x.numel(), _p(seed_dev), float(p), None,
                      _s(x))
            return out
        if base:
            raise ValueError("dropout: base needs the device seed path")
        _lib_call("hvk_dropout", _p(x), DT[x.dtype], _p(out), DT[out.dtype],
                  x.numel(), int(seed) & 0xFFFFFFFF, float(p), None, _s(x))
        return out
    keep = dropout_mask_ref(x.numel(), seed, p, base).view(x.shape)
    scale = 1.0 / (1.0 - p) if p < 1 else 0.0
    out.copy_((x.float() * keep * scale).to(out.dtype))
    return out


def seed_advance_ref(seed):
    """Host mirror of hvk_seed_advance: seed <- hash32(seed + 1)."""
    i = torch.tensor([(int(seed) + 1) & 0xFFFFFFFF], dtype=torch.int64)
    return int(_hash32(i, 0x2545F491)[0])


def seed_advance(seed_dev):
    """Advance a device-resident dropout seed (int32 [1]) in place - a
    stream-ordered kernel, so a captured step draws a new mask every
    replay."""
    if _gpu(seed_dev):
        _lib_call("hvk_seed_advance", _p(seed_dev), _s(seed_dev))
        return seed_dev
    v = seed_advance_ref(int(seed_dev.reshape(-1)[0]) & 0xFFFFFFFF)
    seed_dev.fill_(v - (1 << 32) if v >= (1 << 31) else v)
    return seed_dev


def trace_marker(tag=0, stream=None):
    """Launch the empty marker kernel on ``stream`` (default: the current
    one; bench.py --mark-steps passes the workflow's compute stream) to
    bracket the timed steps in a rocprofv3 kernel trace."""
    if torch.cuda.is_available():
        st = stream if stream is not None else torch.cuda.current_stream()
        _lib_call("hvk_trace_marker", int(tag), st.cuda_stream)


# --------------------------------------------------------------------- RNG
def xorshift1024star(states, rounds, out=None):
    """states: int64 [n,16] (raw uint64 bits, updated in place); returns int64
    [rounds*16*n] laid out out[round*16*n + i*n + id]."""
    n = states.shape[0]
    if out is None:
        out = torch.empty(rounds * 16 * n, dtype=torch.int64,
                          device=states.device)
    if _gpu(states):
        _lib_call("hvk_xorshift1024star", _p(states), n, int(rounds), _p(out),
                  _s(states))
        return out
    from veles_amd.prng.random_generator import xorshift1024star as ref
    s = states.numpy().view("uint64")
    r = ref(s, rounds)
    out.copy_(torch.from_numpy(r.view("int64")))
    return out


def xorshift128plus(states, out=None):
    n = states.shape[0]
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=states.device)
    if _gpu(states):
        _lib_call("hvk_xorshift128plus", _p(states), n, _p(out), _s(states))
        return out
    from veles_amd.prng.random_generator import xorshift128plus as ref
    r = ref(states.numpy().view("uint64"), 1)
    out.copy_(torch.from_numpy(r.view("int64")))
    return out


# ------------------------------------------------------------- data moving
def join(inputs, out=None):
    """Feature-wise concatenation of [B, n_i] inputs (InputJoiner)."""
    B = inputs[0].shape[0]
    lens = [t.numel() // B for t in inputs]
    if out is None:
        out = torch.empty(B, sum(lens), dtype=inputs[0].dtype,
                          device=inputs[0].device)
    if _gpu(out) and len(inputs) <= 16:
        import ctypes
        arr = (ctypes.c_void_p * len(inputs))(*[t.data_ptr() for t in inputs])
        la = (ctypes.c_int * len(inputs))(*lens)
        _lib_call("hvk_join", ctypes.cast(arr, ctypes.c_void_p),
                  ctypes.cast(la, ctypes.c_void_p), len(inputs),
                  DT[out.dtype], _p(out), B, _s(out))
        return out
    out.copy_(torch.cat([t.reshape(B, -1).to(out.dtype) for t in inputs], 1))
    return out


def cast(x, dtype, scale=1.0, out=None):
    if out is None:
        out = torch.empty(x.shape, dtype=dtype, device=x.device)
    if _gpu(x) and x.dtype in DT and out.dtype in DT:
        _lib_call("hvk_cast", _p(x), DT[x.dtype], _p(out), DT[out.dtype],
                  x.numel(), float(scale), _s(x))
        return out
    out.copy_((x.float() * scale).to(dtype))
    return out


def fill_minibatch(src, shuffled, start, count, dst, *, mean=None,
                   rdisp=None, labels=None, labels_out=None, idx_out=None):
    """Gather a minibatch: dst[i] = (src[shuffled[start+i]] - mean) * rdisp
    for i < count, zeros after; labels/indices gathered (-1 padding)."""
    max_mb = dst.shape[0]
    sample = src.numel() // src.shape[0]
    if _gpu(dst):
        _lib_call("hvk_fill_minibatch", _p(src), DT[src.dtype], _p(shuffled),
                  int(start), int(count), max_mb, sample, _p(mean), _p(rdisp),
                  _p(dst), DT[dst.dtype], _p(labels), _p(labels_out),
                  _p(idx_out), _s(dst))
        return dst
    idx = shuffled[start:start + count].long()
    v = src.reshape(src.shape[0], -1)[idx].float()
    if mean is not None:
        v = v - mean.reshape(1, -1).float()
    if rdisp is not None:
        v = v * rdisp.reshape(1, -1).float()
    d = dst.view(max_mb, -1)
    d[:count] = v.to(dst.dtype)
    d[count:] = 0
    if labels_out is not None:
        labels_out[:count] = labels[idx] if labels is not None else -1
        labels_out[count:] = -1
    if idx_out is not None:
        idx_out[:count] = idx.to(idx_out.dtype)
        idx_out[count:] = -1
    return dst


def image_batch_ref(src, idx, params, Ho, Wo, sobel=False, mean=None,
                    rdisp=None, bg=None, bgcolor=None):
    """Torch (f32) reference of hvk_image_batch: crop (cy, cx) -> mirror ->
    rotate (bilinear, cv2 centre and angle convention) -> optional Sobel
    magnitude channel -> (v - mean) * rdisp.  src uint8 [N][Hs][Ws][C];
    params [B][6] = (cy, cx, cos, sin, mirror, -)."""
    N, Hs, Ws, C = src.shape
    B = idx.shape[0]
    dev = src.device
    p = params.float()
    oy = torch.arange(Ho, device=dev, dtype=torch.float32).view(1, Ho, 1)
    ox = torch.arange(Wo, device=dev, dtype=torch.float32).view(1, 1, Wo)

    def sample(yy, xx):
        cy, cx = p[:, 0].view(B, 1, 1), p[:, 1].view(B, 1, 1)
        ct, st = p[:, 2].view(B, 1, 1), p[:, 3].view(B, 1, 1)
        mir = (p[:, 4] != 0).view(B, 1, 1)
        ccx, ccy = float(Wo // 2), float(Ho // 2)
        dx, dy = xx - ccx, yy - ccy
        sx = ccx + ct * dx - st * dy
        sy = ccy + st * dx + ct * dy
        sx = torch.where(mir, (Wo - 1) - sx, sx)
        x0, y0 = torch.floor(sx), torch.floor(sy)
        axx, ayy = sx - x0, sy - y0
        v = torch.zeros(B, Ho, Wo, C, device=dev)
        can = src[idx.clamp_min(0).long()].float()   # [B,Hs,Ws,C]
        for t in range(4):
            ty, tx = t >> 1, t & 1
            w = (ayy if ty else 1 - ayy) * (axx if tx else 1 - axx)
            yi, xi = (y0 + ty).long(), (x0 + tx).long()
            inb = (yi >= 0) & (yi < Ho) & (xi >= 0) & (xi < Wo) & \
                (cy.long() + yi < Hs) & (cx.long() + xi < Ws)
            gy = (cy.long() + yi).clamp(0, Hs - 1)
            gx = (cx.long() + xi).clamp(0, Ws - 1)
            bi = torch.arange(B, device=dev).view(B, 1, 1).expand_as(gy)
            val = can[bi, gy, gx]                      # [B,Ho,Wo,C]
            if bg is not None:
                bgv = bg.float()[yi.clamp(0, Ho - 1), xi.clamp(0, Wo - 1)]
            elif bgcolor is not None:
                bgv = bgcolor.float().view(1, 1, 1, C).expand_as(val)
            else:
                bgv = torch.zeros_like(val)
            val = torch.where(inb.unsqueeze(-1), val, bgv)
            v = v + w.unsqueeze(-1) * val
        return v

    yy = oy.expand(B, Ho, Wo)
    xx = ox.expand(B, Ho, Wo)
    v = sample(yy, xx)
    if sobel:
        def gray(a):
            return (0.299 * a[..., 0] + 0.587 * a[..., 1] + 0.114 * a[..., 2]
                    if C >= 3 else a[..., 0])
        g = {}
        for t in range(9):
            ry = (yy + (t // 3 - 1)).clamp(0, Ho - 1)
            rx = (xx + (t % 3 - 1)).clamp(0, Wo - 1)
            g[t] = gray(sample(ry, rx))
        gx = (g[2] + 2 * g[5] + g[8]) - (g[0] + 2 * g[3] + g[6])
        gy = (g[6] + 2 * g[7] + g[8]) - (g[0] + 2 * g[1] + g[2])
        v = torch.cat([v, torch.sqrt(gx * gx + gy * gy).unsqueeze(-1)], -1)
    if mean is not None:
        v = v - mean.float().view(1, Ho, Wo, -1)
    if rdisp is not None:
        v = v * rdisp.float().view(1, Ho, Wo, -1)
    return v * (idx >= 0).float().view(B, 1, 1, 1)


def image_batch(src, idx, params, out, sobel=False, mean=None, rdisp=None,
                bg=None, bgcolor=None):
    """Augmented, normalised image minibatch from uint8 canvases (the image
    loaders' device path, hvk_image_batch): out [B][Ho][Wo][C + sobel]."""
    B, Ho, Wo = out.shape[0], out.shape[1], out.shape[2]
    N, Hs, Ws, C = src.shape
    if _gpu(out):
        _lib_call("hvk_image_batch", _p(src), Hs * Ws * C, Hs, Ws, C,
                  _p(idx), _p(params), B, Ho, Wo, 1 if sobel else 0,
                  _p(mean), _p(rdisp), _p(bg), _p(bgcolor), _p(out), _s(out))
        return out
    out.copy_(image_batch_ref(src, idx, params, Ho, Wo, sobel, mean, rdisp,
                              bg, bgcolor).to(out.dtype))
    return out


def mean_disp_normalize(x, mean, rdisp, out=None, out_dtype=None):
    """out = (float(x) - mean) * rdisp, mean/rdisp broadcast per sample."""
    if out is None:
        out = torch.empty(x.shape, dtype=out_dtype or torch.float32,
                          device=x.device)
    sample = mean.numel()
    if _gpu(x):
        _lib_call("hvk_mean_disp_normalize", _p(x), DT[x.dtype], _p(mean),
                  _p(rdisp), _p(out), DT[out.dtype], x.numel(), sample, _s(x))
        return out
    v = (x.float().reshape(-1, sample) - mean.reshape(1, -1).float()) * \
        rdisp.reshape(1, -1).float()
    out.copy_(v.reshape(out.shape).to(out.dtype))
    return out
