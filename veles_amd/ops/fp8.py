"""FP8 compute path (OCP e4m3 activations / weights, e5m2 gradients) with
per-tensor delayed scaling (BASELINE config 5).

GPU: ``csrc/kernels/gemm_fp8.hip`` - quantizers that record the tensor's amax
on the device, and MFMA kernels on ``v_mfma_scale_f32_16x16x128_f8f6f4``
(2x the bf16 rate) for the conv forward / backward-data and the
fully-connected forward GEMMs.  Weight gradients and the fully-connected
backward-data GEMM stay bf16 (docs/OPS.md §FP8).  CPU: the same quantization
in PyTorch (``float8_e4m3fn`` / ``float8_e5m2`` casts) followed by the
float32 reference op, so CPU tests pin the GPU numerics up to accumulation
order.

Scaling recipe (per tensor, no host synchronisation):

* every ``Scaler`` owns a row ``[history(HIST), current_amax]`` of a
  device-resident state block;
* ``scale = fmax / 2**margin / max(history)`` (1 while the history is empty)
  is recomputed inside every kernel that needs it from that row, so the
  quantizer and the GEMM that consumes its output always agree;
* quantizers ``atomicMax`` the unscaled amax into ``current``; once per step
  ``roll()`` moves ``current`` into the history ring (one tiny kernel for all
  scalers of the device);
* the first use of a scaler primes its history from the tensor itself
  (one amax pass), so step 0 is "current scaling".
"""
from __future__ import annotations

import torch

from veles_amd.ops import _lib

__all__ = ["E4M3", "E5M2", "Scaler", "registry", "quantize", "gemm",
           "save_scalers", "restore_scaler",
           "conv_fwd", "conv_dgrad", "conv_wgrad", "permute_for_dgrad",
           "transpose", "dequantize", "HIST"]

E4M3, E5M2 = 0, 1
HIST = 16
FMAX = {E4M3: 448.0, E5M2: 57344.0}
TORCH_DT = {E4M3: torch.float8_e4m3fn, E5M2: torch.float8_e5m2}
_CHUNK = 256
SHARDS = 32


def _s(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _call(name, *args):
    _lib.check(getattr(_lib.lib(), name)(*args), name)


class _Registry(object):
    """All scaler states of one device, in fixed [CHUNK][HIST + 1] blocks."""

    def __init__(self, device):
        self.device = device
        self.blocks = []
        # per scaler: 32 amax shards, 32 floats (128 B) apart, that the
        # fused-quantising fp8 epilogues atomicMax into (one per workgroup);
        # the roll folds them into the current amax
        self.shard_blocks = []
        self.used = 0
        self.step = 0
        self.step_dev = None  # device mirror of ``step`` (GPU roll)
        # multi-rank DataParallel whose ranks share the amaxes (set by the
        # parameter store with engine.dp.fp8_amax_sync): primes are reduced
        self.dp = None

    def allocate(self):
        """(state row [HIST + 1], shard row [1024]) of a new scaler."""
        i = self.used
        if i // _CHUNK >= len(self.blocks):
            self.blocks.append(torch.zeros(_CHUNK, HIST + 1,
                                           dtype=torch.float32,
                                           device=self.device))
            self.shard_blocks.append(torch.zeros(_CHUNK, SHARDS * 32,
                                                 dtype=torch.float32,
                                                 device=self.device))
        self.used += 1
        return (self.blocks[i // _CHUNK][i % _CHUNK],
                self.shard_blocks[i // _CHUNK][i % _CHUNK])

    def roll(self, dp=None):
        """End of step: current amax -> history slot; current = 0.  On the
        GPU the slot index comes from a device step counter advanced in the
        same stream, so a captured HIP graph of the step rolls correctly on
        every replay.

        ``dp`` (a multi-rank DataParallel): the current amaxes are first
        all-reduced with MAX over the ranks, so every rank scales with the
        amax of the GLOBAL minibatch - the scales, and so the quantisation,
        of a 1-rank run over the same global batch (one small stream-ordered
        collective per step: the scalers' state and shard rows)."""
        if dp is not None and getattr(dp, "multi", False):
            import torch.distributed as dist
            for bi, blk in enumerate(self.blocks):
                count = min(_CHUNK, self.used - bi * _CHUNK)
                if count <= 0:
                    break
                dist.all_reduce(blk[:count], op=dist.ReduceOp.MAX)
                dist.all_reduce(self.shard_blocks[bi][:count],
                                op=dist.ReduceOp.MAX)
        idx = self.step % HIST
        gpu_step = None
        for bi, blk in enumerate(self.blocks):
            count = min(_CHUNK, self.used - bi * _CHUNK)
            if count <= 0:
                break
            if blk.is_cuda:
                if gpu_step is None:
                    if self.step_dev is None:
                        self.step_dev = torch.full(
                            (1,), self.step, dtype=torch.int32,
                            device=blk.device)
                    gpu_step = self.step_dev
                _call("hvk_fp8_roll_dev", blk.data_ptr(), count, HIST,
                      gpu_step.data_ptr(),
                      self.shard_blocks[bi].data_ptr(), _s(blk))
            else:
                sh = self.shard_blocks[bi][:count].view(count, SHARDS, 32)
                blk[:count, HIST] = torch.maximum(blk[:count, HIST],
                                                  sh[:, :, 0].max(1).values)
                sh.zero_()
                cur = blk[:count, HIST]
                keep = cur > 0
                blk[:count, idx] = torch.where(keep, cur, blk[:count, idx])
                blk[:count, HIST] = 0
        if gpu_step is not None:
            gpu_step.add_(1)
        self.step += 1

    def set_step(self, step):
        """Restore the roll counter (the history slot the next roll writes)
        from a snapshot, host and device mirror alike."""
        self.step = int(step)
        if self.step_dev is not None:
            self.step_dev.fill_(self.step)


_REGISTRIES = {}


def release_dp(dp):
    """Forget ``dp`` in every registry (DataParallel.shutdown): a later
    workflow in the same process must not prime through a destroyed
    process group."""
    for r in _REGISTRIES.values():
        if r.dp is dp:
            r.dp = None


def registry(device):
    device = torch.device(device)
    key = (device.type, device.index)
    r = _REGISTRIES.get(key)
    if r is None:
        r = _REGISTRIES[key] = _Registry(device)
    return r


class Scaler(object):
    """Per-tensor delayed scaling state (one row of the device registry)."""

    def __init__(self, device, fmt=E4M3, margin=0):
        self.fmt = fmt
        self.margin = margin
        self.registry = registry(device)
        self.state, self.shard = self.registry.allocate()
        self.primed = False

    @property
    def fmax_eff(self):
        return FMAX[self.fmt] / (2.0 ** self.margin)

    def scale(self):
        """Current scale (host read: tests / diagnostics only)."""
        m = float(self.state[:HIST].max())
        return self.fmax_eff / m if m > 0 else 1.0

    def _scale_t(self):
        m = self.state[:HIST].max()
        return torch.where(m > 0, self.fmax_eff / m, torch.ones_like(m))

    def state_dict(self):
        """Host copy of the scaling state for a snapshot: amax history and
        current amax, the epilogues' amax shards, the primed flag and the
        registry's roll counter (exact resume)."""
        if self.state.is_cuda:
            torch.cuda.synchronize(self.state.device)
        return {"fmt": self.fmt, "margin": self.margin,
                "primed": bool(self.primed),
                "state": self.state.detach().cpu().numpy().copy(),
                "shard": self.shard.detach().cpu().numpy().copy(),
                "step": int(self.registry.step)}

    def load_state_dict(self, d):
        if int(d["fmt"]) != self.fmt:
            raise ValueError("fp8 scaler snapshot of format %s restored into "
                             "a %s scaler" % (d["fmt"], self.fmt))
        self.margin = d.get("margin", self.margin)
        self.primed = bool(d["primed"])
        self.state.copy_(torch.as_tensor(d["state"]))
        self.shard.copy_(torch.as_tensor(d["shard"]))
        self.registry.set_step(d["step"])

    def prime(self, x):
        if self.primed:
            return
        self.primed = True
        st = self.state
        if x.is_cuda:
            xf = x if x.dtype in (torch.float32, torch.bfloat16) else x.float()
            xf = xf.contiguous()
            _call("hvk_fp8_amax", xf.data_ptr(),
                  int(xf.dtype == torch.float32), xf.numel(), st.data_ptr(),
                  HIST, _s(xf))
            _call("hvk_fp8_roll", st.data_ptr(), 1, HIST, 0, 1, None, _s(xf))
        else:
            st[:HIST] = x.float().abs().max()
            st[HIST] = 0
        dp = self.registry.dp
        import torch.distributed as dist
        if dp is not None and getattr(dp, "multi", False) and \
                dist.is_initialized():
            # the first scale of every rank from the GLOBAL batch's amax
            dist.all_reduce(st, op=dist.ReduceOp.MAX)


def save_scalers(unit, names):
    """``__getstate__`` helper: the unit's live scalers (attributes
    ``names``, transient ``*_``) as host dicts in the pickled
    ``fp8_saved``."""
    saved = {n: getattr(unit, n).state_dict() for n in names
             if getattr(unit, n, None) is not None}
    if saved or getattr(unit, "fp8_saved", None) is None:
        unit.fp8_saved = saved or None


def restore_scaler(unit, name):
    """Load the snapshot state of scaler ``name`` (just created by the
    restored unit) once: the resumed run scales exactly as the
    uninterrupted one would have."""
    saved = getattr(unit, "fp8_saved", None)
    if saved and name in saved and getattr(unit, name, None) is not None:
        getattr(unit, name).load_state_dict(saved.pop(name))


def quantize(x, scaler, out=None, record=True):
    """fp8 copy of ``x`` (bf16 / f32) at the scaler's current scale; records
    amax|x| for the next roll.  Returns a ``float8_e4m3fn``/``e5m2`` tensor."""
    scaler.prime(x)
    dt = TORCH_DT[scaler.fmt]
    if out is None or out.shape != x.shape or out.dtype != dt or \
            out.device != x.device:
        out = torch.empty(x.shape, dtype=dt, device=x.device)
    if x.is_cuda:
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        x = x.contiguous()
        _call("hvk_fp8_quant", x.data_ptr(), int(x.dtype == torch.float32),
              x.numel(), out.data_ptr(), scaler.fmt, scaler.state.data_ptr(),
              HIST, float(scaler.fmax_eff), int(bool(record)), _s(x))
        return out
    xf = x.float()
    lim = FMAX[scaler.fmt]
    q = (xf * scaler._scale_t()).clamp(-lim, lim).to(dt)
    out.copy_(q)
    if record:
        st = scaler.state
        st[HIST] = torch.maximum(st[HIST], xf.abs().max())
    return out


def dequantize(q, scaler):
    return q.float() / scaler._scale_t()


def _u8(t):
    return t.view(torch.uint8)


def transpose(w8):
    """[R][C] fp8 -> contiguous [C][R]."""
    return _u8(w8).t().contiguous().view(w8.dtype)


def permute_for_dgrad(w8, groups):
    """[OC][KH][KW][Cg] -> [g][Cg][KH][KW][OCg] (dense K-major dgrad B)."""
    OC, KH, KW, Cg = w8.shape
    OCg = OC // groups
    u = _u8(w8).view(groups, OCg, KH, KW, Cg).permute(0, 4, 2, 3, 1)
    return u.contiguous().view(w8.dtype)


def gemm(a8, sa, b8, sb, bias=None, act=0, aux=None, aux_act=0, out=None):
    """out[M][N] (bf16 on GPU) = act(deq(a8) @ deq(b8)^T + bias) * f'(aux)."""
    from veles_amd import ops
    M, K = a8.shape
    N = b8.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16 if a8.is_cuda else
                          torch.float32, device=a8.device)
    if a8.is_cuda:
        _call("hvk_gemm_fp8", M, N, K, a8.data_ptr(), a8.stride(0), sa.fmt,
              b8.data_ptr(), b8.stride(0), sb.fmt, out.data_ptr(),
              out.stride(0), ops._p(bias), ops.act_code(act), ops._p(aux),
              0 if aux is None else aux.stride(0), ops.act_code(aux_act),
              sa.state.data_ptr(), sb.state.data_ptr(), HIST,
              float(sa.fmax_eff), float(sb.fmax_eff), _s(a8))
        return out
    return ops.gemm(dequantize(a8, sa), dequantize(b8, sb), trans_b=True,
                    bias=bias, act=act, aux=aux, aux_act=aux_act, out=out)


def fp8_conv_ok(C, OC, groups, KH=1, KW=1):
    """Geometry the fp8 implicit-GEMM loaders take: 16-B channel chunks, and
    kernels of at most 32 taps per axis (the tap bit masks of the branch-free
    forward addressing, conv_geom.h)."""
    return C % 16 == 0 and (C // groups) % 16 == 0 and OC % 16 == 0 and \
        (OC // groups) % 16 == 0 and KH <= 32 and KW <= 32


def fp8_conv_pays(C, OH, OW):
    """Layers left on bf16 in an fp8 model because the bf16 kernels beat the
    fp8 ones there: 64 input channels at >= 200 x 200 outputs (VGG-16
    conv1_2).  Its fp8 forward (im2col T4, 256 x 64 tiles) took 3.0 ms and
    backward-data (128-row loop, K = 576) 3.56 ms at b512 against 2.46 /
    3.23 ms for the bf16 halo conv and GEMM, and its e4m3 input copy cost
    the bf16 conv1_1 epilogue 0.78 ms (profiles/r6/vgg16_b512_{float8,
    bfloat16}_step_r6w.md).  ``root.common.engine.fp8_all_convs = True``
    (or VELES_AMD_FP8_ALL_CONVS=1) keeps every eligible conv on fp8."""
    import os
    from veles_amd.utils.config import root, get
    if get(root.common.engine.fp8_all_convs, False) or \
            os.environ.get("VELES_AMD_FP8_ALL_CONVS", "0") not in ("", "0"):
        return True
    return not (C <= 64 and OH * OW >= 200 * 200)


def _q8_args(q8, qs):
    """Kernel arguments of a fused output quantisation (or none)."""
    if q8 is None:
        return [None, None, None, 1.0, 0]
    return [q8.data_ptr(), qs.state.data_ptr(), qs.shard.data_ptr(),
            float(qs.fmax_eff), qs.fmt]


def _q8_ref(y, q8, qs):
    """CPU model of the fused quantisation: q8 = quantize(y) - y as stored,
    exactly what the consumer would quantize (the GPU epilogue quantizes the
    bf16-rounded output it stores) - with the amax recorded in the scaler's
    first shard."""
    if q8 is None:
        return
    yb = y.float()
    lim = FMAX[qs.fmt]
    q8.copy_((yb * qs._scale_t()).clamp(-lim, lim).to(q8.dtype))
    qs.shard[0] = torch.maximum(qs.shard[0], yb.abs().max())


def conv_fwd(x8, sx, w8, sw, bias=None, sliding=(1, 1), padding=(0, 0, 0, 0),
             groups=1, act=0, out=None, q8=None, q8_scaler=None):
    """y (bf16 on GPU) = act(conv(deq(x8), deq(w8)) + bias).  ``q8`` /
    ``q8_scaler``: also write the fp8 copy of y the NEXT fp8 layer reads
    (its input scaler; the amax is recorded for the scaler's roll) from the
    same epilogue - no separate quantize pass."""
    from veles_amd import ops
    N, H, W, C = x8.shape
    OC, KH, KW, Cg = w8.shape
    sxx, syy = sliding
    pl, pt, pr, pb = padding
    OH, OW = ops.conv_out_size(H, W, KH, KW, sliding, padding)
    if out is None:
        out = torch.empty(N, OH, OW, OC, dtype=torch.bfloat16 if x8.is_cuda
                          else torch.float32, device=x8.device)
    if x8.is_cuda:
        # image chunks under the 32-bit buffer offsets (ops._image_chunks)
        for n0, n1 in ops._image_chunks(N, x8):
            qa = _q8_args(q8, q8_scaler)
            if q8 is not None:
                qa[0] += n0 * OH * OW * OC
            _call("hvk_conv_fwd_fp8", x8[n0:n1].data_ptr(), w8.data_ptr(),
                  ops._p(bias), out[n0:n1].data_ptr(), n1 - n0, H, W, C, OC,
                  KH, KW, syy, sxx, pt, pl, OH, OW, groups,
                  ops.act_code(act), sx.fmt, sw.fmt, sx.state.data_ptr(),
                  sw.state.data_ptr(), HIST, float(sx.fmax_eff),
                  float(sw.fmax_eff), *qa, _s(x8))
        return out
    y = ops.conv_fwd(dequantize(x8, sx), dequantize(w8, sw), bias, sliding,
                     padding, groups, act, out=out)
    _q8_ref(y, q8, q8_scaler)
    return y


def conv_dgrad(dy8, sdy, w8, sw, x_shape, sliding=(1, 1),
               padding=(0, 0, 0, 0), groups=1, aux=None, aux_act=0, out=None,
               wt8=None, q8=None, q8_scaler=None):
    """dx = conv^T(deq(dy8), deq(w8)) [* f'(aux)]; ``wt8`` is the
    ``permute_for_dgrad`` image of w8 (computed here when not given)."""
    from veles_amd import ops
    N, H, W, C = x_shape
    _, OH, OW, OC = dy8.shape
    _, KH, KW, Cg = w8.shape
    sxx, syy = sliding
    pl, pt, pr, pb = padding
    if out is None:
        out = torch.empty(N, H, W, C, dtype=torch.bfloat16 if dy8.is_cuda
                          else torch.float32, device=dy8.device)
    if dy8.is_cuda:
        if wt8 is None:
            wt8 = permute_for_dgrad(w8, groups)
        for n0, n1 in ops._image_chunks(N, dy8):
            qa = _q8_args(q8, q8_scaler)
            if q8 is not None:
                qa[0] += n0 * H * W * C
            _call("hvk_conv_dgrad_fp8", dy8[n0:n1].data_ptr(), wt8.data_ptr(),
                  out[n0:n1].data_ptr(), n1 - n0, H, W, C, OC, KH, KW, syy,
                  sxx, pt, pl, OH, OW, groups,
                  ops._p(None if aux is None else aux[n0:n1]),
                  ops.act_code(aux_act), sdy.fmt, sw.fmt,
                  sdy.state.data_ptr(), sw.state.data_ptr(), HIST,
                  float(sdy.fmax_eff), float(sw.fmax_eff), *qa, _s(dy8))
        return out
    dx = ops.conv_dgrad(dequantize(dy8, sdy), dequantize(w8, sw), x_shape,
                        sliding, padding, groups, aux=aux, aux_act=aux_act,
                        out=out)
    _q8_ref(dx, q8, q8_scaler)
    return dx


def _halo_wgrad8(x8, sx, dy8, sdy, dw, dbias, pt, pl, OH, OW, groups,
                 splits):
    """Stride-1 fp8 weight gradient on the halo kernel (csrc/kernels/
    wgrad_halo.hip wgrad_halo8_kernel) when the shape takes it; False
    leaves the call to hvk_conv_wgrad_fp8."""
    from veles_amd import ops
    # the kernel's LDS-DMA needs 16-B aligned operands: refuse here (the
    # launch would return -1, an error, after a plan that said yes)
    if not ops._HALO_WGRAD or not dw.is_contiguous() or \
            not x8.is_contiguous() or not dy8.is_contiguous() or \
            x8.data_ptr() % 16 or dy8.data_ptr() % 16:
        return False
    N, H, W, C = x8.shape
    OC = dy8.shape[3]
    KH, KW = dw.shape[1], dw.shape[2]
    fn = ops._lib.lib().hvk_conv_wgrad_halo_fp8
    geo = (N, H, W, C, OC, KH, KW, pt, pl, OH, OW, groups,
           int(splits) if splits else 0, sx.fmt, sdy.fmt,
           sx.state.data_ptr(), sdy.state.data_ptr(), HIST,
           float(sx.fmax_eff), float(sdy.fmax_eff), _s(x8))
    db = None if dbias is None else dbias.data_ptr()
    need = fn(x8.data_ptr(), dy8.data_ptr(), dw.data_ptr(), db, None, *geo)
    if need < 0:
        return False
    ws = ops._grow_ws("wgrad_halo_ws", int(need), torch.float32, x8.device)
    rc = fn(x8.data_ptr(), dy8.data_ptr(), dw.data_ptr(), db, ws.data_ptr(),
            *geo)
    ops._lib.check(int(rc), "hvk_conv_wgrad_halo_fp8")
    return True


def conv_wgrad(x8, sx, dy8, sdy, dw, sliding=(1, 1), padding=(0, 0, 0, 0),
               groups=1, splits=None, dbias=None):
    """dw (float32 [OC][KH][KW][C/g]) += conv weight gradient of deq(x8)
    (the layer's input copy) and deq(dy8) (its output-gradient copy), and
    ``dbias`` (float32 [OC]) += the pixel sums of deq(dy8): the e5m2 x e4m3
    MFMA kernel on the GPU (the bias from MFMAs against an all-ones operand),
    split over pixels with f32 atomics; the float32 op on dequantized
    operands on the CPU."""
    from veles_amd import ops
    N, H, W, C = x8.shape
    _, OH, OW, OC = dy8.shape
    _, KH, KW, Cg = dw.shape
    sxx, syy = sliding
    pl, pt, pr, pb = padding
    if x8.is_cuda:
        # a sum over pixels: image chunks (32-bit buffer offsets) accumulate
        for n0, n1 in ops._image_chunks(N, x8, dy8):
            n = n1 - n0
            if (syy, sxx) == (1, 1) and _halo_wgrad8(
                    x8[n0:n1], sx, dy8[n0:n1], sdy, dw, dbias, pt, pl, OH,
                    OW, groups, splits):
                continue
            sp = splits if splits is not None else ops.wgrad_splits(
                n * OH * OW, OC // groups, KH * KW * Cg, groups)
            _call("hvk_conv_wgrad_fp8", x8[n0:n1].data_ptr(),
                  dy8[n0:n1].data_ptr(), dw.data_ptr(),
                  None if dbias is None else dbias.data_ptr(),
                  n, H, W, C, OC, KH, KW, syy, sxx, pt, pl, OH, OW,
                  groups, int(sp), sx.fmt, sdy.fmt, sx.state.data_ptr(),
                  sdy.state.data_ptr(), HIST, float(sx.fmax_eff),
                  float(sdy.fmax_eff), _s(x8))
        return dw
    acc = torch.zeros_like(dw)
    dq = dequantize(dy8, sdy)
    ops.conv_wgrad(dequantize(x8, sx), dq, acc, sliding, padding, groups)
    dw += acc
    if dbias is not None:
        dbias += dq.reshape(-1, OC).sum(0)
    return dw
