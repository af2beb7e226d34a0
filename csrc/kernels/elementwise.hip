// elementwise.hip - memory-bound kernels of the veles_amd library (gfx950).
//
// Reference kernels replaced: ocl/fullbatch_loader.cl
// (fill_minibatch_data_labels / fill_minibatch_target), mean_disp_normalizer.cl,
// matrix_reduce.cl (bias gradients), join.jcl (InputJoiner), random.cl
// (xorshift1024*, xorshift128+), plus the Znicz evaluator / GD / dropout /
// activation element-wise work.  Every kernel vectorises its bf16 traffic to
// 8-16 B per lane (cdna_hip_programming.md Guideline 13) and grid-strides
// over at most 2048 blocks (Guideline 11).
#include "hvk_common.h"

using namespace hvk;

namespace {
inline int grid_for(long long n, int per_block = 256) {
  long long g = (n + per_block - 1) / per_block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// dtype codes shared with python (veles_amd/ops/_lib.py)
enum DT { DT_F32 = 0, DT_BF16 = 1, DT_U8 = 2, DT_I32 = 3, DT_F16 = 4 };

__device__ __forceinline__ float ld_any(const void* p, long long i, int dt) {
  switch (dt) {
    case DT_F32: return ((const float*)p)[i];
    case DT_BF16: return bf2f(((const uint16_t*)p)[i]);
    case DT_U8: return (float)((const uint8_t*)p)[i];
    case DT_I32: return (float)((const int*)p)[i];
    default: return (float)((const _Float16*)p)[i];
  }
}
__device__ __forceinline__ void st_any(void* p, long long i, int dt, float v) {
  switch (dt) {
    case DT_F32: ((float*)p)[i] = v; break;
    case DT_BF16: ((uint16_t*)p)[i] = f2bf(v); break;
    case DT_U8: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case DT_I32: ((int*)p)[i] = (int)v; break;
    default: ((_Float16*)p)[i] = (_Float16)v; break;
  }
}

// ---------------------------------------------------------------- loader
// out[i][:] = (in[idx[start+i]][:] - mean) * rdisp   (i < count), else 0
// labels_out[i] = labels[idx[start+i]] or -1; indices_out[i] = idx or -1.
__global__ void fill_minibatch_kernel(const void* src, int src_dt,
                                      const int* shuffled, int start, int count,
                                      int max_mb, long long sample_size,
                                      const float* mean, const float* rdisp,
                                      void* dst, int dst_dt, const int* labels,
                                      int* labels_out, int* idx_out) {
  long long total = (long long)max_mb * sample_size;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int i = (int)(e / sample_size);
    long long j = e - (long long)i * sample_size;
    float v = 0.f;
    if (i < count) {
      int s = shuffled[start + i];
      v = ld_any(src, (long long)s * sample_size + j, src_dt);
      if (mean) v -= mean[j];
      if (rdisp) v *= rdisp[j];
    }
    st_any(dst, e, dst_dt, v);
    if (j == 0) {
      int s = i < count ? shuffled[start + i] : -1;
      if (labels_out) labels_out[i] = (s >= 0 && labels) ? labels[s] : -1;
      if (idx_out) idx_out[i] = s;
    }
  }
}

// Row kernel for arbitrary sample sizes: blockIdx.y = row, threads sweep
// the row (coalesced byte loads, no 64-bit division).
__global__ void fill_minibatch_rows_kernel(const void* src, int src_dt,
                                           const int* shuffled, int start,
                                           int count, long long sample_size,
                                           const float* mean,
                                           const float* rdisp, void* dst,
                                           int dst_dt, const int* labels,
                                           int* labels_out, int* idx_out) {
  const int i = blockIdx.y;
  const int s = i < count ? shuffled[start + i] : -1;
  const long long sbase = (long long)s * sample_size;
  const long long dbase = (long long)i * sample_size;
  for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       j < sample_size; j += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (s >= 0) {
      v = ld_any(src, sbase + j, src_dt);
      if (mean) v -= mean[j];
      if (rdisp) v *= rdisp[j];
    }
    st_any(dst, dbase + j, dst_dt, v);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (labels_out) labels_out[i] = (s >= 0 && labels) ? labels[s] : -1;
    if (idx_out) idx_out[i] = s;
  }
}

// Vectorised special case: uint8 source, bf16 destination, sample_size % 16
// == 0.  16 bytes in, 32 bytes out per lane.
__global__ void fill_minibatch_u8_bf16_kernel(const uint8_t* src,
                                              const int* shuffled, int start,
                                              int count, int max_mb,
                                              long long sample_size,
                                              const float* mean,
                                              const float* rdisp, uint16_t* dst,
                                              const int* labels, int* labels_out,
                                              int* idx_out) {
  long long vecs = sample_size / 16;
  long long total = (long long)max_mb * vecs;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int i = (int)(e / vecs);
    long long jv = e - (long long)i * vecs;
    long long j0 = jv * 16;
    uint16_t o[16];
    if (i < count) {
      int s = shuffled[start + i];
      uint4 raw = *(const uint4*)(src + (long long)s * sample_size + j0);
      const uint8_t* b = (const uint8_t*)&raw;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float v = (float)b[q];
        if (mean) v -= mean[j0 + q];
        if (rdisp) v *= rdisp[j0 + q];
        o[q] = f2bf(v);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) o[q] = 0;
    }
    uint4* d = (uint4*)(dst + (long long)i * sample_size + j0);
    d[0] = *(uint4*)&o[0];
    d[1] = *(uint4*)&o[8];
    if (jv == 0) {
      int s = i < count ? shuffled[start + i] : -1;
      if (labels_out) labels_out[i] = (s >= 0 && labels) ? labels[s] : -1;
      if (idx_out) idx_out[i] = s;
    }
  }
}

// out[b][j] = (in[b][j] - mean[j]) * rdisp[j]
__global__ void mean_disp_kernel(const void* in, int in_dt, const float* mean,
                                 const float* rdisp, void* out, int out_dt,
                                 long long total, long long sample) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    long long j = e % sample;
    st_any(out, e, out_dt, (ld_any(in, e, in_dt) - mean[j]) * rdisp[j]);
  }
}

// ------------------------------------------------------------- evaluator
// One wave per row: softmax of logits, then
//   err[i][c] = (p[c] - (c == label)) * scale       (dL/dlogits of mean CE)
//   probs (optional f32 output), per-row loss, argmax; block reductions of
//   n_err and loss into metrics[0..1] (atomics, f32).
// NV > 0: the row's C <= 64 NV logits are read once into registers (NV per
// lane, the same lane-strided order, so the same sums: bit-identical to the
// NV = 0 form, which reads the row three times; AlexNet's 1000 classes at
// b3072: 42 -> 20 us, profiles/r6/softmax_ce_regs_r6ll.log)
template <int NV>
__global__ void softmax_ce_kernel(const void* logits, int in_dt, int B, int C,
                                  const int* labels, float scale, void* err,
                                  int err_dt, float* probs, int* max_idx,
                                  float* metrics, int* confusion) {
  // one wave per row, rows grid-strided: the metric sums stay in registers
  // and reach memory as ONE atomic per block and metric (per-row atomics
  // on the same three addresses serialised at L2: CIFAR quick b4096 spent
  // 82 us per call on them)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float m_err = 0.f, m_loss = 0.f, m_n = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
    long long base = (long long)row * C;
    float mx = -INFINITY;
    int amax = 0;
    constexpr int NR = NV > 0 ? NV : 1;
    float rv[NR];
    if constexpr (NV > 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = lane + 64 * k;
        rv[k] = c < C ? ld_any(logits, base + c, in_dt) : 0.f;
      }
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (lane + 64 * k < C && rv[k] > mx) { mx = rv[k]; amax = lane + 64 * k; }
    } else {
      for (int c = lane; c < C; c += 64) {
        float v = ld_any(logits, base + c, in_dt);
        if (v > mx) { mx = v; amax = c; }
      }
    }
    // wave argmax (first index on ties)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float om = __shfl_xor(mx, o, 64);
      int oa = __shfl_xor(amax, o, 64);
      if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
    }
    float sum = 0.f;
    if constexpr (NV > 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (lane + 64 * k < C) sum += __expf(rv[k] - mx);
    } else {
      for (int c = lane; c < C; c += 64)
        sum += __expf(ld_any(logits, base + c, in_dt) - mx);
    }
    sum = wave_sum(sum);
    float inv = 1.f / sum;
    int lab = labels ? labels[row] : -1;
    auto emit = [&](int c, float v) {
      float p = __expf(v - mx) * inv;
      if (probs) probs[base + c] = p;
      if (err) {
        float g = lab < 0 ? 0.f : (p - (c == lab ? 1.f : 0.f)) * scale;
        st_any(err, base + c, err_dt, g);
      }
    };
    if constexpr (NV > 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if (lane + 64 * k < C) emit(lane + 64 * k, rv[k]);
    } else {
      for (int c = lane; c < C; c += 64)
        emit(c, ld_any(logits, base + c, in_dt));
    }
    if (lane == 0) {
      if (max_idx) max_idx[row] = amax;
      if (lab >= 0 && metrics) {
        float pl = __expf(ld_any(logits, base + lab, in_dt) - mx) * inv;
        m_err += amax != lab ? 1.f : 0.f;
        m_loss += -__logf(fmaxf(pl, 1e-30f));
        m_n += 1.f;
        if (confusion) atomicAdd(&confusion[amax * C + lab], 1);
      }
    }
  }
  if (!metrics) return;
  __shared__ float red[3][4];
  if (lane == 0) {
    red[0][wave] = m_err;
    red[1][wave] = m_loss;
    red[2][wave] = m_n;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float v = red[threadIdx.x][0] + red[threadIdx.x][1] +
                    red[threadIdx.x][2] + red[threadIdx.x][3];
    if (v != 0.f) atomicAdd(&metrics[threadIdx.x], v);
  }
}

// MSE evaluator: err = (y - t) * scale; metrics[0] += sum sq, per-sample
// max/min mse optional.
__global__ void mse_kernel(const void* y, int y_dt, const void* t, int t_dt,
                           int B, int D, float scale, void* err, int err_dt,
                           float* mse_out, float* metrics, int valid_rows) {
  // rows grid-strided per wave; one metric atomic per block (softmax_ce)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float m0 = 0.f, m1 = 0.f, m2 = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
    long long base = (long long)row * D;
    float s = 0.f;
    bool valid = row < valid_rows;
    for (int c = lane; c < D; c += 64) {
      float d = ld_any(y, base + c, y_dt) - ld_any(t, base + c, t_dt);
      if (!valid) d = 0.f;
      s += d * d;
      if (err) st_any(err, base + c, err_dt, d * scale);
    }
    s = wave_sum(s);
    if (lane == 0) {
      float mse = s / D;
      if (mse_out) mse_out[row] = mse;
      if (valid) {
        m0 += mse;
        m1 += sqrtf(mse);
        m2 += 1.f;
      }
    }
  }
  if (!metrics) return;
  __shared__ float red[3][4];
  if (lane == 0) {
    red[0][wave] = m0;
    red[1][wave] = m1;
    red[2][wave] = m2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const float v = red[threadIdx.x][0] + red[threadIdx.x][1] +
                    red[threadIdx.x][2] + red[threadIdx.x][3];
    if (v != 0.f) atomicAdd(&metrics[threadIdx.x], v);
  }
}

// ---------------------------------------------------------- optimizer
// Fused SGD with momentum and L1/L2 decay over a flat parameter buffer split
// into segments with their own hyper-parameters (Znicz GD semantics,
// docs/OPS.md):
//   g = grad*gscale + decay*((1-l1)*w + l1*sign(w))
//   v = moment*v - lr*g ;  w += v ; w_lp = bf16(w)
struct SgdSeg {
  long long begin, end;
  float lr, decay, l1, moment;
};
__global__ void sgd4_kernel(float4* w, float4* grad, float4* mom,
                            uint2* w_lp, const SgdSeg* segs, int nseg,
                            long long total4, float gscale,
                            long long zero_from) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       i < total4; i += (long long)gridDim.x * blockDim.x) {
    long long e = i * 4;
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (segs[mid].begin <= e) lo = mid; else hi = mid - 1;
    }
    const SgdSeg sg = segs[lo];
    float4 wv = w[i], gv = grad[i];
    float4 mv = mom ? mom[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float* wp = (float*)&wv;
    float* gp = (float*)&gv;
    float* mp = (float*)&mv;
    bool in = e >= sg.begin && e < sg.end;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float wi = wp[q];
      float g = gp[q] * gscale;
      if (sg.decay != 0.f)
        g += sg.decay * ((1.f - sg.l1) * wi +
                         sg.l1 * (wi > 0.f ? 1.f : (wi < 0.f ? -1.f : 0.f)));
      float v = -sg.lr * g + sg.moment * mp[q];
      if (!in) v = 0.f;
      mp[q] = in ? v : mp[q];
      wp[q] = wi + v;
    }
    w[i] = wv;
    if (mom) mom[i] = mv;
    // gradients at and past zero_from (a 64-aligned parameter offset) are
    // cleared for the next step's split-K atomics
    if (e >= zero_from) grad[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (w_lp) {
      uint2 o;
      o.x = f2bf(wp[0]) | ((uint32_t)f2bf(wp[1]) << 16);
      o.y = f2bf(wp[2]) | ((uint32_t)f2bf(wp[3]) << 16);
      w_lp[i] = o;
    }
  }
}

__global__ void sgd_kernel(float* w, const float* grad, float* mom,
                           uint16_t* w_lp, const SgdSeg* segs, int nseg,
                           long long total, float gscale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    // segments are few and sorted: linear probe from a binary search
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (segs[mid].begin <= i) lo = mid; else hi = mid - 1;
    }
    const SgdSeg sg = segs[lo];
    float wi = w[i];
    float g = grad[i] * gscale;
    if (sg.decay != 0.f)
      g += sg.decay * ((1.f - sg.l1) * wi + sg.l1 * (wi > 0.f ? 1.f : (wi < 0.f ? -1.f : 0.f)));
    float v = -sg.lr * g;
    if (mom) {
      v += sg.moment * mom[i];
      mom[i] = v;
    }
    wi += v;
    w[i] = wi;
    if (w_lp) w_lp[i] = f2bf(wi);
  }
}

// ------------------------------------------------------------ reductions
// out[c] (+)= sum_r in[r][c]  for in [R][C] (bias gradients / column sums).
// Block = 256 threads covering 256*VEC columns... simple form: each thread
// owns one column and a slab of rows; atomics once per block-column.
__global__ void col_sum_kernel(const void* in, int dt, int R, int C, float* out,
                               int rows_per_block, float scale) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  int r0 = blockIdx.y * rows_per_block;
  int r1 = min(R, r0 + rows_per_block);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += ld_any(in, (long long)r * C + c, dt);
  atomicAdd(&out[c], s * scale);
}

// bf16 column sums, 8 columns (16 B) per thread.  A block sweeps a slab of
// rows; threads with the same chunk are reduced through LDS, then one
// atomic per column per block.
__global__ void col_sum_bf16x8_kernel(const uint16_t* in, int R, int C,
                                      float* out, int rows_per_block,
                                      float scale) {
  const int CH = C >> 3;                 // chunks per row (<= 256)
  const int rpi = blockDim.x / CH;       // rows per sweep
  const int t = threadIdx.x;
  const int ch = t % CH, rr = t / CH;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  if (rr < rpi) {
    for (int r = r0 + rr; r < r1; r += rpi) {
      uint4 v = *(const uint4*)(in + (long long)r * C + ch * 8);
      const uint16_t* h = (const uint16_t*)&v;
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += bf2f(h[q]);
    }
  }
  __shared__ float red[256 * 8];
#pragma unroll
  for (int q = 0; q < 8; ++q) red[t * 8 + q] = (rr < rpi) ? acc[q] : 0.f;
  __syncthreads();
  if (t < CH) {
    float s[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = 0.f;
    for (int k = 0; k < rpi; ++k) {
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += red[(k * CH + t) * 8 + q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) atomicAdd(&out[t * 8 + q], s[q] * scale);
  }
}

// bf16 column sums of any C % 8 == 0 (the FC bias gradients: C = 4096 and
// more): a block is 64 chunks (512 columns) x 4 row lanes over a slab of
// rows, each thread keeping four 16-B loads in flight; the row lanes meet in
// LDS and each column takes one atomic per slab.  Enough slabs that the
// grid covers the CUs several times (an 8 MB read is otherwise latency-
// bound at a few hundred GB/s).
__global__ void __launch_bounds__(256)
col_sum_bf16_wide_kernel(const uint16_t* __restrict__ in, int R, int C,
                         float* out, int rows_per_slab, float scale) {
  const int CH = C >> 3;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rows_per_slab;
  const int r1 = min(R, r0 + rows_per_slab);
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (ch < CH) {
    const uint16_t* p = in + (long long)ch * 8;
    int r = r0 + rl;
    for (; r + 12 < r1; r += 16) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = *(const uint4*)(p + (long long)(r + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[2 * q] += __uint_as_float(w[q] << 16);
          acc[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
        }
      }
    }
    for (; r < r1; r += 4) {
      const uint4 v = *(const uint4*)(p + (long long)r * C);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[2 * q] += __uint_as_float(w[q] << 16);
        acc[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
      }
    }
  }
  __shared__ float red[3][64][9];
  if (rl > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) red[rl - 1][cl][q] = acc[q];
  }
  __syncthreads();
  if (rl == 0 && ch < CH) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += red[k][cl][q];
#pragma unroll
    for (int q = 0; q < 8; ++q) atomicAdd(&out[ch * 8 + q], acc[q] * scale);
  }
}

// out[r] = sum_c in[r][c] * scale  (one wave per row)
__global__ void row_sum_kernel(const void* in, int dt, int R, int C, float* out,
                               float scale) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (r >= R) return;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += ld_any(in, (long long)r * C + c, dt);
  s = wave_sum(s);
  if (lane == 0) out[r] = s * scale;
}

// --------------------------------------------------------- activations
__global__ void act_fwd_kernel(const void* x, int xdt, void* y, int ydt,
                               long long n, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    st_any(y, i, ydt, act_fwd(ld_any(x, i, xdt), act));
}
// dx = dy * act_bwd(y)
__global__ void act_bwd_kernel(const void* dy, int dydt, const void* y, int ydt,
                               void* dx, int dxdt, long long n, int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    st_any(dx, i, dxdt, ld_any(dy, i, dydt) * act_bwd(ld_any(y, i, ydt), act));
}
// bf16 -> bf16 activation / its backward, 8 elements per lane, one switch
// per chunk (standalone activation units: CIFAR quick's ReLU after pooling)
__global__ void act_fwd_bf16x8_kernel(const uint16_t* __restrict__ x,
                                      uint16_t* __restrict__ y, long long n8,
                                      int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const uint4 a = ((const uint4*)x)[i];
    const uint16_t* h = (const uint16_t*)&a;
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = bf2f(h[q]);
    act_fwd8(v, act);
    ((uint4*)y)[i] = pack_bf16x8(v);
  }
}
__global__ void act_bwd_bf16x8_kernel(const uint16_t* __restrict__ dy,
                                      const uint16_t* __restrict__ y,
                                      uint16_t* __restrict__ dx, long long n8,
                                      int act) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const uint4 a = ((const uint4*)dy)[i], b = ((const uint4*)y)[i];
    const uint16_t* ha = (const uint16_t*)&a;
    const uint16_t* hb = (const uint16_t*)&b;
    float v[8], yv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[q] = bf2f(ha[q]);
      yv[q] = bf2f(hb[q]);
    }
    act_bwd_mul8(v, yv, act);
    ((uint4*)dx)[i] = pack_bf16x8(v);
  }
}
// bf16 strict-relu backward, 8 elements per lane (the AlexNet hot case)
__global__ void relu_bwd_bf16x8_kernel(const uint16_t* dy, const uint16_t* y,
                                       uint16_t* dx, long long n8) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    uint4 a = ((const uint4*)dy)[i], b = ((const uint4*)y)[i];
    uint32_t* pa = (uint32_t*)&a;
    const uint32_t* pb = (const uint32_t*)&b;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t m = 0;
      if ((pb[q] & 0x7fff) && !(pb[q] & 0x8000)) m |= 0xffff;
      if ((pb[q] & 0x7fff0000) && !(pb[q] & 0x80000000)) m |= 0xffff0000;
      pa[q] &= m;
    }
    ((uint4*)dx)[i] = a;
  }
}

// --------------------------------------------------------------- dropout
// Counter-based mask (no state; the backward pass regenerates it):
//   keep(i) = hash(seed, i) >= p * 2^32 ; y = keep ? x / (1-p) : 0
__device__ __forceinline__ uint32_t hash32(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// seed_dev (optional): the seed is read from device memory instead, so a
// captured HIP graph draws a fresh mask every replay (hvk_seed_advance).
// element i's mask is hash32(base + i, seed): a rank passes the global index
// of its shard's first element (rank x local elements), so the ranks of a
// data-parallel step draw exactly the masks a single process would draw for
// the whole global minibatch
__global__ void dropout_kernel(const void* x, int xdt, void* y, int ydt,
                               long long n, uint32_t seed, uint32_t thresh,
                               float scale, uint8_t* mask_out,
                               const uint32_t* seed_dev, long long base) {
  if (seed_dev) seed = __builtin_amdgcn_readfirstlane(seed_dev[0]);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    bool keep = hash32((uint32_t)(base + i), seed) >= thresh;
    st_any(y, i, ydt, keep ? ld_any(x, i, xdt) * scale : 0.f);
    if (mask_out) mask_out[i] = keep;
  }
}

// bf16 -> bf16 without a mask output: 8 elements (16-B loads and stores)
// per thread, the same hash per element index and the same f32 product and
// rounding as dropout_kernel (bit-identical; AlexNet's fc6 / fc7 dropout at
// b3072 was 23 us on the per-element form)
__global__ void dropout_bf16x8_kernel(const uint4* __restrict__ x,
                                      uint4* __restrict__ y, long long n8,
                                      uint32_t seed, uint32_t thresh,
                                      float scale, const uint32_t* seed_dev,
                                      long long base) {
  if (seed_dev) seed = __builtin_amdgcn_readfirstlane(seed_dev[0]);
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n8;
       q += (long long)gridDim.x * blockDim.x) {
    const uint4 v = x[q];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool keep = hash32((uint32_t)(base + q * 8 + e), seed) >= thresh;
      const uint16_t h = (uint16_t)(w[e >> 1] >> (16 * (e & 1)));
      f[e] = keep ? bf2f(h) * scale : 0.f;
    }
    y[q] = pack_bf16x8(f);
  }
}

// ------------------------------------------------------------------- RNG
// xorshift1024*: bit-exact with veles_amd.prng.xorshift1024star (and with the
// reference ocl/random.cl:42-70): out[round*16*n + i*n + id].
__global__ void xorshift1024_kernel(uint64_t* states, int n_states, int rounds,
                                    uint64_t* out) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n_states) return;
  uint64_t s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = states[id * 16 + i];
  long long offs = id;
  for (int r = 0; r < rounds; ++r) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint64_t s0 = s[i];
      uint64_t s1 = s[(i + 1) & 15];
      s1 ^= s1 << 31;
      s1 ^= s1 >> 11;
      s0 ^= s0 >> 30;
      s[(i + 1) & 15] = s0 ^ s1;
      out[offs] = s[(i + 1) & 15] * 1181783497276652981ull;
      offs += n_states;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) states[id * 16 + i] = s[i];
}

__global__ void xorshift128p_kernel(uint64_t* states, int n, uint64_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s1 = states[2 * i], s0 = states[2 * i + 1];
  states[2 * i] = s0;
  s1 ^= s1 << 23;
  uint64_t ns = s1 ^ s0 ^ (s1 >> 17) ^ (s0 >> 26);
  states[2 * i + 1] = ns;
  out[i] = ns + s0;
}

// uniform floats in [lo, hi) from uint64 stream
__global__ void u64_to_uniform_kernel(const uint64_t* in, float* out,
                                      long long n, float lo, float hi) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = lo + (hi - lo) * ((float)(in[i] >> 40) * (1.0f / 16777216.0f));
}

// ---------------------------------------------------------------- concat
// out[b][offs_k + j] = in_k[b][j]
struct JoinArgs {
  const void* in[16];
  int len[16];
  int offs[16];
};
__global__ void join_kernel(JoinArgs a, int nin, int dt, void* out, int B,
                            int out_len) {
  long long total = (long long)B * out_len;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    int b = (int)(e / out_len);
    int j = (int)(e - (long long)b * out_len);
    int k = 0;
    while (k + 1 < nin && j >= a.offs[k + 1]) ++k;
    int jj = j - a.offs[k];
    float v = jj < a.len[k] ? ld_any(a.in[k], (long long)b * a.len[k] + jj, dt) : 0.f;
    st_any(out, e, dt, v);
  }
}

// ------------------------------------------------------------------ cast
__global__ void cast_kernel(const void* in, int idt, void* out, int odt,
                            long long n, float scale) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    st_any(out, i, odt, ld_any(in, i, idt) * scale);
}
__global__ void f32_to_bf16x4_kernel(const float4* in, uint2* out, long long n4) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 v = in[i];
    uint2 o;
    o.x = f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
    o.y = f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
    out[i] = o;
  }
}
}  // namespace


// Space-to-depth for strided small-channel convs (AlexNet conv1: 227x227x3,
// 11x11 stride 4 -> 57x57x48 image, 3x3 stride 1 kernel): y[n][Y][X][(dy*s +
// dx)*C + c] = x[n][s*Y+dy-pt][s*X+dx-pl][c] (0 outside).  The result has
// C2 = s*s*C % 8 == 0 channels, so the conv runs on the aligned LDS-DMA
// implicit-GEMM path instead of per-element run gathers.
__global__ void space_to_depth_kernel(const uint16_t* __restrict__ x,
                                      uint16_t* __restrict__ y, int H, int W,
                                      int C, int s, int pt, int pl, int H2,
                                      int W2, FastDiv fS, FastDiv fW2,
                                      FastDiv fH2, long long runs) {
  // one thread = one (output pixel, dy) run: the s*C contiguous input
  // elements x[n][s*Y+dy-pt][s*X-pl .. +s)[0..C) land contiguously at
  // channel offset dy*s*C of the output pixel
  const int RUN = s * C;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       q < runs; q += (long long)gridDim.x * blockDim.x) {
    // X fastest: a wave reads consecutive runs of one input row
    uint32_t r, dy, X, t, Y, n, pix;
    fdivmod((uint32_t)q, fW2, r, X);
    fdivmod(r, fS, t, dy);
    fdivmod(t, fH2, n, Y);
    pix = (n * H2 + Y) * W2 + X;
    uint16_t* out = y + (long long)pix * s * RUN + dy * RUN;
    int iy = s * (int)Y + (int)dy - pt, ix0 = s * (int)X - pl;
    if (iy < 0 || iy >= H) {
      for (int e = 0; e < RUN; ++e) out[e] = 0;
      continue;
    }
    const uint16_t* in = x + ((long long)n * H + iy) * W * C;
    if (ix0 >= 0 && ix0 + s <= W) {
      const uint16_t* src = in + (long long)ix0 * C;
      for (int e = 0; e < RUN; ++e) out[e] = src[e];
    } else {
      for (int e = 0; e < RUN; ++e) {
        int ix = ix0 + e / C;
        out[e] = (ix >= 0 && ix < W) ? in[(long long)ix * C + e % C]
                                     : (uint16_t)0;
      }
    }
  }
}


// Adaptive solvers over the same flat buffers (Znicz GD "solvers":
// docs/source/manualrst_veles_workflow_parameters.rst:543-578), one mode per
// segment:
//   0 momentum  v = m*v - lr*g ; w += v                         (s1 = v)
//   1 adagrad   s1 += g^2 ; w -= lr*g/(sqrt(s1)+eps)
//   2 adadelta  s1 = r*s1+(1-r)g^2 ; d = g*sqrt(s2+eps)/sqrt(s1+eps) ;
//               s2 = r*s2+(1-r)d^2 ; w -= lr*d
//   3 rprop     (iRprop-) s1 = step, s2 = previous gradient:
//               same sign -> step*1.2 (<= 50), flip -> step*0.5 (>= 1e-6),
//               g = 0 ; w -= sign(g)*step ; s2 = g
struct SolverSeg {
  long long begin, end;
  float lr, decay, l1, moment;
  int mode;
  float eps, rho, pad;
};
__global__ void solver_kernel(float* w, float* grad, float* s1, float* s2,
                              uint16_t* w_lp, const SolverSeg* segs, int nseg,
                              long long total, float gscale,
                              long long zero_from) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       i < total; i += (long long)gridDim.x * blockDim.x) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (segs[mid].begin <= i) lo = mid; else hi = mid - 1;
    }
    const SolverSeg sg = segs[lo];
    float wi = w[i];
    if (i < sg.end) {
      float g = grad[i] * gscale;
      if (sg.decay != 0.f)
        g += sg.decay * ((1.f - sg.l1) * wi +
                         sg.l1 * (wi > 0.f ? 1.f : (wi < 0.f ? -1.f : 0.f)));
      switch (sg.mode) {
        case 1: {
          float a = s1[i] + g * g;
          s1[i] = a;
          wi -= sg.lr * g / (sqrtf(a) + sg.eps);
          break;
        }
        case 2: {
          float a = sg.rho * s1[i] + (1.f - sg.rho) * g * g;
          float d = g * sqrtf(s2[i] + sg.eps) / sqrtf(a + sg.eps);
          s1[i] = a;
          s2[i] = sg.rho * s2[i] + (1.f - sg.rho) * d * d;
          wi -= sg.lr * d;
          break;
        }
        case 3: {
          float step = s1[i] > 0.f ? s1[i] : sg.lr;
          float pg = s2[i];
          if (pg * g > 0.f) step = fminf(step * 1.2f, 50.f);
          else if (pg * g < 0.f) { step = fmaxf(step * 0.5f, 1e-6f); g = 0.f; }
          wi -= (g > 0.f ? step : (g < 0.f ? -step : 0.f));
          s1[i] = step;
          s2[i] = g;
          break;
        }
        default: {
          float v = sg.moment * s1[i] - sg.lr * g;
          s1[i] = v;
          wi += v;
        }
      }
      w[i] = wi;
    }
    if (i >= zero_from) grad[i] = 0.f;
    if (w_lp) w_lp[i] = f2bf(wi);
  }
}


// uint8 -> bf16 rows of any length (e.g. 227*227*3): 8 elements per lane,
// unaligned 8-B loads / 16-B stores (gfx950 unaligned access), per-feature
// mean / rdisp as float4 pairs; the row tail is scalar.
template <int SPT>
__global__ void fill_rows_u8_bf16_kernel(const uint8_t* __restrict__ src,
                                         const int* shuffled, int start,
                                         int count, int max_mb,
                                         long long sample_size,
                                         const float* __restrict__ mean,
                                         const float* __restrict__ rdisp,
                                         uint16_t* __restrict__ dst,
                                         const int* labels, int* labels_out,
                                         int* idx_out) {
  // SPT samples per thread: the per-feature mean / rdisp (2 x 32 B per 8
  // features) are loaded once and reused across the samples
  const int i0 = blockIdx.y * SPT;
  int sidx[SPT];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int i = i0 + q;
    sidx[q] = i < count ? shuffled[start + i] : -1;
  }
  const long long nv = sample_size / 8;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       v < nv; v += (long long)gridDim.x * blockDim.x) {
    const long long j = v * 8;
    float4 m0 = make_float4(0.f, 0.f, 0.f, 0.f), m1 = m0;
    float4 r0 = make_float4(1.f, 1.f, 1.f, 1.f), r1 = r0;
    if (mean) { m0 = ((const float4*)(mean + j))[0]; m1 = ((const float4*)(mean + j))[1]; }
    if (rdisp) { r0 = ((const float4*)(rdisp + j))[0]; r1 = ((const float4*)(rdisp + j))[1]; }
    const float mm[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    const float rr[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    uint8_t b[SPT][8];
#pragma unroll
    for (int q = 0; q < SPT; ++q)
      if (sidx[q] >= 0)
        __builtin_memcpy(b[q], src + (long long)sidx[q] * sample_size + j, 8);
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      const int i = i0 + q;
      if (i >= max_mb) break;
      uint16_t o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = sidx[q] >= 0 ? f2bf(((float)b[q][e] - mm[e]) * rr[e]) : 0;
      __builtin_memcpy(dst + (long long)i * sample_size + j, o, 16);
    }
  }
  if (blockIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      const int i = i0 + q;
      if (i >= max_mb) break;
      const uint8_t* in = src + (long long)(sidx[q] < 0 ? 0 : sidx[q]) * sample_size;
      uint16_t* out = dst + (long long)i * sample_size;
      for (long long j = nv * 8 + threadIdx.x; j < sample_size; j += blockDim.x) {
        float x = 0.f;
        if (sidx[q] >= 0) {
          x = (float)in[j];
          if (mean) x -= mean[j];
          if (rdisp) x *= rdisp[j];
        }
        out[j] = f2bf(x);
      }
      if (threadIdx.x == 0) {
        if (labels_out) labels_out[i] = (sidx[q] >= 0 && labels) ? labels[sidx[q]] : -1;
        if (idx_out) idx_out[i] = sidx[q];
      }
    }
  }
}


// Loader gather fused with the space-to-depth transform of the first
// (strided, small-channel) convolution: uint8 samples [H][W][C] ->
// normalised bf16 s2d images [H2][W2][S][S][C] (the layout hvk_conv_fwd reads
// for the stride-1 conv that replaces the strided one), so the bf16 NHWC
// image is never written and re-read.  mean2 / rdisp2 are the per-feature
// affine map already laid out in s2d order (0 / 1 where no input pixel is,
// so such elements come out 0: the conv's zero padding).
// A lane owns one 16-B output chunk (8 elements) of SPT samples, so each
// wave stores 1 KiB contiguous: the chunk's affine map is loaded once; its 8
// source bytes are one or two pieces of the S*C-byte input row runs, read
// by aligned dword loads + v_alignbyte (the runs are not dword aligned).
__device__ __forceinline__ uint64_t load_u8x8(const uint8_t* __restrict__ src,
                                              long long off, int n,
                                              long long src_bytes) {
  // n <= 8 bytes at src + off, little-endian in the low bytes
  const long long a = off & ~3ll;
  if (a + 12 <= src_bytes) {
    const uint32_t* w = (const uint32_t*)(src + a);
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
    const uint32_t sh = (uint32_t)(off & 3);
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    uint64_t v = ((uint64_t)hi << 32) | lo;
    return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
  }
  uint64_t v = 0;
  for (int b = 0; b < n; ++b) v |= (uint64_t)src[off + b] << (8 * b);
  return v;
}

// Per thread: the SPT sample ids first, then every source load of the SPT
// samples (both row pieces, three aligned dwords each, at clamped in-range
// addresses - absent pieces are masked afterwards), then the arithmetic and
// the stores: one memory round trip per thread instead of one per sample and
// piece (the branchy per-sample form waited on each load in turn).
template <int S, int C, int SPT>
__global__ void __launch_bounds__(256)
fill_s2d_u8_bf16_kernel(const uint8_t* __restrict__ src, long long src_bytes,
                        const int* shuffled, int start, int count, int max_mb,
                        int H, int W, int pt, int pl, int H2, int W2,
                        const float* __restrict__ mean2,
                        const float* __restrict__ rdisp2,
                        uint16_t* __restrict__ dst, const int* labels,
                        int* labels_out, int* idx_out) {
  constexpr int RUN = S * C, PIX = S * RUN, CPP = PIX / 8;
  static_assert(PIX % 8 == 0 && RUN >= 8, "16-B chunks, <= 2 row pieces");
  const int chunks = H2 * W2 * CPP;
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  const int i0 = blockIdx.y * SPT;
  const long long sample = (long long)H * W * C;
  if (ch < chunks) {
    const int q = ch / CPP, j = ch - (ch / CPP) * CPP;
    const int Y = q / W2, X = q - (q / W2) * W2;
    // the chunk's elements 8j .. 8j+7: piece 0 in row dy0 from r0 (n0
    // bytes), piece 1 (if any) at the start of row dy0 + 1
    const int e0 = 8 * j, dy0 = e0 / RUN, r0 = e0 - dy0 * RUN;
    const int n0 = RUN - r0 < 8 ? RUN - r0 : 8;
    const int ix0 = S * X - pl;
    const bool xin = ix0 >= 0 && ix0 + S <= W;
    const int iy0 = S * Y + dy0 - pt, iy1 = iy0 + 1;
    const bool y0in = iy0 >= 0 && iy0 < H, y1in = iy1 >= 0 && iy1 < H;
    int sid[SPT];
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int i = i0 + u;
      sid[u] = (i < max_mb && i < count) ? shuffled[start + i] : -1;
    }
    uint64_t v[SPT];
    if (xin) {
      // in-image offsets of the two pieces (the byte shift within the
      // aligned dwords depends on the sample base too: H*W*C may be odd)
      const long long o0 = ((long long)iy0 * W + ix0) * C + r0;
      const long long o1 = ((long long)iy1 * W + ix0) * C;
      uint32_t d[SPT][6];
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const long long base = (long long)(sid[u] < 0 ? 0 : sid[u]) * sample;
        long long a0 = (base + o0) & ~3ll, a1 = (base + o1) & ~3ll;
        // clamp into the buffer (out-of-image rows, the last image's tail):
        // such words are masked or re-read exactly below
        a0 = min(max(a0, 0ll), src_bytes - 12);
        a1 = min(max(a1, 0ll), src_bytes - 12);
        const uint32_t* w0 = (const uint32_t*)(src + a0);
        const uint32_t* w1 = (const uint32_t*)(src + a1);
        d[u][0] = w0[0]; d[u][1] = w0[1]; d[u][2] = w0[2];
        d[u][3] = w1[0]; d[u][4] = w1[1]; d[u][5] = w1[2];
      }
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        const long long base = (long long)(sid[u] < 0 ? 0 : sid[u]) * sample;
        const uint32_t sh0 = (uint32_t)((base + o0) & 3);
        const uint32_t sh1 = (uint32_t)((base + o1) & 3);
        uint64_t p0 = ((uint64_t)__builtin_amdgcn_alignbyte(d[u][2], d[u][1], sh0)
                       << 32) |
                      __builtin_amdgcn_alignbyte(d[u][1], d[u][0], sh0);
        uint64_t p1 = ((uint64_t)__builtin_amdgcn_alignbyte(d[u][5], d[u][4], sh1)
                       << 32) |
                      __builtin_amdgcn_alignbyte(d[u][4], d[u][3], sh1);
        // the rare clamped tail: exact byte reads
        if (((base + o0) & ~3ll) + 12 > src_bytes && y0in)
          p0 = load_u8x8(src, base + o0, n0, src_bytes);
        if (n0 < 8 && ((base + o1) & ~3ll) + 12 > src_bytes && y1in)
          p1 = load_u8x8(src, base + o1, 8 - n0, src_bytes);
        if (n0 < 8) p0 &= (1ull << (8 * n0)) - 1;
        uint64_t r = y0in ? p0 : 0;
        if (n0 < 8 && y1in) r |= p1 << (8 * n0);
        v[u] = sid[u] >= 0 ? r : 0;
      }
    } else {
      // image border: per element, zero outside the image
#pragma unroll
      for (int u = 0; u < SPT; ++u) {
        v[u] = 0;
        if (sid[u] < 0) continue;
        const long long base = (long long)sid[u] * sample;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int ee = e0 + e, dy = ee / RUN, rr2 = ee - dy * RUN;
          const int iy = S * Y + dy - pt, ix = ix0 + rr2 / C;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W)
            v[u] |= (uint64_t)src[base + ((long long)iy * W + ix) * C +
                                  rr2 % C] << (8 * e);
        }
      }
    }
    float mm[8], rr[8];
    {
      const float4* m4 = (const float4*)(mean2 + (long long)ch * 8);
      const float4* r4 = (const float4*)(rdisp2 + (long long)ch * 8);
      const float4 a = m4[0], b = m4[1], c = r4[0], d = r4[1];
      mm[0] = a.x; mm[1] = a.y; mm[2] = a.z; mm[3] = a.w;
      mm[4] = b.x; mm[5] = b.y; mm[6] = b.z; mm[7] = b.w;
      rr[0] = c.x; rr[1] = c.y; rr[2] = c.z; rr[3] = c.w;
      rr[4] = d.x; rr[5] = d.y; rr[6] = d.z; rr[7] = d.w;
    }
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int i = i0 + u;
      if (i >= max_mb) break;
      uint4 o = make_uint4(0, 0, 0, 0);
      if (sid[u] >= 0) {
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          f[e] = ((float)((v[u] >> (8 * e)) & 0xFF) - mm[e]) * rr[e];
        o = pack_bf16x8(f);
      }
      *(uint4*)(dst + (long long)i * chunks * 8 + (long long)ch * 8) = o;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < SPT) {
    const int i = i0 + threadIdx.x;
    if (i < max_mb) {
      const int sid = i < count ? shuffled[start + i] : -1;
      if (labels_out) labels_out[i] = (sid >= 0 && labels) ? labels[sid] : -1;
      if (idx_out) idx_out[i] = sid;
    }
  }
}

// Row-staged form (the default): a workgroup builds RPB output rows Y of
// IPB samples (4; hvk_gemm_variant 61: one).  Their S input rows are S * W * C CONTIGUOUS bytes, loaded into
// LDS by 16-B loads (unaligned addresses are fine on gfx950), out-of-image
// rows zero-filled; each lane then assembles 16-B output chunks (8 s2d
// elements) from LDS bytes and stores them, a wave writing 1 KiB
// contiguous.  Global traffic is two streams of whole lines (the per-chunk
// kernel above read three dwords per row piece per lane).  The chunk's
// mean / 1/dispersion (32 B of loads per 16 B written) and its LDS byte
// offsets serve all IPB samples.
extern int hvk_gemm_variant;

template <int S, int C, int RPB, int IPB>
__global__ void __launch_bounds__(256)
fill_s2d_rows_kernel(const uint8_t* __restrict__ src, long long src_bytes,
                     const int* shuffled, int start, int count, int max_mb,
                     int H, int W, int pt, int pl, int H2, int W2,
                     const float* __restrict__ mean2,
                     const float* __restrict__ rdisp2,
                     uint16_t* __restrict__ dst, const int* labels,
                     int* labels_out, int* idx_out) {
  constexpr int PIX = S * S * C, CPP = PIX / 8;
  static_assert(PIX % 8 == 0, "16-B chunks");
  extern __shared__ __attribute__((aligned(16))) uint8_t rows_lds[];
  const int i0 = blockIdx.y * IPB;
  const int Y0 = blockIdx.x * RPB;
  const int WC = W * C;
  const int RB = (S * WC + 15) & ~15;   // LDS bytes per output row's input
  const int t = threadIdx.x;
  int sid[IPB];
#pragma unroll
  for (int b = 0; b < IPB; ++b) {
    const int i = i0 + b;
    sid[b] = (i < max_mb && i < count) ? shuffled[start + i] : -1;
    if (blockIdx.x == 0 && t == 0 && i < max_mb) {
      if (labels_out) labels_out[i] = (sid[b] >= 0 && labels) ? labels[sid[b]] : -1;
      if (idx_out) idx_out[i] = sid[b];
    }
  }
  const int nrow = min(RPB, H2 - Y0);
  const int cpr = W2 * CPP;             // output chunks per row
  // stage: for each image and each of the nrow output rows, its S input rows
  const int nch = RB / 16;
  for (int q = t; q < IPB * nrow * nch; q += 256) {
    const int b = q / (nrow * nch);
    const int q2 = q - b * (nrow * nch);
    const int r = q2 / nch, c = q2 - (q2 / nch) * nch;
    const int byte = c * 16;                 // within the S rows
    uint4 v = make_uint4(0, 0, 0, 0);
    int sidb = -1;   // sid[b] (a register array: no dynamic index)
#pragma unroll
    for (int bb = 0; bb < IPB; ++bb)
      if (bb == b) sidb = sid[bb];
    if (sidb >= 0) {
      const long long base = (long long)sidb * H * WC;
      const int iy = S * (Y0 + r) - pt + byte / WC;
      // the chunk may straddle input rows: load it whole when every row it
      // touches is in the image and the 16 bytes stay inside the buffer,
      // else byte by byte
      const long long g = base + (long long)(S * (Y0 + r) - pt) * WC + byte;
      const int dy2 = min(byte + 15, S * WC - 1) / WC;
      const int iy2 = S * (Y0 + r) - pt + dy2;
      if (iy >= 0 && iy2 < H && g + 16 <= src_bytes) {
        __builtin_memcpy(&v, src + g, 16);
      } else {
        uint8_t e8[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int bb2 = byte + e;
          const int ry = S * (Y0 + r) - pt + bb2 / WC;
          e8[e] = (bb2 < S * WC && ry >= 0 && ry < H) ? src[g + e] : 0;
        }
        __builtin_memcpy(&v, e8, 16);
      }
    }
    *(uint4*)(rows_lds + (b * RPB + r) * RB + byte) = v;
  }
  __syncthreads();
  // each output chunk: its 8 LDS byte offsets, mean and 1/dispersion once,
  // then the IPB images
  for (int q = t; q < nrow * cpr; q += 256) {
    const int r = q / cpr, cc = q - (q / cpr) * cpr;
    const int X = cc / CPP, j = cc - (cc / CPP) * CPP;
    const long long ch = ((long long)(Y0 + r) * W2 * CPP + cc);
    const float4* m4 = (const float4*)(mean2 + ch * 8);
    const float4* r4 = (const float4*)(rdisp2 + ch * 8);
    const float4 ma = m4[0], mb = m4[1], ra = r4[0], rb = r4[1];
    const float mm[8] = {ma.x, ma.y, ma.z, ma.w, mb.x, mb.y, mb.z, mb.w};
    const float rr[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
    int off[8];
    bool in[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int el = 8 * j + e;
      const int dy = el / (S * C), rem = el - dy * (S * C);
      const int dx = rem / C, c = rem - dx * C;
      const int ix = S * X + dx - pl;
      // outside the image: the affine map is (0, 1) there, the byte 0
      in[e] = ix >= 0 && ix < W;
      off[e] = r * RB + dy * WC + ix * C + c;
    }
#pragma unroll
    for (int b = 0; b < IPB; ++b) {
      if (i0 + b >= max_mb) break;
      uint16_t* out = dst + (long long)(i0 + b) * H2 * cpr * 8;
      uint4 o = make_uint4(0, 0, 0, 0);
      if (sid[b] >= 0) {
        const uint8_t* lb = rows_lds + b * RPB * RB;
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t v = in[e] ? lb[off[e]] : (uint8_t)0;
          f[e] = ((float)v - mm[e]) * rr[e];
        }
        o = pack_bf16x8(f);
      }
      *(uint4*)(out + ch * 8) = o;
    }
  }
}

HVK_API int hvk_fill_minibatch_s2d(const void* src, long long src_bytes,
                                   const int* shuffled, int start, int count,
                                   int max_mb, int H, int W, int C, int S,
                                   int pt, int pl, int H2, int W2,
                                   const float* mean2, const float* rdisp2,
                                   void* dst, const int* labels,
                                   int* labels_out, int* idx_out,
                                   hipStream_t s) {
  if (S != 4 || C != 3 || ((uintptr_t)dst & 15) || ((uintptr_t)mean2 & 15) ||
      ((uintptr_t)rdisp2 & 15) || max_mb > 65535 * 4)
    return -1;
  if (hvk_gemm_variant == 61 && max_mb <= 65535) {   // one image per block
    constexpr int RPB = 2;
    const size_t lds = (size_t)RPB * ((S * W * C + 15) & ~15);
    hipLaunchKernelGGL((fill_s2d_rows_kernel<4, 3, RPB, 1>),
                       dim3((H2 + RPB - 1) / RPB, max_mb), dim3(256), lds, s,
                       (const uint8_t*)src, src_bytes, shuffled, start, count,
                       max_mb, H, W, pt, pl, H2, W2, mean2, rdisp2,
                       (uint16_t*)dst, labels, labels_out, idx_out);
    return (int)launch_status(s);
  }
  if (hvk_gemm_variant != 60 && max_mb <= 65535 * 4) {
    // four images per block: the mean / dispersion loads and the chunk's
    // byte offsets once for all four
    constexpr int RPB = 2, IPB = 4;
    const size_t lds = (size_t)IPB * RPB * ((S * W * C + 15) & ~15);
    hipLaunchKernelGGL((fill_s2d_rows_kernel<4, 3, RPB, IPB>),
                       dim3((H2 + RPB - 1) / RPB, (max_mb + IPB - 1) / IPB),
                       dim3(256), lds, s,
                       (const uint8_t*)src, src_bytes, shuffled, start, count,
                       max_mb, H, W, pt, pl, H2, W2, mean2, rdisp2,
                       (uint16_t*)dst, labels, labels_out, idx_out);
    return (int)launch_status(s);
  }
  constexpr int SPT = 4;
  const int chunks = H2 * W2 * (4 * 4 * 3 / 8);
  hipLaunchKernelGGL((fill_s2d_u8_bf16_kernel<4, 3, SPT>),
                     dim3((chunks + 255) / 256, (max_mb + SPT - 1) / SPT),
                     dim3(256), 0, s, (const uint8_t*)src, src_bytes, shuffled,
                     start, count, max_mb, H, W, pt, pl, H2, W2, mean2, rdisp2,
                     (uint16_t*)dst, labels, labels_out, idx_out);
  return (int)launch_status(s);
}

// ---------------------------------------------------------------------------
// Image minibatch with augmentation (the image loaders' device path): output
// sample b is built from the uint8 canvas src[idx[b]] ([Hs][Ws][C], NHWC):
//   crop   a Ho x Wo window at (cy, cx) of the canvas,
//   mirror it horizontally (mirror != 0),
//   rotate it by theta about its centre (cv2.getRotationMatrix2D semantics:
//          the source of output pixel p is c + R(-theta) (p - c), sampled
//          bilinearly; taps outside the crop window read the background -
//          bg image [Ho][Wo][C] or the per-channel bgcolor),
//   sobel  optionally append the gradient magnitude of the grey image
//          (3x3 Sobel on the final geometry, edges replicated),
//   normalise (v - mean[f]) * rdisp[f] per output feature f (or 0 / 1),
// written as bf16 [B][Ho][Wo][C + sobel].  params[b] = {cy, cx, cos, sin,
// mirror, -}; idx[b] < 0 writes a zero sample.  Replaces the reference's
// per-image cv2 crop / flip / warpAffine / Sobel on the host
// (veles/loader/image.py:458-551); the random parameters come from the
// loader's PRNG on the host, so no device->host sync is needed.
struct ImgGeom {
  int Hs, Ws, C, Ho, Wo, Co;
  long long src_stride;  // bytes per canvas
};

__device__ __forceinline__ void img_sample(const uint8_t* __restrict__ can,
                                           const ImgGeom& g, const float* pr,
                                           const uint8_t* __restrict__ bg,
                                           const float* __restrict__ bgcolor,
                                           int oy, int ox, float* v) {
  const int cy = (int)pr[0], cx = (int)pr[1];
  const float ct = pr[2], st = pr[3];
  const bool mir = pr[4] != 0.f;
  // centre as cv2 uses it: (W // 2, H // 2)
  const float ccx = (float)(g.Wo / 2), ccy = (float)(g.Ho / 2);
  const float dx = (float)ox - ccx, dy = (float)oy - ccy;
  float sx = ccx + ct * dx - st * dy;
  float sy = ccy + st * dx + ct * dy;
  if (mir) sx = (float)(g.Wo - 1) - sx;
  const float fx = floorf(sx), fy = floorf(sy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float ax = sx - fx, ay = sy - fy;
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int yy = y0 + (t >> 1), xx = x0 + (t & 1);
    const float w = ((t >> 1) ? ay : 1.f - ay) * ((t & 1) ? ax : 1.f - ax);
    if (w == 0.f) continue;
    const bool in = yy >= 0 && yy < g.Ho && xx >= 0 && xx < g.Wo &&
                    cy + yy < g.Hs && cx + xx < g.Ws;
    for (int c = 0; c < g.C; ++c) {
      float s;
      if (in) {
        s = (float)can[((long long)(cy + yy) * g.Ws + (cx + xx)) * g.C + c];
      } else if (bg) {
        const int by = min(max(yy, 0), g.Ho - 1), bx = min(max(xx, 0), g.Wo - 1);
        s = (float)bg[((long long)by * g.Wo + bx) * g.C + c];
      } else {
        s = bgcolor ? bgcolor[c] : 0.f;
      }
      v[c] += w * s;
    }
  }
}

__device__ __forceinline__ float img_gray(const float* v, int C) {
  return C >= 3 ? 0.299f * v[0] + 0.587f * v[1] + 0.114f * v[2] : v[0];
}

__global__ void __launch_bounds__(256)
image_batch_kernel(const uint8_t* __restrict__ src, ImgGeom g,
                   const int* __restrict__ idx, const float* __restrict__ params,
                   int B, int sobel, const float* __restrict__ mean,
                   const float* __restrict__ rdisp,
                   const uint8_t* __restrict__ bg,
                   const float* __restrict__ bgcolor,
                   uint16_t* __restrict__ out) {
  const long long pix = (long long)g.Ho * g.Wo;
  const long long total = (long long)B * pix;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       e < total; e += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(e / pix);
    const int q = (int)(e - (long long)b * pix);
    const int oy = q / g.Wo, ox = q - (q / g.Wo) * g.Wo;
    uint16_t* o = out + e * g.Co;
    const int s = idx[b];
    if (s < 0) {
      for (int c = 0; c < g.Co; ++c) o[c] = 0;
      continue;
    }
    const uint8_t* can = src + (long long)s * g.src_stride;
    const float* pr = params + 6 * b;
    float v[4];
    img_sample(can, g, pr, bg, bgcolor, oy, ox, v);
    float sob = 0.f;
    if (sobel) {
      float gr[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = min(max(oy + t / 3 - 1, 0), g.Ho - 1);
        const int xx = min(max(ox + t % 3 - 1, 0), g.Wo - 1);
        float w[4];
        img_sample(can, g, pr, bg, bgcolor, yy, xx, w);
        gr[t] = img_gray(w, g.C);
      }
      const float gx = (gr[2] + 2.f * gr[5] + gr[8]) - (gr[0] + 2.f * gr[3] + gr[6]);
      const float gy = (gr[6] + 2.f * gr[7] + gr[8]) - (gr[0] + 2.f * gr[1] + gr[2]);
      sob = sqrtf(gx * gx + gy * gy);
    }
    const long long f0 = (long long)q * g.Co;
    for (int c = 0; c < g.Co; ++c) {
      float x = c < g.C ? v[c] : sob;
      if (mean) x -= mean[f0 + c];
      if (rdisp) x *= rdisp[f0 + c];
      o[c] = f2bf(x);
    }
  }
}

HVK_API int hvk_image_batch(const void* src, long long src_stride, int Hs,
                            int Ws, int C, const int* idx, const float* params,
                            int B, int Ho, int Wo, int sobel,
                            const float* mean, const float* rdisp,
                            const void* bg, const float* bgcolor, void* out,
                            hipStream_t s) {
  if (C < 1 || C > 4 || Ho > Hs || Wo > Ws) return -1;
  ImgGeom g;
  g.Hs = Hs; g.Ws = Ws; g.C = C; g.Ho = Ho; g.Wo = Wo; g.Co = C + (sobel ? 1 : 0);
  g.src_stride = src_stride;
  const long long total = (long long)B * Ho * Wo;
  hipLaunchKernelGGL(image_batch_kernel, dim3(grid_for(total)), dim3(256), 0,
                     s, (const uint8_t*)src, g, idx, params, B, sobel, mean,
                     rdisp, (const uint8_t*)bg, bgcolor, (uint16_t*)out);
  return (int)launch_status(s);
}

HVK_API int hvk_fill_minibatch(const void* src, int src_dt, const int* shuffled,
                               int start, int count, int max_mb,
                               long long sample_size, const float* mean,
                               const float* rdisp, void* dst, int dst_dt,
                               const int* labels, int* labels_out, int* idx_out,
                               hipStream_t s) {
  if (src_dt == DT_U8 && dst_dt == DT_BF16 && sample_size % 16 == 0 &&
      ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
    long long total = (long long)max_mb * (sample_size / 16);
    hipLaunchKernelGGL(fill_minibatch_u8_bf16_kernel, dim3(grid_for(total)),
                       dim3(256), 0, s, (const uint8_t*)src, shuffled, start,
                       count, max_mb, sample_size, mean, rdisp, (uint16_t*)dst,
                       labels, labels_out, idx_out);
  } else if (src_dt == DT_U8 && dst_dt == DT_BF16 && max_mb <= 65535 &&
             (!mean || ((uintptr_t)mean & 15) == 0) &&
             (!rdisp || ((uintptr_t)rdisp & 15) == 0)) {
    long long gx = (sample_size / 8 + 255) / 256;
    if (gx > 1024) gx = 1024;
    if (gx < 1) gx = 1;
    constexpr int SPT = 4;
    hipLaunchKernelGGL(fill_rows_u8_bf16_kernel<SPT>,
                       dim3((int)gx, (max_mb + SPT - 1) / SPT), dim3(256), 0,
                       s, (const uint8_t*)src, shuffled, start, count, max_mb,
                       sample_size, mean, rdisp, (uint16_t*)dst, labels,
                       labels_out, idx_out);
  } else if (max_mb <= 65535) {
    long long gx = (sample_size + 1023) / 1024;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(fill_minibatch_rows_kernel, dim3((int)gx, max_mb),
                       dim3(256), 0, s, src, src_dt, shuffled, start, count,
                       sample_size, mean, rdisp, dst, dst_dt, labels,
                       labels_out, idx_out);
  } else {
    long long total = (long long)max_mb * sample_size;
    hipLaunchKernelGGL(fill_minibatch_kernel, dim3(grid_for(total)), dim3(256), 0,
                       s, src, src_dt, shuffled, start, count, max_mb,
                       sample_size, mean, rdisp, dst, dst_dt, labels, labels_out,
                       idx_out);
  }
  return (int)launch_status(s);
}

HVK_API int hvk_mean_disp_normalize(const void* in, int in_dt, const float* mean,
                                    const float* rdisp, void* out, int out_dt,
                                    long long total, long long sample,
                                    hipStream_t s) {
  hipLaunchKernelGGL(mean_disp_kernel, dim3(grid_for(total)), dim3(256), 0, s,
                     in, in_dt, mean, rdisp, out, out_dt, total, sample);
  return (int)launch_status(s);
}

HVK_API int hvk_softmax_ce(const void* logits, int in_dt, int B, int C,
                           const int* labels, float scale, void* err, int err_dt,
                           float* probs, int* max_idx, float* metrics,
                           int* confusion, hipStream_t s) {
  int blocks = (B + 3) / 4;
  if (blocks < 1) blocks = 1;
  if (C <= 64 * 16 && hvk_gemm_variant != 65) {
    // the row in registers; one row per wave up to 4096 rows (one metric
    // atomic per block and metric)
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(softmax_ce_kernel<16>, dim3(blocks), dim3(256), 0, s,
                       logits, in_dt, B, C, labels, scale, err, err_dt, probs,
                       max_idx, metrics, confusion);
    return (int)launch_status(s);
  }
  if (blocks > 256) blocks = 256;  // >= 4 rows per wave beyond 4096 rows
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(softmax_ce_kernel<0>, dim3(blocks), dim3(256), 0, s,
                     logits, in_dt, B, C, labels, scale, err, err_dt, probs,
                     max_idx, metrics, confusion);
  return (int)launch_status(s);
}

HVK_API int hvk_mse(const void* y, int y_dt, const void* t, int t_dt, int B,
                    int D, float scale, void* err, int err_dt, float* mse_out,
                    float* metrics, int valid_rows, hipStream_t s) {
  int blocks = (B + 3) / 4;
  if (blocks > 256) blocks = 256;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(mse_kernel, dim3(blocks), dim3(256), 0, s, y, y_dt, t,
                     t_dt, B, D, scale, err, err_dt, mse_out, metrics,
                     valid_rows);
  return (int)launch_status(s);
}

HVK_API int hvk_sgd4(float* w, float* grad, float* mom, void* w_lp,
                     const void* segs, int nseg, long long total, float gscale,
                     long long zero_from, hipStream_t s) {
  if (total % 4 || ((uintptr_t)w & 15) || ((uintptr_t)grad & 15) ||
      ((uintptr_t)mom & 15) || ((uintptr_t)w_lp & 7))
    return -1;
  hipLaunchKernelGGL(sgd4_kernel, dim3(grid_for(total / 4)), dim3(256), 0, s,
                     (float4*)w, (float4*)grad, (float4*)mom, (uint2*)w_lp,
                     (const SgdSeg*)segs, nseg, total / 4, gscale, zero_from);
  return (int)launch_status(s);
}

// The same update on at most `max_blocks` workgroups (grid-stride): a
// data-parallel bucket update running on a side stream next to the backward
// GEMMs takes a few CUs instead of every free slot on the chip.
HVK_API int hvk_sgd4_grid(float* w, float* grad, float* mom, void* w_lp,
                          const void* segs, int nseg, long long total,
                          float gscale, long long zero_from, int max_blocks,
                          hipStream_t s) {
  if (total % 4 || ((uintptr_t)w & 15) || ((uintptr_t)grad & 15) ||
      ((uintptr_t)mom & 15) || ((uintptr_t)w_lp & 7) || max_blocks < 1)
    return -1;
  int g = grid_for(total / 4);
  if (g > max_blocks) g = max_blocks;
  hipLaunchKernelGGL(sgd4_kernel, dim3(g), dim3(256), 0, s, (float4*)w,
                     (float4*)grad, (float4*)mom, (uint2*)w_lp,
                     (const SgdSeg*)segs, nseg, total / 4, gscale, zero_from);
  return (int)launch_status(s);
}

HVK_API int hvk_solver(float* w, float* grad, float* s1, float* s2,
                       void* w_lp, const void* segs, int nseg,
                       long long total, float gscale, long long zero_from,
                       hipStream_t s) {
  hipLaunchKernelGGL(solver_kernel, dim3(grid_for(total)), dim3(256), 0, s, w,
                     grad, s1, s2, (uint16_t*)w_lp, (const SolverSeg*)segs,
                     nseg, total, gscale, zero_from);
  return (int)launch_status(s);
}

HVK_API int hvk_sgd(float* w, const float* grad, float* mom, void* w_lp,
                    const void* segs, int nseg, long long total, float gscale,
                    hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(total)), dim3(256), 0, s, w,
                     grad, mom, (uint16_t*)w_lp, (const SgdSeg*)segs, nseg,
                     total, gscale);
  return (int)launch_status(s);
}

// out[C][R] = in[R][C]^T (bf16) and ws[R/(64 RT)][C] = the column sums of
// each 64 RT-row slab of in (f32, in row order): the FC weight gradient's
// dY^T for the NN GEMM (K-major A, the 256 x 128 ping-pong loop) plus its
// bias gradient, in one pass over dY.  A block moves RT 64 x 64 tiles down
// the rows through LDS, each column's sum kept in the four adjacent lanes
// that hold its 16-row runs; R % (64 RT) == C % 64 == 0.
template <int RT>
__global__ void __launch_bounds__(256)
transpose_colsum_bf16_kernel(const uint16_t* __restrict__ in, int R, int C,
                             uint16_t* __restrict__ out,
                             float* __restrict__ ws) {
  __shared__ uint16_t tile[64][64 + 8];
  const int c0 = blockIdx.x * 64, t = threadIdx.x;
  const int col = t >> 2, rr = (t & 3) * 16;
  float sum = 0.f;
  for (int rt = 0; rt < RT; ++rt) {
    const int r0 = (blockIdx.y * RT + rt) * 64;
    const uint4* src =
        (const uint4*)(in + (long long)(r0 + (t >> 2)) * C + c0 + rr);
    const uint4 a = src[0], b = src[1];
    if (rt) __syncthreads();   // the last tile's reads
    *(uint4*)&tile[t >> 2][rr] = a;
    *(uint4*)&tile[t >> 2][rr + 8] = b;
    __syncthreads();
    // thread: rows rr .. rr+15 of column col, a 32-B run of the output row
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t lo = tile[rr + 2 * j][col], hi = tile[rr + 2 * j + 1][col];
      sum += bf2f(lo);
      sum += bf2f(hi);
      w[j] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
    uint4* dst = (uint4*)(out + (long long)(c0 + col) * R + r0 + rr);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
  // over the four lanes of the column (a fixed order: deterministic)
  sum += __shfl_xor(sum, 1);
  sum += __shfl_xor(sum, 2);
  if ((t & 3) == 0) ws[(long long)blockIdx.y * C + c0 + col] = sum;
}

// colsum[c] (+)= sum over the slabs of ws[slab][c], in slab order
__global__ void colsum_finish_kernel(const float* __restrict__ ws, int slabs,
                                     int C, float* __restrict__ colsum,
                                     int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float sum = 0.f;
  for (int p = 0; p < slabs; ++p) sum += ws[(long long)p * C + c];
  colsum[c] = accumulate ? colsum[c] + sum : sum;
}

// out = in^T and colsum (+)= the column sums of in; ws holds R / 64 * C
// floats.  -1 when a shape or alignment is off (the caller falls back).
HVK_API int hvk_transpose_colsum(const void* in, int R, int C, void* out,
                                 float* colsum, int accumulate, float* ws,
                                 hipStream_t s) {
  if (R % 64 || C % 64 || R <= 0 || C <= 0 || ((uintptr_t)in & 15) ||
      ((uintptr_t)out & 15) || R / 64 > 65535)
    return -1;
  // four tiles per block where the rows allow: a quarter of the slabs for
  // the finishing pass to add
  const int rt = R % 256 == 0 ? 4 : 1;
  hipLaunchKernelGGL(rt == 4 ? transpose_colsum_bf16_kernel<4>
                             : transpose_colsum_bf16_kernel<1>,
                     dim3(C / 64, R / (64 * rt)), dim3(256), 0, s,
                     (const uint16_t*)in, R, C, (uint16_t*)out, ws);
  if (colsum)
    hipLaunchKernelGGL(colsum_finish_kernel, dim3((C + 255) / 256), dim3(256),
                       0, s, (const float*)ws, R / (64 * rt), C, colsum,
                       accumulate);
  return (int)launch_status(s);
}

HVK_API int hvk_col_sum(const void* in, int dt, int R, int C, float* out,
                        float scale, hipStream_t s) {
  if (dt == DT_BF16 && C % 8 == 0 && C >= 512 &&
      ((uintptr_t)in & 15) == 0) {
    // >= ~1024 blocks: slabs of 16+ rows
    const int cgroups = (C / 8 + 63) / 64;
    int slabs = (1024 + cgroups - 1) / cgroups;
    int rps = (R + slabs - 1) / slabs;
    if (rps < 16) rps = 16;
    slabs = (R + rps - 1) / rps;
    hipLaunchKernelGGL(col_sum_bf16_wide_kernel, dim3(cgroups, slabs),
                       dim3(256), 0, s, (const uint16_t*)in, R, C, out, rps,
                       scale);
    return (int)launch_status(s);
  }
  if (dt == DT_BF16 && C % 8 == 0 && C / 8 <= 256 &&
      ((uintptr_t)in & 15) == 0) {
    // ~2048 blocks over the rows
    int rpb = (R + 2047) / 2048;
    if (rpb < 64) rpb = 64;
    int blocks = (R + rpb - 1) / rpb;
    hipLaunchKernelGGL(col_sum_bf16x8_kernel, dim3(blocks), dim3(256), 0, s,
                       (const uint16_t*)in, R, C, out, rpb, scale);
    return (int)launch_status(s);
  }
  int rpb = 256;
  // aim for >= 1024 blocks in total
  int cb = (C + 255) / 256;
  int rb = (R + rpb - 1) / rpb;
  while (rb * cb < 1024 && rpb > 16) { rpb >>= 1; rb = (R + rpb - 1) / rpb; }
  hipLaunchKernelGGL(col_sum_kernel, dim3(cb, rb), dim3(256), 0, s, in, dt, R, C,
                     out, rpb, scale);
  return (int)launch_status(s);
}

HVK_API int hvk_row_sum(const void* in, int dt, int R, int C, float* out,
                        float scale, hipStream_t s) {
  hipLaunchKernelGGL(row_sum_kernel, dim3((R + 3) / 4), dim3(256), 0, s, in, dt,
                     R, C, out, scale);
  return (int)launch_status(s);
}

HVK_API int hvk_act_fwd(const void* x, int xdt, void* y, int ydt, long long n,
                        int act, hipStream_t s) {
  if (xdt == DT_BF16 && ydt == DT_BF16 && n % 8 == 0 &&
      ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    hipLaunchKernelGGL(act_fwd_bf16x8_kernel, dim3(grid_for(n / 8)),
                       dim3(256), 0, s, (const uint16_t*)x, (uint16_t*)y,
                       n / 8, act);
    return (int)launch_status(s);
  }
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, xdt,
                     y, ydt, n, act);
  return (int)launch_status(s);
}

HVK_API int hvk_act_bwd(const void* dy, int dydt, const void* y, int ydt,
                        void* dx, int dxdt, long long n, int act, hipStream_t s) {
  if (act == ACT_STRICT_RELU && dydt == DT_BF16 && ydt == DT_BF16 &&
      dxdt == DT_BF16 && n % 8 == 0 && ((uintptr_t)dy & 15) == 0 &&
      ((uintptr_t)y & 15) == 0 && ((uintptr_t)dx & 15) == 0) {
    hipLaunchKernelGGL(relu_bwd_bf16x8_kernel, dim3(grid_for(n / 8)), dim3(256),
                       0, s, (const uint16_t*)dy, (const uint16_t*)y,
                       (uint16_t*)dx, n / 8);
  } else if (dydt == DT_BF16 && ydt == DT_BF16 && dxdt == DT_BF16 &&
             n % 8 == 0 && ((uintptr_t)dy & 15) == 0 &&
             ((uintptr_t)y & 15) == 0 && ((uintptr_t)dx & 15) == 0) {
    hipLaunchKernelGGL(act_bwd_bf16x8_kernel, dim3(grid_for(n / 8)),
                       dim3(256), 0, s, (const uint16_t*)dy,
                       (const uint16_t*)y, (uint16_t*)dx, n / 8, act);
  } else {
    hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, dy,
                       dydt, y, ydt, dx, dxdt, n, act);
  }
  return (int)launch_status(s);
}

static void launch_dropout(const void* x, int xdt, void* y, int ydt,
                           long long n, uint32_t seed, uint32_t thresh,
                           float scale, void* mask_out, const void* seed_dev,
                           long long base, hipStream_t s) {
  if (xdt == DT_BF16 && ydt == DT_BF16 && !mask_out && n % 8 == 0 &&
      ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
      hvk_gemm_variant != 66) {
    hipLaunchKernelGGL(dropout_bf16x8_kernel, dim3(grid_for(n / 8)),
                       dim3(256), 0, s, (const uint4*)x, (uint4*)y, n / 8,
                       seed, thresh, scale, (const uint32_t*)seed_dev, base);
    return;
  }
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(256), 0, s, x,
                     xdt, y, ydt, n, seed, thresh, scale, (uint8_t*)mask_out,
                     (const uint32_t*)seed_dev, base);
}

HVK_API int hvk_dropout(const void* x, int xdt, void* y, int ydt, long long n,
                        unsigned seed, float p, void* mask_out, hipStream_t s) {
  uint32_t thresh = (uint32_t)fminf(4294967295.f, p * 4294967296.f);
  float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  launch_dropout(x, xdt, y, ydt, n, seed, thresh, scale, mask_out, nullptr,
                 0ll, s);
  return (int)launch_status(s);
}

// dropout with the seed in device memory (graph-safe: the forward unit
// advances it with hvk_seed_advance inside the captured step)
HVK_API int hvk_dropout_dev(const void* x, int xdt, void* y, int ydt,
                            long long n, const void* seed_dev, float p,
                            void* mask_out, hipStream_t s) {
  uint32_t thresh = (uint32_t)fminf(4294967295.f, p * 4294967296.f);
  float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  launch_dropout(x, xdt, y, ydt, n, 0u, thresh, scale, mask_out, seed_dev,
                 0ll, s);
  return (int)launch_status(s);
}

// as hvk_dropout_dev, with the mask index of element i at base + i
HVK_API int hvk_dropout_dev_at(const void* x, int xdt, void* y, int ydt,
                               long long n, const void* seed_dev, float p,
                               long long base, hipStream_t s) {
  uint32_t thresh = (uint32_t)fminf(4294967295.f, p * 4294967296.f);
  float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  launch_dropout(x, xdt, y, ydt, n, 0u, thresh, scale, nullptr, seed_dev,
                 base, s);
  return (int)launch_status(s);
}

// ------------------------------------------------ input-derivative activations
// The Znicz standalone activations whose derivative is a function of the
// INPUT (docs/OPS.md §Activations): log (asinh), tanhlog (scaled tanh up to
// |x| = D, logarithmic growth beyond, C1-continuous), sincos (sin on even,
// cos on odd feature columns), mul (k x).  p = D for tanhlog, k for mul.
enum { XACT_LOG = 1, XACT_TANHLOG = 2, XACT_SINCOS = 3, XACT_MUL = 4 };
struct XactParams {
  int kind;
  float p, edge, slope;  // tanhlog: edge = f(D), slope = f'(D)
};
__device__ __forceinline__ XactParams xact_params(int kind, float p) {
  XactParams q{kind, p, 0.f, 0.f};
  if (kind == XACT_TANHLOG) {
    const float t = tanhf(0.6666f * p);
    q.edge = 1.7159f * t;
    q.slope = 1.7159f * 0.6666f * (1.f - t * t);
  }
  return q;
}
__device__ __forceinline__ float xact_f(float x, const XactParams& q,
                                        int odd) {
  switch (q.kind) {
    case XACT_LOG: return logf(x + sqrtf(x * x + 1.f));
    case XACT_TANHLOG: {
      const float a = fabsf(x);
      if (a <= q.p) return 1.7159f * tanhf(0.6666f * x);
      return copysignf(q.edge + q.slope * q.p * logf(a / q.p), x);
    }
    case XACT_SINCOS: return odd ? cosf(x) : sinf(x);
    case XACT_MUL: return q.p * x;
    default: return x;
  }
}
__device__ __forceinline__ float xact_d(float x, const XactParams& q,
                                        int odd) {
  switch (q.kind) {
    case XACT_LOG: return rsqrtf(x * x + 1.f);
    case XACT_TANHLOG: {
      const float a = fabsf(x);
      if (a <= q.p) {
        const float t = tanhf(0.6666f * x);
        return 1.7159f * 0.6666f * (1.f - t * t);
      }
      return q.slope * q.p / a;
    }
    case XACT_SINCOS: return odd ? -sinf(x) : cosf(x);
    case XACT_MUL: return q.p;
    default: return 1.f;
  }
}
// bwd = 0: y = f(x); bwd = 1: y = err * f'(x).  rowlen: features per sample
// (sincos parity is the column's); 8 elements per thread when vec
__global__ void xact_kernel(const void* x, int xdt, const void* err,
                            int edt, void* y, int ydt, long long n, int kind,
                            float p, long long rowlen, int bwd, int vec) {
  const XactParams q = xact_params(kind, p);
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (vec) {  // bf16, n % 8 == 0, 16-B aligned, even rowlen
    for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x;
         v < n / 8; v += stride) {
      float xv[8], o[8];
      const uint4 xr = ((const uint4*)x)[v];
      const uint16_t* xh = (const uint16_t*)&xr;
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = bf2f(xh[e]);
      if (bwd) {
        const uint4 er = ((const uint4*)err)[v];
        const uint16_t* eh = (const uint16_t*)&er;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = bf2f(eh[e]) * xact_d(xv[e], q, e & 1);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = xact_f(xv[e], q, e & 1);
      }
      ((uint4*)y)[v] = pack_bf16x8(o);
    }
    return;
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const int odd = (int)((i % rowlen) & 1);
    const float xv = ld_any(x, i, xdt);
    st_any(y, i, ydt, bwd ? ld_any(err, i, edt) * xact_d(xv, q, odd)
                          : xact_f(xv, q, odd));
  }
}

HVK_API int hvk_xact(const void* x, int xdt, const void* err, int edt,
                     void* y, int ydt, long long n, int kind, float p,
                     long long rowlen, int bwd, hipStream_t s) {
  if (kind < XACT_LOG || kind > XACT_MUL || rowlen < 1) return -1;
  const int vec = xdt == DT_BF16 && ydt == DT_BF16 &&
                  (!bwd || edt == DT_BF16) && n % 8 == 0 &&
                  rowlen % 2 == 0 && ((uintptr_t)x & 15) == 0 &&
                  ((uintptr_t)y & 15) == 0 &&
                  (!bwd || ((uintptr_t)err & 15) == 0);
  hipLaunchKernelGGL(xact_kernel, dim3(grid_for(vec ? n / 8 : n)), dim3(256),
                     0, s, x, xdt, err, edt, y, ydt, n, kind, p, rowlen, bwd,
                     vec);
  return (int)launch_status(s);
}

// ------------------------------------------------------------- gather
// y[i] = x[idx[i]] (int32 indices; idx < 0 gives 0): the depooling backward
__global__ void gather_kernel(const void* x, int xdt, const int* idx, void* y,
                              int ydt, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = idx[i];
    st_any(y, i, ydt, j >= 0 ? ld_any(x, j, xdt) : 0.f);
  }
}
HVK_API int hvk_gather(const void* x, int xdt, const int* idx, void* y,
                       int ydt, long long n, hipStream_t s) {
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, xdt,
                     idx, y, ydt, n);
  return (int)launch_status(s);
}

// seed <- hash(seed + 1): a per-step seed sequence that lives on the device
// An empty kernel that brackets a region of a kernel trace (bench.py
// --mark-steps; tools/prof_summary.py --window keeps the dispatches between
// the two markers: step-only profiles).
__global__ void hvk_trace_marker_kernel(int tag) {
  if (tag == -12345 && threadIdx.x == 1024) __builtin_trap();  // never
}
HVK_API int hvk_trace_marker(int tag, hipStream_t s) {
  hipLaunchKernelGGL(hvk_trace_marker_kernel, dim3(1), dim3(64), 0, s, tag);
  return (int)launch_status(s);
}

__global__ void seed_advance_kernel(uint32_t* seed) {
  if (threadIdx.x == 0) seed[0] = hash32(seed[0] + 1u, 0x2545F491u);
}
HVK_API int hvk_seed_advance(void* seed, hipStream_t s) {
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(64), 0, s,
                     (uint32_t*)seed);
  return (int)launch_status(s);
}

HVK_API int hvk_xorshift1024star(void* states, int n_states, int rounds,
                                 void* out, hipStream_t s) {
  int bs = 64;
  hipLaunchKernelGGL(xorshift1024_kernel, dim3((n_states + bs - 1) / bs),
                     dim3(bs), 0, s, (uint64_t*)states, n_states, rounds,
                     (uint64_t*)out);
  return (int)launch_status(s);
}

HVK_API int hvk_xorshift128plus(void* states, int n, void* out, hipStream_t s) {
  hipLaunchKernelGGL(xorshift128p_kernel, dim3((n + 255) / 256), dim3(256), 0, s,
                     (uint64_t*)states, n, (uint64_t*)out);
  return (int)launch_status(s);
}

HVK_API int hvk_u64_to_uniform(const void* in, float* out, long long n, float lo,
                               float hi, hipStream_t s) {
  hipLaunchKernelGGL(u64_to_uniform_kernel, dim3(grid_for(n)), dim3(256), 0, s,
                     (const uint64_t*)in, out, n, lo, hi);
  return (int)launch_status(s);
}

HVK_API int hvk_join(const void* const* ins, const int* lens, int nin, int dt,
                     void* out, int B, hipStream_t s) {
  if (nin > 16) return -1;
  JoinArgs a;
  int off = 0;
  for (int k = 0; k < nin; ++k) {
    a.in[k] = ins[k];
    a.len[k] = lens[k];
    a.offs[k] = off;
    off += lens[k];
  }
  long long total = (long long)B * off;
  hipLaunchKernelGGL(join_kernel, dim3(grid_for(total)), dim3(256), 0, s, a, nin,
                     dt, out, B, off);
  return (int)launch_status(s);
}

// The same image with one 16-B output chunk per lane (chunks of a pixel on
// consecutive lanes): a wave's stores cover one contiguous 1 KiB span; each
// lane gathers its 8 elements from <= 2 input rows with 2-B loads.
template <int S, int C>
__global__ void space_to_depth_chunk_kernel(const uint16_t* __restrict__ x,
                                            uint16_t* __restrict__ y, int H,
                                            int W, int pt, int pl, FastDiv fW2,
                                            FastDiv fH2, long long chunks) {
  constexpr int RUN = S * C, PIX = S * RUN, CPP = PIX / 8;
  static_assert(PIX % 8 == 0, "vector shape");
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       e < chunks; e += (long long)gridDim.x * blockDim.x) {
    const uint32_t q = (uint32_t)(e / CPP), j = (uint32_t)(e - (long long)q * CPP);
    uint32_t t, X, n, Y;
    fdivmod(q, fW2, t, X);
    fdivmod(t, fH2, n, Y);
    uint16_t v[8];
    const int iy0 = S * (int)Y - pt, ix0 = S * (int)X - pl;
    if (RUN % 4 == 0 && iy0 >= 0 && iy0 + S <= H && ix0 >= 0 &&
        ix0 + S <= W) {
      // interior pixel: each half-chunk (4 elements) lies in one row run,
      // one unaligned 8-B load (gfx950 unaligned global access)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = (int)j * 8 + 4 * h;
        const int dy = i / RUN, r = i - dy * RUN;
        __builtin_memcpy(&v[4 * h],
                         x + (((long long)n * H + iy0 + dy) * W + ix0) * C + r,
                         8);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = (int)j * 8 + k;          // element of the pixel vector
        const int dy = i / RUN, r = i - dy * RUN;
        const int dx = r / C, c = r - dx * C;
        const int iy = iy0 + dy, ix = ix0 + dx;
        const bool in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        v[k] = in ? x[(((long long)n * H + iy) * W + ix) * C + c] : (uint16_t)0;
      }
    }
    *(uint4*)(y + e * 8) = *(const uint4*)v;
  }
}

HVK_API int hvk_space_to_depth(const void* x, void* y, int N, int H, int W,
                               int C, int s, int pt, int pl, int H2, int W2,
                               hipStream_t st) {
  int C2 = s * s * C;
  if (C2 % 8) return -1;
  long long runs = (long long)N * H2 * W2 * s;
  if (runs >= (1ll << 32)) return -1;
  if (s == 4 && C == 3 && ((uintptr_t)y & 15) == 0) {
    const long long chunks = (long long)N * H2 * W2 * 6;
    hipLaunchKernelGGL((space_to_depth_chunk_kernel<4, 3>),
                       dim3(grid_for(chunks)), dim3(256), 0, st,
                       (const uint16_t*)x, (uint16_t*)y, H, W, pt, pl,
                       make_fastdiv(W2), make_fastdiv(H2), chunks);
    return (int)launch_status(st);
  }
  hipLaunchKernelGGL(space_to_depth_kernel, dim3(grid_for(runs)), dim3(256), 0,
                     st, (const uint16_t*)x, (uint16_t*)y, H, W, C, s, pt, pl,
                     H2, W2, make_fastdiv(s), make_fastdiv(W2),
                     make_fastdiv(H2), runs);
  return (int)launch_status(st);
}

// Space-to-depth weights: w [OC][KH][KW][C] -> w2 [OC][KH2][KW2][s][s][C],
// w2[o][a][b][dy][dx][c] = w[o][a*s+dy][b*s+dx][c] (0 past KH / KW): the
// stride-1 conv on the space-to-depth image equals the strided conv on x.
__global__ void s2d_weights_kernel(const uint16_t* __restrict__ w,
                                   uint16_t* __restrict__ w2, int OC, int KH,
                                   int KW, int C, int s, int KH2, int KW2) {
  const long long total = (long long)OC * KH2 * KW2 * s * s * C;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       q < total; q += (long long)gridDim.x * blockDim.x) {
    long long r = q;
    const int c = (int)(r % C); r /= C;
    const int dx = (int)(r % s); r /= s;
    const int dy = (int)(r % s); r /= s;
    const int b = (int)(r % KW2); r /= KW2;
    const int a = (int)(r % KH2);
    const int o = (int)(r / KH2);
    const int kh = a * s + dy, kw = b * s + dx;
    w2[q] = (kh < KH && kw < KW)
                ? w[(((long long)o * KH + kh) * KW + kw) * C + c]
                : (uint16_t)0;
  }
}

// The inverse fold of the weight gradient: dw[o][kh][kw][c] += dw2[o][kh/s]
// [kw/s][kh%s][kw%s][c]; clear = 1 zeroes all of dw2 (padded taps too), so
// the next step's split-K atomics start from zeros without a memset.
__global__ void s2d_grad_fold_kernel(float* __restrict__ dw2,
                                     float* __restrict__ dw, int OC, int KH,
                                     int KW, int C, int s, int KH2, int KW2,
                                     int clear) {
  const long long total = (long long)OC * KH2 * KW2 * s * s * C;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
       q < total; q += (long long)gridDim.x * blockDim.x) {
    long long r = q;
    const int c = (int)(r % C); r /= C;
    const int dx = (int)(r % s); r /= s;
    const int dy = (int)(r % s); r /= s;
    const int b = (int)(r % KW2); r /= KW2;
    const int a = (int)(r % KH2);
    const int o = (int)(r / KH2);
    const int kh = a * s + dy, kw = b * s + dx;
    const float v = dw2[q];
    if (kh < KH && kw < KW)
      dw[(((long long)o * KH + kh) * KW + kw) * C + c] += v;
    if (clear) dw2[q] = 0.f;
  }
}

HVK_API int hvk_s2d_weights(const void* w, void* w2, int OC, int KH, int KW,
                            int C, int s, hipStream_t st) {
  const int KH2 = (KH + s - 1) / s, KW2 = (KW + s - 1) / s;
  const long long total = (long long)OC * KH2 * KW2 * s * s * C;
  hipLaunchKernelGGL(s2d_weights_kernel, dim3(grid_for(total)), dim3(256), 0,
                     st, (const uint16_t*)w, (uint16_t*)w2, OC, KH, KW, C, s,
                     KH2, KW2);
  return (int)launch_status(st);
}

HVK_API int hvk_s2d_grad_fold(float* dw2, float* dw, int OC, int KH, int KW,
                              int C, int s, int clear, hipStream_t st) {
  const int KH2 = (KH + s - 1) / s, KW2 = (KW + s - 1) / s;
  const long long total = (long long)OC * KH2 * KW2 * s * s * C;
  hipLaunchKernelGGL(s2d_grad_fold_kernel, dim3(grid_for(total)), dim3(256), 0,
                     st, dw2, dw, OC, KH, KW, C, s, KH2, KW2, clear);
  return (int)launch_status(st);
}

HVK_API int hvk_cast(const void* in, int idt, void* out, int odt, long long n,
                     float scale, hipStream_t s) {
  if (idt == DT_F32 && odt == DT_BF16 && scale == 1.f && n % 4 == 0 &&
      ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 7) == 0) {
    hipLaunchKernelGGL(f32_to_bf16x4_kernel, dim3(grid_for(n / 4)), dim3(256), 0,
                       s, (const float4*)in, (uint2*)out, n / 4);
  } else {
    hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(256), 0, s, in, idt,
                       out, odt, n, scale);
  }
  return (int)launch_status(s);
}

// ---------------------------------------------------------------------------
// Direct convolution for tiny reductions (C * KH * KW <= 64, OC <= 64: LeNet's
// conv1, C = 1, 5 x 5 -> 20).  The implicit GEMM spends a whole 128 x 64 tile
// with ONE 64-deep K step on such a layer (latency bound: 0.37 ms at b4096
// for 2.4 GFLOP); here a lane computes every output channel of one pixel
// from the K taps, the weights broadcast from LDS as f32 [k][oc].
template <int OCMAX>
__global__ __launch_bounds__(256) void conv_fwd_direct_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
    const float* __restrict__ bias, uint16_t* __restrict__ y, int N, int H,
    int W, int C, int OC, int KH, int KW, int sy, int sx, int pt, int pl,
    int OH, int OW, int act, FastDiv fOW, FastDiv fOH) {
  __shared__ float ws[64 * 64];
  __shared__ float bs[64];
  const int K = KH * KW * C;
  for (int i = threadIdx.x; i < OC * K; i += blockDim.x) {
    const int oc = i / K, k = i - oc * K;
    ws[k * OCMAX + oc] = bf2f(w[i]);
  }
  for (int i = threadIdx.x; i < OCMAX; i += blockDim.x)
    bs[i] = (bias && i < OC) ? bias[i] : 0.f;
  __syncthreads();
  const uint32_t P = (uint32_t)N * OH * OW;
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += gridDim.x * blockDim.x) {
    uint32_t t, ow, n, oh;
    fdivmod(p, fOW, t, ow);
    fdivmod(t, fOH, n, oh);
    float acc[OCMAX];
#pragma unroll
    for (int o = 0; o < OCMAX; ++o) acc[o] = bs[o];
    const int ih0 = (int)oh * sy - pt, iw0 = (int)ow * sx - pl;
    const uint16_t* img = x + (long long)n * H * W * C;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = ih0 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = iw0 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const uint16_t* px = img + ((long long)ih * W + iw) * C;
        const float* wk = ws + ((kh * KW + kw) * C) * OCMAX;
        for (int c = 0; c < C; ++c) {
          const float xv = bf2f(px[c]);
#pragma unroll
          for (int o = 0; o < OCMAX; ++o) acc[o] += xv * wk[c * OCMAX + o];
        }
      }
    }
#pragma unroll
    for (int o = 0; o < OCMAX; o += 8) act_fwd8(acc + o, act);
    uint16_t* out = y + (long long)p * OC;
    if ((OC & 1) == 0) {
#pragma unroll
      for (int o = 0; o < OCMAX; o += 2)
        if (o < OC)
          *(uint32_t*)(out + o) = (uint32_t)f2bf(acc[o]) |
                                  ((uint32_t)f2bf(acc[o + 1]) << 16);
    } else {
#pragma unroll
      for (int o = 0; o < OCMAX; ++o)
        if (o < OC) out[o] = f2bf(acc[o]);
    }
  }
}

HVK_API int hvk_conv_fwd_direct(const void* X, const void* Wt,
                                const float* bias, void* Y, int N, int H,
                                int W, int C, int OC, int KH, int KW, int sy,
                                int sx, int pt, int pl, int OH, int OW,
                                int act, hipStream_t s) {
  const int K = KH * KW * C;
  if (K > 64 || OC > 64 || OC < 1 || ((uintptr_t)Y & 3) ||
      (long long)N * OH * OW >= (1ll << 31))
    return -1;
  const long long P = (long long)N * OH * OW;
  const int grid = grid_for(P);
  auto k = OC <= 16 ? conv_fwd_direct_kernel<16>
         : OC <= 32 ? conv_fwd_direct_kernel<32>
                    : conv_fwd_direct_kernel<64>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, (const uint16_t*)X,
                     (const uint16_t*)Wt, bias, (uint16_t*)Y, N, H, W, C, OC,
                     KH, KW, sy, sx, pt, pl, OH, OW, act, make_fastdiv(OW),
                     make_fastdiv(OH));
  return (int)launch_status(s);
}

