// fp8_common.h - OCP fp8 (e4m3 / e5m2) quantisation helpers shared by the
// fp8 GEMM epilogues (gemm_fp8.hip) and the kernels that produce an fp8
// layer's input (pooling, pool_lrn.hip): delayed per-tensor scaling from a
// scaler state row, saturating packs, and the fused-quantisation output
// (Q8) a producer writes beside its bf16 result.
#pragma once
#include "hvk_common.h"

namespace hvk {

// A scaler state is float st[hist + 1]: amax history, then the running amax
// of the current step.  scale = fmax_eff / max(history) (1 when empty); the
// quantizer multiplies by it and the GEMM epilogue divides by sA * sB.
__device__ __forceinline__ float fp8_scale(const float* st, int hist,
                                           float fmax_eff) {
  float m = 0.f;
  for (int i = 0; i < hist; ++i) m = fmaxf(m, st[i]);
  return m > 0.f ? fmax_eff / m : 1.f;
}

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c,
                                              float d, int fmt) {
  int v;
  if (fmt == 0) {
    v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  } else {
    v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  }
  return (uint32_t)v;
}

__device__ __forceinline__ float sat(float v, float lim) {
  return fminf(fmaxf(v, -lim), lim);
}

// Fused quantisation output: q (same element indexing as the bf16 result)
// = sat(bf16(result) * scale(st)) in format fmt; the workgroup's amax of
// |bf16(result)| goes to one of 32 shards of `shard` (32 floats apart),
// folded into the scaler's current amax by the registry's roll.
struct Q8 {
  uint8_t* q;          // nullptr: off
  const float* st;
  float* shard;
  float fmax;
  int fmt, hist;
};

// 8 bf16 results (packed) at element idx: their fp8 copy, amax updated
__device__ __forceinline__ void q8_store8(const Q8& z, long long idx,
                                          const uint4& ob, float qs,
                                          float& amax) {
  const uint32_t w4[4] = {ob.x, ob.y, ob.z, ob.w};
  float r[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r[2 * q] = __uint_as_float(w4[q] << 16);
    r[2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
  }
  const float lim = z.fmt == 0 ? 448.f : 57344.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(r[q]));
  uint2 v;
  v.x = pack4_fp8(sat(r[0] * qs, lim), sat(r[1] * qs, lim),
                  sat(r[2] * qs, lim), sat(r[3] * qs, lim), z.fmt);
  v.y = pack4_fp8(sat(r[4] * qs, lim), sat(r[5] * qs, lim),
                  sat(r[6] * qs, lim), sat(r[7] * qs, lim), z.fmt);
  *(uint2*)(z.q + idx) = v;
}

// one atomicMax per workgroup (256 threads) into shard blockIdx.x & 31;
// red: 4 floats of LDS.  Every thread of the workgroup must call it.
__device__ __forceinline__ void q8_block_amax(const Q8& z, float amax,
                                              float* red) {
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
    if (m > 0.f)
      atomicMax((unsigned int*)(z.shard + (blockIdx.x & 31) * 32),
                __float_as_uint(m));
  }
}

}  // namespace hvk
