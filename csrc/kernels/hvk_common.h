// hvk_common.h - shared device helpers for the veles_amd HIP kernel library
// (gfx950 / CDNA4 only: wave64, MFMA, 160 KiB LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HVK_API extern "C" __attribute__((visibility("default")))

// Status of the launch just enqueued on stream s.  hipGetLastError() also
// returns an error left pending on this thread by an earlier, abandoned
// graph capture (hipErrorStreamCaptureInvalidated after a capture broken by
// a synchronising op); a launch on a stream that is NOT capturing did not
// cause it, so it is not reported as this launch's failure (the entry
// points would otherwise fail the next kernel of an eager pass).
inline hipError_t launch_status(hipStream_t s) {
  const hipError_t e = hipGetLastError();
  if (e == hipErrorStreamCaptureInvalidated ||
      e == hipErrorStreamCaptureUnsupported ||
      e == hipErrorStreamCaptureImplicit) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusActive;
    if (hipStreamIsCapturing(s, &st) == hipSuccess &&
        st == hipStreamCaptureStatusNone)
      return hipSuccess;
  }
  return e;
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace hvk {

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// Round-to-nearest-even; hipcc lowers the cast to v_cvt_pk_bf16_f32 which
// keeps NaNs NaN (MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

// two floats -> packed bf16 pair (lo = a) in ONE v_cvt_pk_bf16_f32 (RNE,
// NaN-preserving); a per-element cast + shift/or costs three instructions
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ uint4 pack_bf16x8(const float* v) {
  return make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                    pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}
// Strict ReLU on a packed bf16 pair as 16-bit integers: a bf16 is > 0
// exactly when its bit pattern is a positive int16, so max(x, 0) and the
// derivative mask (x > 0 ? 0xffff : 0) are one / three packed-i16 ops per
// two values instead of an unpack, compare and select per value.
// relu(bf16(x)) == bf16(relu(x)); masking gives +0 where x * 0 gave -0.
typedef __attribute__((ext_vector_type(2))) short s16x2_t;
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t p) {
  const s16x2_t z = {0, 0};
  return __builtin_bit_cast(
      uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, p), z));
}
// (0 -sat y) is negative exactly when y > 0 (y = -32768 saturates to
// +32767); its sign spread over the lane is the mask
__device__ __forceinline__ uint32_t relu_mask_bf16x2(uint32_t y) {
  const s16x2_t z = {0, 0}, sh = {15, 15};
  const s16x2_t t =
      __builtin_elementwise_sub_sat(z, __builtin_bit_cast(s16x2_t, y));
  return __builtin_bit_cast(uint32_t, t >> sh);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Fast unsigned division by a runtime-constant divisor (n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.s = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.m);
  return (hi + n) >> f.s;
}
__device__ __forceinline__ void fdivmod(uint32_t n, const FastDiv& f,
                                        uint32_t& q, uint32_t& r) {
  q = fdiv(n, f);
  r = n - q * f.d;
}

// Activation codes (Znicz semantics, docs/OPS.md):
//   0 linear, 1 tanh (1.7159*tanh(0.6666x)), 2 relu (softplus: log(1+e^x)),
//   3 strict relu max(0,x), 4 sigmoid, 5 log (asinh-like, see OPS.md)
enum Act { ACT_LINEAR = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_STRICT_RELU = 3,
           ACT_SIGMOID = 4 };

__device__ __forceinline__ float act_fwd(float x, int act) {
  switch (act) {
    case ACT_TANH: return 1.7159f * tanhf(0.6666f * x);
    case ACT_RELU: return x > 15.f ? x : log1pf(__expf(x));
    case ACT_STRICT_RELU: return x > 0.f ? x : 0.f;
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    default: return x;
  }
}
// act_fwd over NV values with ONE switch on the (wave-uniform) code: the
// per-element switch of an unrolled loop costs a branch ladder per element
template <int NV>
__device__ __forceinline__ void act_fwd_n(float* v, int act) {
  switch (act) {
    case ACT_LINEAR: return;
    case ACT_STRICT_RELU:
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q] = v[q] > 0.f ? v[q] : 0.f;
      return;
    case ACT_TANH:
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q] = 1.7159f * tanhf(0.6666f * v[q]);
      return;
    case ACT_RELU:
#pragma unroll
      for (int q = 0; q < NV; ++q)
        v[q] = v[q] > 15.f ? v[q] : log1pf(__expf(v[q]));
      return;
    case ACT_SIGMOID:
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q] = 1.f / (1.f + __expf(-v[q]));
      return;
    default:
      return;
  }
}
__device__ __forceinline__ void act_fwd8(float* v, int act) {
  act_fwd_n<8>(v, act);
}
// derivative expressed through the activation OUTPUT y
__device__ __forceinline__ float act_bwd(float y, int act) {
  switch (act) {
    case ACT_TANH: return 0.6666f * 1.7159f - (0.6666f / 1.7159f) * y * y;
    case ACT_RELU: return 1.f - __expf(-y);
    case ACT_STRICT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: return y * (1.f - y);
    default: return 1.f;
  }
}

}  // namespace hvk

namespace hvk {
// v[q] *= act_bwd(y[q], act) for NV values, one switch (see act_fwd_n)
template <int NV>
__device__ __forceinline__ void act_bwd_mul_n(float* v, const float* y,
                                              int act) {
  switch (act) {
    case ACT_LINEAR: return;
    case ACT_STRICT_RELU:
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q] *= y[q] > 0.f ? 1.f : 0.f;
      return;
    default:
#pragma unroll
      for (int q = 0; q < NV; ++q) v[q] *= act_bwd(y[q], act);
      return;
  }
}
__device__ __forceinline__ void act_bwd_mul8(float* v, const float* y,
                                             int act) {
  act_bwd_mul_n<8>(v, y, act);
}
}  // namespace hvk
