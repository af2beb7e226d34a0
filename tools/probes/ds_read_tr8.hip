// Probe: what ds_read_b64_tr_b8 returns on gfx950.  LDS byte at offset a holds
// a & 0xff (and offset / 256 in a second run); lane l supplies address 8 * l
// (its own 8-byte chunk).  Prints, per lane, the 8 source offsets it received
// - the permutation defines the instruction for the fp8 transposed loader.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(2))) int i32x2;

__global__ void probe(uint32_t* out, int hi) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64)
    lds[i] = hi ? (uint8_t)(i >> 8) : (uint8_t)(i & 0xff);
  __syncthreads();
  const int l = threadIdx.x;
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) i32x2*)(lds + 8 * l));
  out[2 * l] = v[0];
  out[2 * l + 1] = v[1];
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 512);
  uint32_t h[2][128];
  for (int hi = 0; hi < 2; ++hi) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, hi);
    hipMemcpy(h[hi], d, 512, hipMemcpyDeviceToHost);
  }
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) {
      const int w = j / 4, b = j % 4;
      const int lo = (h[0][2 * l + w] >> (8 * b)) & 0xff;
      const int hb = (h[1][2 * l + w] >> (8 * b)) & 0xff;
      printf(" %4d", hb * 256 + lo);
    }
    printf("\n");
  }
  hipFree(d);
  return 0;
}
