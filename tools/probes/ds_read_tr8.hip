// Probe: what ds_read_b64_tr_b8 delivers on gfx950.  LDS holds a 64 x 64
// byte image with byte (r, c) = (r & 15) * 16 + (c & 15) and a second plane
// telling r / c >> 4 apart; each lane supplies the address of row
// (lane & 63) (64-B rows) at column 8 * ((lane >> 4) & 3)... and prints
// the 8 bytes it receives, so the transposition pattern can be read off.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((address_space(3))) i32x2 lds_i32x2;

__global__ void probe(int mode, unsigned char* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) {
    const int r = i / 64, c = i % 64;
    s[i] = (unsigned char)((r & 15) * 16 + (c & 15));
  }
  __syncthreads();
  const int l = threadIdx.x;
  int addr;
  if (mode == 0)        // lane l -> row l, column 0
    addr = l * 64;
  else if (mode == 1)   // lane l -> row (l & 15), column 8 * (l >> 4)
    addr = (l & 15) * 64 + 8 * (l >> 4);
  else                  // lane l -> row (l >> 3), column 8 * (l & 7)
    addr = (l >> 3) * 64 + 8 * (l & 7);
  i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)(s + addr));
  const unsigned char* b = (const unsigned char*)&v;
  for (int j = 0; j < 8; ++j) out[(mode * 64 + l) * 8 + j] = b[j];
}

int main() {
  unsigned char* d;
  unsigned char h[3 * 64 * 8];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  for (int m = 0; m < 3; ++m) hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, m, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int m = 0; m < 3; ++m) {
    printf("mode %d\n", m);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d:", l);
      for (int j = 0; j < 8; ++j) {
        const int v = h[(m * 64 + l) * 8 + j];
        printf(" r%02d c%02d", v >> 4, v & 15);
      }
      printf("\n");
    }
  }
  hipFree(d);
  return 0;
}
