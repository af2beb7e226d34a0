// Probe: does buffer_load_dwordx4 ... lds (LDS-DMA through a buffer
// descriptor) write ZEROS to LDS for lanes whose voffset is out of range
// (>= num_records)?  The branch-free conv DMA addressing relies on it.
// Build: hipcc --offload-arch=gfx950 -O2 buffer_lds_oob.hip -o probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k(const unsigned short* p, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned short s[512];
  for (int i = threadIdx.x; i < 512; i += 64) s[i] = 0xBEEF;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p, (short)0, (int)0x80000000u, 0x00020000);
  // even lanes: in range (16 B each), odd lanes: offset 0x80000000 (OOB)
  unsigned voff = (threadIdx.x & 1) ? 0x80000000u : threadIdx.x * 16u;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)s, 16, voff, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = s[i];
}

int main() {
  std::vector<unsigned short> h(64 * 8);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned short)(i + 1);
  unsigned short* d;
  unsigned* o;
  hipMalloc(&d, h.size() * 2);
  hipMalloc(&o, 512 * 4);
  hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  std::vector<unsigned> r(512);
  hipMemcpy(r.data(), o, 512 * 4, hipMemcpyDeviceToHost);
  int bad = 0, zeros = 0;
  for (int lane = 0; lane < 64; ++lane)
    for (int e = 0; e < 8; ++e) {
      unsigned v = r[lane * 8 + e];
      unsigned want = (lane & 1) ? 0u : (unsigned)(lane * 8 + e + 1);
      if (v != want) ++bad;
      if ((lane & 1) && v == 0) ++zeros;
    }
  printf("buffer_lds_oob: %s (mismatches %d, OOB zeros %d of 256)\n",
         bad ? "FAIL" : "OK", bad, zeros);
  return bad ? 1 : 0;
}
