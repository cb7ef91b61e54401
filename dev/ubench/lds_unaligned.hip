// Microbenchmark (development): does ds_read_b32 at a byte-unaligned LDS
// address return the 4 bytes at that address on gfx950, and at what cost?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(uint32_t *out, uint32_t misalign, uint32_t iters, unsigned long long *cyc) {
  __shared__ uint8_t buf[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) buf[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t base = (uint32_t)(uintptr_t)&buf[0];
  uint32_t addr = lane * 24 + misalign;
  uint32_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(base + addr + (acc & 0)) : "memory");
    acc += v;
    addr = (addr + 4) & 4095;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  // correctness: one read per lane at lane*24+misalign
  uint32_t a = base + lane * 24 + misalign, v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  if (buf[lane] == 0xEE && lane == 99) v = 0;  // keep buf alive
  out[blockIdx.x * blockDim.x + threadIdx.x] = v + (acc & 0) * 0;
}

int main() {
  uint32_t *d; unsigned long long *c;
  hipMalloc(&d, 256 * 4); hipMalloc(&c, 8);
  for (uint32_t mis = 0; mis < 4; ++mis) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mis, 1000, c);
    uint32_t h[64]; unsigned long long cy;
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int l = 0; l < 64; ++l) {
      uint32_t a = l * 24 + mis, e = 0;
      for (int b = 0; b < 4; ++b) e |= (uint32_t)((uint8_t)((a + b) * 7 + 3)) << (8 * b);
      if (h[l] != e) { ok = 0; if (l < 2) printf("  lane %d got %08x want %08x\n", l, h[l], e); }
    }
    printf("misalign %u: %s, %.1f cycles per dependent ds_read_b32\n", mis, ok ? "correct" : "WRONG", cy / 1000.0);
  }
  return 0;
}
