// Dependent LDS lookup chain latency vs occupancy / chains per lane
// (development microbenchmark; not part of the product).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

template <int CHAINS>
__global__ __launch_bounds__(256) void chain(const uint32_t *g, uint32_t *out, int steps, int pad_rows) {
  extern __shared__ uint32_t tab[];  // 257*16 words + padding (occupancy knob)
  for (int i = threadIdx.x; i < 257 * 16; i += 256) tab[i] = g[i];
  __syncthreads();
  uint32_t e[CHAINS], x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) { e[c] = 0; x[c] = threadIdx.x * 2654435761u + c * 97 + blockIdx.x; }
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      x[c] = x[c] * 1664525u + 1013904223u;
      const uint32_t nib = (x[c] >> 26) << 2;  // nibble * 4
      e[c] = *(const uint32_t *)((const char *)tab + (e[c] >> 16) + nib);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r += e[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  // random FSM-like table: entry = next_row_offset << 16 (rows of 64 B)
  std::vector<uint32_t> h(257 * 16);
  uint32_t s = 12345;
  for (auto &w : h) { s = s * 1103515245u + 12345u; w = ((s >> 8) % 257) * 64u << 16; }
  uint32_t *g, *out;
  hipMalloc(&g, h.size() * 4); hipMemcpy(g, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  int ncu = 256; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipMalloc(&out, (size_t)ncu * 16 * 256 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int steps = 4096;
  for (int bpc : {1, 2, 4, 8}) {
    const size_t lds = 160 * 1024 / bpc - 1024;  // limits blocks per CU
    for (int chains : {1, 2, 4}) {
      auto k = chains == 1 ? chain<1> : chains == 2 ? chain<2> : chain<4>;
      const int grid = ncu * bpc;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, g, out, 64, 0);
      hipEventRecord(a);
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, g, out, steps, 0);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      const double cyc = ms * 1e-3 * 2.4e9;
      printf("blocks/CU %d (waves/SIMD %d) chains %d: %.1f cycles per step per wave, %.2f lookups/cycle/CU\n",
             bpc, bpc, chains, cyc / steps, (double)grid * 256 * steps * chains / (cyc * ncu));
    }
  }
  return 0;
}
