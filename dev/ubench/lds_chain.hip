// Dependent LDS lookup chain: latency and throughput vs occupancy and chains
// per lane (development microbenchmark; not part of the product).
// Table: FSM-shaped, 257 rows x 16 dwords, entry = next_row_offset << 16.
// Nibble source: a per-chain register rotated by 4 bits per step (one
// v_alignbit), so the loop is LDS-bound, not VALU-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

template <int CHAINS, bool STORE>
__global__ __launch_bounds__(256) void chain(const uint32_t *g, uint32_t *out, int steps) {
  extern __shared__ uint32_t tab[];  // 257*16 words + ring + padding
  for (int i = threadIdx.x; i < 257 * 16; i += 256) tab[i] = g[i];
  __syncthreads();
  uint8_t *ring = reinterpret_cast<uint8_t *>(tab + 257 * 16) + threadIdx.x * 48;
  uint32_t e[CHAINS], x[CHAINS], k = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) {
    e[c] = 0;
    x[c] = (threadIdx.x * 2654435761u) ^ (c * 0x9E3779B9u) ^ (blockIdx.x * 40503u);
  }
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      x[c] = __builtin_amdgcn_alignbit(x[c], x[c], 4);  // rotate by 4
      const uint32_t nib = x[c] & 0x3Cu;
      e[c] = *(const uint32_t *)((const char *)tab + (e[c] >> 16) + nib);
      if (STORE) {
        ring[k & 31] = (uint8_t)e[c];
        k += (e[c] >> 8) & 1u;
      }
    }
  }
  uint32_t r = k;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r += e[c];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  std::vector<uint32_t> h(257 * 16);
  uint32_t s = 12345;
  for (auto &w : h) {
    s = s * 1103515245u + 12345u;
    w = (((s >> 8) % 257) * 64u << 16) | ((s >> 3) & 0x1FFu);
  }
  uint32_t *g, *out;
  (void)hipMalloc(&g, h.size() * 4);
  (void)hipMemcpy(g, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipMalloc(&out, (size_t)ncu * 16 * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int steps = 4096;
  double best = 0, w4c1 = 0;  // lookups/s: best of all shapes; 4 waves/SIMD, one chain per lane
  for (int store = 0; store < 2; ++store)
    for (int bpc : {2, 4, 8}) {
      const size_t lds = 160 * 1024 / bpc - 1024;  // limits blocks per CU
      for (int chains : {1, 2, 4}) {
        auto k = store ? (chains == 1 ? chain<1, true> : chains == 2 ? chain<2, true> : chain<4, true>)
                       : (chains == 1 ? chain<1, false> : chains == 2 ? chain<2, false> : chain<4, false>);
        const int grid = ncu * bpc;
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, g, out, 64);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, g, out, steps);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("store %d waves/SIMD %d chains %d: %6.1f cyc/step/wave  %.2f lookups/cyc/CU\n",
               store, bpc, chains, cyc / steps,
               (double)grid * 256 * steps * chains / (cyc * ncu));
        const double rate = (double)grid * 256 * steps * chains / (ms * 1e-3);
        if (rate > best) best = rate;
        if (!store && bpc == 4 && chains == 1) w4c1 = rate;
      }
    }
  printf("{\"chained_lookups_per_s_best\": %.4e, \"chained_lookups_per_s_4waves_1chain\": %.4e, \"cus\": %d}\n",
         best, w4c1, ncu);
  return 0;
}
