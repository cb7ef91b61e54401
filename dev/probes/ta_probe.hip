// Development probe: how fast can a wave read 2^20 strings of 8-256 bytes
// (config 3's plaintext) when each lane owns one string?
//   mode 0: lane l loads 16-byte piece k of its own string (a 4-deep ring of
//           registers, as qh_k_enc_lanes does): 64 distinct lines per load
//   mode 1: cooperative: load instruction q, lane l takes quarter (l & 3) of
//           the 64-byte group of string 16 q + (l >> 2): 16 lines per load;
//           the groups land in LDS (global_load_lds_dwordx4), each lane then
//           reads its own 64 bytes
//   mode 2: coalesced streaming of the same bytes (each wave 1 KB per load)
// Each mode sums the bytes into a checksum so nothing is optimised away.
// Build: hipcc --offload-arch=gfx950 -O3 -o ta_probe ta_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hsum(u32x4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__device__ __forceinline__ void dma16(const uint8_t *g, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// strings: off[i], len[i]; wave takes 64 consecutive strings per window
__global__ __launch_bounds__(256) void k_lane(const uint8_t *src, const uint64_t *off,
                                              const uint32_t *len, uint64_t n, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwv = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (uint64_t w = gw * 64; w < n; w += nwv * 64) {
    const uint64_t i = w + lane;
    if (i >= n) break;
    const uint8_t *p = src + (off[i] & ~15ull);
    const uint32_t nst = (uint32_t)(((off[i] & 15) + len[i] + 15) >> 4), last = nst - 1;
    auto piece = [&](uint32_t k) { return *reinterpret_cast<const u32x4 *>(p + 16 * min(k, last)); };
    u32x4 q0 = piece(0), q1 = piece(1), q2 = piece(2), q3 = piece(3);
    for (uint32_t st = 0;; st += 4) {
      acc += hsum(q0); q0 = piece(st + 4); if (st + 1 >= nst) break;
      acc += hsum(q1); q1 = piece(st + 5); if (st + 2 >= nst) break;
      acc += hsum(q2); q2 = piece(st + 6); if (st + 3 >= nst) break;
      acc += hsum(q3); q3 = piece(st + 7); if (st + 4 >= nst) break;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_coop(const uint8_t *src, const uint64_t *off,
                                              const uint32_t *len, uint64_t n, uint32_t *sink) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4][2][4096];
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wid, nwv = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (uint64_t w = gw * 64; w < n; w += nwv * 64) {
    // lane l's string for the loads: quarter (l & 3) of string 16 q + (l >> 2)
    const uint64_t i = w + lane;
    const bool own = i < n;
    const uint64_t base = own ? (off[i] & ~15ull) : 0;
    const uint32_t nst = own ? (uint32_t)(((off[i] & 15) + len[i] + 15) >> 4) : 0;
    const uint32_t ngr = (nst + 3) / 4;  // 64-byte groups
    uint32_t wg = ngr;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wg = max(wg, (uint32_t)__shfl_xor((int)wg, o));
    // each load instruction q serves strings 16 q .. 16 q + 15 (4 lanes each)
    uint64_t gb[4];
    uint32_t gl[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s = 16 * q + (lane >> 2);
      gb[q] = __shfl(base, s);
      gl[q] = __shfl(nst, s);
    }
    uint32_t b = 0;
    auto issue = [&](uint32_t g, uint32_t bb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t k = min(4 * g + (lane & 3), gl[q] ? gl[q] - 1 : 0u);
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)&buf[wid][bb][1024 * q]);
        dma16(src + gb[q] + 16 * k, lds);
      }
    };
    issue(0, 0);
    for (uint32_t g = 0; g < wg; ++g, b ^= 1) {
      if (g + 1 < wg) {
        issue(g + 1, b ^ 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_wave_barrier();
      // my group: instruction q = lane >> 4, lanes 4 (lane & 15) .. + 3
      const u32x4 *my = reinterpret_cast<const u32x4 *>(&buf[wid][b][1024 * (lane >> 4) + 64 * (lane & 15)]);
      if (g < ngr) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += hsum(my[k]);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const uint8_t *src, uint64_t bytes, uint32_t *sink) {
  const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
  const uint64_t nv = bytes / 16;
  uint32_t acc = 0;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < nv; k += (uint64_t)gridDim.x * 256 * 4) {
    u32x4 a = s[k];
    u32x4 b = k + gridDim.x * 256 < nv ? s[k + gridDim.x * 256] : a;
    u32x4 c = k + 2ull * gridDim.x * 256 < nv ? s[k + 2ull * gridDim.x * 256] : a;
    u32x4 d = k + 3ull * gridDim.x * 256 < nv ? s[k + 3ull * gridDim.x * 256] : a;
    acc += hsum(a) + hsum(b) + hsum(c) + hsum(d);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
  const uint64_t n = 1ull << 20;
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  uint64_t x = 0x5EED0003, at = 0;
  for (uint64_t i = 0; i < n; ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    len[i] = 8 + (uint32_t)((x >> 33) % 249);
    off[i] = at;
    at += len[i];
  }
  uint8_t *d_src;
  uint64_t *d_off;
  uint32_t *d_len, *d_sink;
  CK(hipMalloc(&d_src, at + 4096));
  CK(hipMemset(d_src, 0x61, at + 4096));
  CK(hipMalloc(&d_off, n * 8));
  CK(hipMalloc(&d_len, n * 4));
  CK(hipMalloc(&d_sink, 64));
  CK(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 3; ++mode) {
    for (int grid : {1024, 2048}) {
      float best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a, 0));
        if (mode == 0) hipLaunchKernelGGL(k_lane, dim3(grid), dim3(256), 0, 0, d_src, d_off, d_len, n, d_sink);
        if (mode == 1) hipLaunchKernelGGL(k_coop, dim3(grid), dim3(256), 0, 0, d_src, d_off, d_len, n, d_sink);
        if (mode == 2) hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, d_src, at, d_sink);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep) best = ms < best ? ms : best;
      }
      printf("mode %d grid %d: %.1f us (%.2f TB/s of %llu bytes)\n", mode, grid, best * 1e3,
             at / (best * 1e-3) / 1e12, (unsigned long long)at);
    }
  }
  return 0;
}
