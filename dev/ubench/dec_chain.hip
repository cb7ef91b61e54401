// Microbenchmark (development): the window decoder's lock-step lookup
// iteration with its real per-step VALU -- an 11-bit peek-table lookup per
// symbol, the 64-bit bit buffer shifted by the entry's length, a predicated
// refill every four lookups, the sixteen entries packed with v_perm and one
// 16-byte stage write per iteration -- run as 1, 2 or 3 independent chains
// per lane (strings decoded in lock-step by one lane) at 2-5 resident
// workgroups of four waves per CU.  Question it answers: does a lane with two
// strings in flight (their lookups issued together) decode more symbols per
// second than the shipped one-string lane at four waves per SIMD?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

constexpr int kW = 11;

struct Chain {
  uint64_t bb;
  int nb;
  uint32_t x;  // word source (xorshift: the decoder's F/B word queue stands here)
};

__device__ __forceinline__ uint32_t next_word(uint32_t &x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

template <int C>
__global__ __launch_bounds__(256) void dec_chain(const uint32_t *g, uint32_t *out, int iters) {
  extern __shared__ uint32_t lds[];
  uint32_t *tab = lds;                       // 2^11 entries: len | sym << 8
  uint8_t *stage = reinterpret_cast<uint8_t *>(lds + (1 << kW));  // 16 B per lane and chain
  for (int i = threadIdx.x; i < (1 << kW); i += 256) tab[i] = g[i];
  __syncthreads();
  Chain ch[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    ch[c].x = (threadIdx.x * 2654435761u) ^ (c * 0x9E3779B9u) ^ (blockIdx.x * 40503u) | 1u;
    ch[c].bb = ((uint64_t)next_word(ch[c].x) << 32) | next_word(ch[c].x);
    ch[c].nb = 64;
  }
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t ev[C][16];
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
#pragma unroll
      for (int c = 0; c < C; ++c) {  // refill when <= 32 bits are buffered (predicated)
        const bool r = (uint32_t)ch[c].nb <= 32u;
        const uint32_t w = next_word(ch[c].x);
        ch[c].bb |= (uint64_t)(r ? w : 0u) << ((uint32_t)(32 - ch[c].nb) & 63u);
        ch[c].nb += r ? 32 : 0;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int c = 0; c < C; ++c) {  // one lookup per chain, issued together
          const uint32_t hi = (uint32_t)(ch[c].bb >> 32);
          const uint32_t e = tab[hi >> (32 - kW)];
          const uint32_t f = ch[c].nb >= (int)(e & 0xFFu) ? e : 0x80u;
          ch[c].bb <<= (f & 63u);
          ch[c].nb -= (int)(f & 0xFFu);
          ev[c][4 * grp + k] = f;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      ch[c].nb &= 127;
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = __builtin_amdgcn_perm(__builtin_amdgcn_perm(ev[c][4 * j + 3], ev[c][4 * j + 2], 0x0c0c0501u),
                                     __builtin_amdgcn_perm(ev[c][4 * j + 1], ev[c][4 * j], 0x0c0c0501u),
                                     0x05040100u);
      *reinterpret_cast<uint4 *>(stage + 16u * (threadIdx.x * C + c)) = make_uint4(o[0], o[1], o[2], o[3]);
      acc += o[0] ^ o[3];
    }
  }
  __syncthreads();
  const uint4 v = *reinterpret_cast<const uint4 *>(stage + 16u * threadIdx.x);
  out[blockIdx.x * 256 + threadIdx.x] = acc + v.x + v.w;
}

int main() {
  std::vector<uint32_t> h(1 << kW);
  uint32_t s = 12345;
  for (auto &w : h) {  // lengths 5-8 bits (alphabet A's codes average 6.6), symbol byte
    s = s * 1103515245u + 12345u;
    w = (5u + ((s >> 9) & 3u)) | (((s >> 16) & 0xFFu) << 8);
  }
  uint32_t *g, *out;
  (void)hipMalloc(&g, h.size() * 4);
  (void)hipMemcpy(g, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipMalloc(&out, (size_t)ncu * 8 * 256 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 2048;
  const void *fns[3] = {(const void *)dec_chain<1>, (const void *)dec_chain<2>, (const void *)dec_chain<3>};
  for (int c = 1; c <= 3; ++c) {
    hipFuncAttributes at;
    (void)hipFuncGetAttributes(&at, fns[c - 1]);
    for (int bpc : {2, 3, 4, 5}) {
      const size_t lds = 160 * 1024 / bpc - 512;  // limits resident workgroups per CU
      const int grid = ncu * bpc;
      auto launch = [&](int n) {
        if (c == 1) hipLaunchKernelGGL(dec_chain<1>, dim3(grid), dim3(256), lds, 0, g, out, n);
        if (c == 2) hipLaunchKernelGGL(dec_chain<2>, dim3(grid), dim3(256), lds, 0, g, out, n);
        if (c == 3) hipLaunchKernelGGL(dec_chain<3>, dim3(grid), dim3(256), lds, 0, g, out, n);
      };
      launch(16);
      (void)hipEventRecord(a);
      launch(iters);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      const double sym = (double)grid * 256 * c * 16.0 * iters;
      const int fits = at.numRegs <= 512 / bpc;  // VGPRs per lane for bpc waves per SIMD
      printf("{\"chains\": %d, \"waves_per_simd\": %d, \"vgprs\": %d, \"fits\": %d, \"ms\": %.3f, "
             "\"symbols_per_s\": %.4e}\n", c, bpc, at.numRegs, fits, ms, sym / (ms * 1e-3));
    }
  }
  return 0;
}
