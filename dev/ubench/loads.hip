// Microbenchmark: per-lane string reads, unaligned vs aligned 16-B loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef u4 u4u __attribute__((aligned(1)));

// each lane sums the bytes of its string using 16-B loads at the string start (unaligned)
__global__ void k_unaligned(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t* out) {
  uint32_t s = blockIdx.x * 256 + threadIdx.x; if (s >= n) return;
  const uint8_t* p = src + off[s]; uint32_t l = len[s], acc = 0;
  for (uint32_t i = 0; i + 16 <= l; i += 16) { u4 v = *(const u4u*)(p + i); acc += v.x ^ v.y ^ v.z ^ v.w; }
  out[s] = acc;
}
// same, but loads are 16-B aligned chunks covering the string
__global__ void k_aligned(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t* out) {
  uint32_t s = blockIdx.x * 256 + threadIdx.x; if (s >= n) return;
  uint64_t o = off[s]; uint32_t l = len[s], acc = 0;
  const uint8_t* p = src + (o & ~15ull);
  uint32_t a = o & 15;
  for (uint32_t i = 0; i + 16 <= l + a; i += 16) { u4 v = *(const u4*)(p + i); acc += v.x ^ v.y ^ v.z ^ v.w; }
  out[s] = acc;
}
// aligned, 4 chunks in flight per lane
__global__ void k_aligned4(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint32_t n, uint32_t* out) {
  uint32_t s = blockIdx.x * 256 + threadIdx.x; if (s >= n) return;
  uint64_t o = off[s]; uint32_t l = len[s], acc = 0;
  const uint8_t* p = src + (o & ~15ull);
  uint32_t a = o & 15;
  uint32_t i = 0;
  for (; i + 64 <= l + a; i += 64) {
    u4 v0 = *(const u4*)(p + i), v1 = *(const u4*)(p + i + 16), v2 = *(const u4*)(p + i + 32), v3 = *(const u4*)(p + i + 48);
    acc += (v0.x ^ v1.y ^ v2.z ^ v3.w) + (v0.w ^ v1.x) + (v2.y ^ v3.z);
  }
  for (; i + 16 <= l + a; i += 16) { u4 v = *(const u4*)(p + i); acc += v.x ^ v.y ^ v.z ^ v.w; }
  out[s] = acc;
}
// coalesced baseline: block reads its contiguous byte range 16 B per lane
__global__ void k_coalesced(const uint8_t* src, uint64_t nbytes, uint32_t* out) {
  uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; uint32_t acc = 0;
  for (; i + 16 <= nbytes; i += (uint64_t)gridDim.x * 256 * 16) { u4 v = *(const u4*)(src + i); acc += v.x ^ v.y ^ v.z ^ v.w; }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
int main() {
  const uint32_t n = 1 << 20; std::vector<uint64_t> off(n); std::vector<uint32_t> len(n); uint64_t t = 0;
  srand(1); for (uint32_t i = 0; i < n; ++i) { len[i] = 7 + rand() % 204; off[i] = t; t += len[i]; }
  uint8_t* d_src; uint64_t* d_off; uint32_t *d_len, *d_out; hipMalloc(&d_src, t + 64); hipMemset(d_src, 1, t + 64);
  hipMalloc(&d_off, n * 8); hipMalloc(&d_len, n * 4); hipMalloc(&d_out, n * 4 * 4);
  hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice); hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int k = 0; k < 4; ++k) {
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
      hipEventRecord(a);
      if (k == 0) k_unaligned<<<n / 256, 256>>>(d_src, d_off, d_len, n, d_out);
      if (k == 1) k_aligned<<<n / 256, 256>>>(d_src, d_off, d_len, n, d_out);
      if (k == 2) k_aligned4<<<n / 256, 256>>>(d_src, d_off, d_len, n, d_out);
      if (k == 3) k_coalesced<<<2048, 256>>>(d_src, t, d_out);
      hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    const char* nm[] = {"unaligned16", "aligned16", "aligned16x4", "coalesced"};
    printf("%-12s %8.1f us  %7.1f GB/s\n", nm[k], best * 1e3, t / (best * 1e-3) / 1e9);
  }
  return 0;
}
