// FETCH_SIZE calibration for per-lane 16-byte loads (development tool).
// Each kernel reads every byte of a 256 MiB buffer exactly once:
//   coal   a wave reads 1 KiB contiguous per instruction (16 B a lane)
//   lane   lane l of the grid reads its own 2 KiB region, 16 B per step, in
//          order (the regions of neighbouring lanes are 2 KiB apart)
//   lane64 the same with 64-byte steps (four 16-byte loads per step)
// The sum of the loaded words goes to out[] so no load is dead.
// Run under rocprofv3 --pmc FETCH_SIZE; prints event times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct alignas(16) V4 { uint32_t x, y, z, w; };

__global__ void k_coal(const V4 *d, uint64_t n16, uint32_t *out) {
  uint32_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const V4 v = d[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_lane(const V4 *d, uint32_t steps, uint32_t *out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const V4 *p = d + t * steps;
  uint32_t s = 0;
  for (uint32_t k = 0; k < steps; ++k) {
    const V4 v = p[k];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[t] = s;
}
__global__ void k_lane64(const V4 *d, uint32_t steps, uint32_t *out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const V4 *p = d + t * steps;
  uint32_t s = 0;
  for (uint32_t k = 0; k < steps; k += 4) {
    const V4 a = p[k], b = p[k + 1], c = p[k + 2], e = p[k + 3];
    s += a.x ^ b.y ^ c.z ^ e.w ^ a.w ^ b.x ^ c.y ^ e.z;
  }
  out[t] = s;
}

int main() {
  const uint64_t bytes = 256ull << 20, n16 = bytes / 16;
  const uint32_t region = 2048, steps = region / 16;
  const uint64_t lanes = bytes / region;  // 131072
  V4 *d = nullptr;
  uint32_t *out = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&out, 4u << 20) != hipSuccess) return 1;
  hipMemset(d, 1, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-7s %8.1f us  %7.1f GB/s read\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  run("coal", [&] { hipLaunchKernelGGL(k_coal, dim3(4096), dim3(256), 0, 0, d, n16, out); });
  run("lane", [&] { hipLaunchKernelGGL(k_lane, dim3(lanes / 256), dim3(256), 0, 0, d, steps, out); });
  run("lane64", [&] { hipLaunchKernelGGL(k_lane64, dim3(lanes / 256), dim3(256), 0, 0, d, steps, out); });
  hipFree(d);
  hipFree(out);
  return 0;
}
