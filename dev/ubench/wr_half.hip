// Write-granularity probe (development tool): do 64-byte writes that cover
// half of a 128-byte line make the L2 read from memory?  Four kernels over a
// 1 GiB buffer, each 16 bytes per lane:
//   full    every line whole (8 lanes a line)
//   half0   the first 64 bytes of every line
//   half1   the second 64 bytes of every line (after half0: the line's other half)
//   q32     32 bytes of every 64 (every other 32-byte sector)
// Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE; prints event times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct alignas(16) V4 { uint32_t x, y, z, w; };

__global__ void k_full(V4 *d, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) d[i] = V4{(uint32_t)i, 1, 2, 3};
}
// every line: 16-byte pieces [h*4, h*4+4) of its 8
__global__ void k_half(V4 *d, uint64_t nlines, uint32_t h) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t line = t >> 2, q = t & 3;
  if (line < nlines) d[line * 8 + h * 4 + q] = V4{(uint32_t)t, 1, 2, 3};
}
// every 64-byte half: its first 32 bytes
__global__ void k_q32(V4 *d, uint64_t nhalves) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t hh = t >> 1, q = t & 1;
  if (hh < nhalves) d[hh * 4 + q] = V4{(uint32_t)t, 1, 2, 3};
}

int main() {
  const uint64_t bytes = 1ull << 30, n16 = bytes / 16, nlines = bytes / 128;
  V4 *d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, auto launch, double wbytes) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-6s %8.1f us  %7.1f GB/s written\n", name, ms * 1e3, wbytes / (ms * 1e-3) / 1e9);
  };
  const int B = 256;
  run("full", [&] { hipLaunchKernelGGL(k_full, dim3((n16 + B - 1) / B), dim3(B), 0, 0, d, n16); }, (double)bytes);
  run("half0", [&] { hipLaunchKernelGGL(k_half, dim3((nlines * 4 + B - 1) / B), dim3(B), 0, 0, d, nlines, 0u); },
      bytes / 2.0);
  run("half1", [&] { hipLaunchKernelGGL(k_half, dim3((nlines * 4 + B - 1) / B), dim3(B), 0, 0, d, nlines, 1u); },
      bytes / 2.0);
  run("q32", [&] { hipLaunchKernelGGL(k_q32, dim3((bytes / 64 * 2 + B - 1) / B), dim3(B), 0, 0, d, bytes / 64); },
      bytes / 2.0);
  hipFree(d);
  return 0;
}
