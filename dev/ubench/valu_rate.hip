// Microbenchmark (development): issue cost of the decoder's VALU
// instructions on gfx950 -- eight independent chains per wave, one wave per
// SIMD, s_memtime around 256 x 8 instructions.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP8(X) X X X X X X X X

template <int K>
__global__ void k(uint64_t *out, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  uint32_t a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
  uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3, b4 = a4, b5 = a5, b6 = a6, b7 = a7;
  const uint32_t s = seed & 7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 256; ++it) {
    if (K == 0) {  // v_add_u32
      asm volatile(REP8("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                        "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));
    } else if (K == 1) {  // v_lshlrev_b64
      asm volatile(REP8("v_lshlrev_b64 %0, %8, %0\n\tv_lshlrev_b64 %1, %8, %1\n\tv_lshlrev_b64 %2, %8, %2\n\tv_lshlrev_b64 %3, %8, %3\n\t"
                        "v_lshlrev_b64 %4, %8, %4\n\tv_lshlrev_b64 %5, %8, %5\n\tv_lshlrev_b64 %6, %8, %6\n\tv_lshlrev_b64 %7, %8, %7\n\t")
                   : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) : "v"(s));
    } else if (K == 2) {  // v_alignbit_b32
      asm volatile(REP8("v_alignbit_b32 %0, %0, %1, %8\n\tv_alignbit_b32 %1, %1, %2, %8\n\tv_alignbit_b32 %2, %2, %3, %8\n\tv_alignbit_b32 %3, %3, %4, %8\n\t"
                        "v_alignbit_b32 %4, %4, %5, %8\n\tv_alignbit_b32 %5, %5, %6, %8\n\tv_alignbit_b32 %6, %6, %7, %8\n\tv_alignbit_b32 %7, %7, %0, %8\n\t")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));
    } else if (K == 3) {  // v_cndmask_b32 with vcc
      asm volatile("v_cmp_gt_u32 vcc, %8, %0\n\t"
                   REP8("v_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %1, %1, %2, vcc\n\tv_cndmask_b32 %2, %2, %3, vcc\n\tv_cndmask_b32 %3, %3, %4, vcc\n\t"
                        "v_cndmask_b32 %4, %4, %5, vcc\n\tv_cndmask_b32 %5, %5, %6, vcc\n\tv_cndmask_b32 %6, %6, %7, vcc\n\tv_cndmask_b32 %7, %7, %0, vcc\n\t")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s) : "vcc");
    } else {  // v_perm_b32
      asm volatile(REP8("v_perm_b32 %0, %0, %1, %8\n\tv_perm_b32 %1, %1, %2, %8\n\tv_perm_b32 %2, %2, %3, %8\n\tv_perm_b32 %3, %3, %4, %8\n\t"
                        "v_perm_b32 %4, %4, %5, %8\n\tv_perm_b32 %5, %5, %6, %8\n\tv_perm_b32 %6, %6, %7, %8\n\tv_perm_b32 %7, %7, %0, %8\n\t")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (uint32_t)(b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7) == 12345) out[1] = 1;
}

int main() {
  uint64_t *d;
  hipMalloc(&d, 16);
  const char *names[] = {"v_add_u32", "v_lshlrev_b64", "v_alignbit_b32", "v_cndmask_b32", "v_perm_b32"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int kk = 0; kk < 5; ++kk) {
      uint64_t c = 0;
      switch (kk) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d, 3u); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d, 3u); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d, 3u); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, d, 3u); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, d, 3u); break;
      }
      hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-16s %.2f memtime ticks per instruction (one wave)\n", names[kk], c / (256.0 * 64));
    }
  }
  return 0;
}
