// qh_common.h -- device-side types, tables and helpers shared by the
// QPACK Huffman kernels (included once, from qh_device.hip).
#pragma once

namespace qhk {

// Development knobs -- the QHUFF_* environment variables other than
// QHUFF_VERBOSE, and the kernels' store probes (QHUFF_DEBUG bits that skip or
// misplace output stores) -- exist only in development builds (make dev,
// make stamps, make var ...).  The product library's output never depends on
// its environment, as the reference codec's does not (huffman.c:87-124).
#if defined(QH_DEV_VARIANTS) || defined(QH_STAMPS) || defined(QH_DEV_KNOBS_ON)
#define QH_DEV_KNOBS 1
#else
#define QH_DEV_KNOBS 0
#endif
// A development probe bit of a kernel's dbg word: constant false in the
// product build, so the probe's branch compiles out.
#define QH_PROBE(d, bits) (QH_DEV_KNOBS && ((d) & (bits)) != 0u)

// Phase timers for kernel development (make stamps -> libqhuff_stamps.so):
// wave 0 of every workgroup adds s_memtime deltas per phase slot.  Compiled
// out of the product library.
#ifdef QH_STAMPS
__device__ unsigned long long g_stamps[16];
// per block (blockIdx.x < 8192): start (realtime), lifetime (realtime,
// 100 MHz), HW_ID register, lifetime in shader clocks (s_memtime)
__device__ unsigned long long g_blk[8192][4];
#define QH_ST_INIT()                                                         \
  unsigned long long _st_t = __builtin_amdgcn_s_memtime(), _st_a[16] = {0};
#define QH_ST(k)                                                             \
  {                                                                          \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();             \
    _st_a[k] += _n - _st_t;                                                  \
    _st_t = _n;                                                              \
  }
#define QH_ST_COUNT(k, v) (_st_a[k] += (v))
#define QH_ST_FLUSH()                                                        \
  if (threadIdx.x == 0)                                                      \
    for (int _k = 0; _k < 16; ++_k)                                          \
      if (_st_a[_k]) atomicAdd(&g_stamps[_k], _st_a[_k]);
// The same as an object a helper function can take by reference.
struct StampAcc {
  unsigned long long t, a[16], t0, r0;
  __device__ void init() {
    t = t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 16; ++k) a[k] = 0;
  }
  __device__ void st(int k) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    a[k] += n - t;
    t = n;
  }
  __device__ void count(int k, unsigned long long v) { a[k] += v; }
  __device__ void wait_mem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
  // slots 0..6 and 11 only (a helper's own phases), from thread 0
  __device__ void add_slots() {
    if (threadIdx.x == 0)
      for (int k = 0; k < 12; ++k)
        if (a[k] && (k < 7 || k == 11)) atomicAdd(&g_stamps[k], a[k]);
  }
  __device__ void flush() {  // slots 12, 13: block lifetime in realtime (100 MHz) / memtime
    const unsigned long long life = __builtin_amdgcn_s_memrealtime() - r0;
    a[12] += life;
    a[13] += __builtin_amdgcn_s_memtime() - t0;
    if (threadIdx.x == 0) {
      atomicMax(&g_stamps[14], life);  // slot 14: the longest block
      // slots 7, 8, 9: ~(earliest start), latest start, latest end (realtime)
      atomicMax(&g_stamps[7], ~r0);
      atomicMax(&g_stamps[8], r0);
      atomicMax(&g_stamps[9], r0 + life);
      if (blockIdx.x < 8192) {
        g_blk[blockIdx.x][0] = r0;
        g_blk[blockIdx.x][1] = life;
        // HW_ID, and the XCD (XCC_ID) in bits 32..34
        g_blk[blockIdx.x][2] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                               (unsigned long long)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u) << 32;
        g_blk[blockIdx.x][3] = __builtin_amdgcn_s_memtime() - t0;
      }
    }
    if (threadIdx.x == 0)
      for (int k = 0; k < 16; ++k)
        if (a[k] && k != 14) atomicAdd(&g_stamps[k], a[k]);
  }
};
#else
struct StampAcc {
  __device__ void init() {}
  __device__ void st(int) {}
  __device__ void count(int, unsigned long long) {}
  __device__ void wait_mem() {}
  __device__ void add_slots() {}
  __device__ void flush() {}
};
#define QH_ST_INIT()
#define QH_ST(k)
#define QH_ST_COUNT(k, v)
#define QH_ST_FLUSH()
#endif

// ---------------------------------------------------------------------------
// device-side types and helpers
// ---------------------------------------------------------------------------

struct SpanIn {
  uint64_t off;
  uint32_t len;
  uint32_t flags;
};
struct SpanOut {
  uint64_t off;
  uint32_t len;
  int32_t status;
};
static_assert(sizeof(SpanIn) == 16 && sizeof(qh_span_in) == 16, "span_in");
static_assert(sizeof(SpanOut) == 16 && sizeof(qh_span_out) == 16, "span_out");

// Device-side accumulators for qh_batch_stats (+ scan bookkeeping).
struct DevStats {
  unsigned long long n;
  unsigned long long in_bytes;
  unsigned long long out_bytes;
  unsigned long long dst_bytes;
  unsigned long long n_errors;
  unsigned long long scan_timeouts;
  // window decoders: lock-step iterations (16 table lookups each) run by
  // lanes, and by waves (each wave's longest lane, per window)
  unsigned long long lane_steps;
  unsigned long long wave_steps;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16-byte vector with 1-byte alignment: gfx950 runs global_load_dwordx4 on
// unaligned addresses (unaligned access mode), so a string can be fetched
// from its own first byte without a head-alignment loop.
typedef u32x4 u32x4_ua __attribute__((aligned(1)));
typedef uint64_t u64_ua __attribute__((aligned(1)));
typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint16_t u16_ua __attribute__((aligned(1)));

// Host images of the tables uploaded to every context (qh_tables.h lists).
#define QH_SYM_PAIR(nbits, code) nbits, code,
const uint32_t kSymPacked[QH_NSYM * 2] = {QH_SYM_LIST(QH_SYM_PAIR)};
#define QH_FSM_WORD(w) w,
#define QH_FSM_FLAT(...) __VA_ARGS__
const uint32_t kFsmPacked[QH_NSTATE * 16] = {QH_FSM_ROWS(QH_FSM_FLAT, QH_FSM_WORD)};

constexpr int kBlock = 256;
constexpr uint32_t kFsmWords = QH_NSTATE * 16;  // 4112 words = 16,448 B
constexpr uint32_t kFlagSymBit = 17;             // QH_FLAG_SYM << 16

__device__ __forceinline__ uint32_t lds_word(const uint32_t *base,
                                             uint32_t byte_off) {
  return *reinterpret_cast<const uint32_t *>(
      reinterpret_cast<const char *>(base) + byte_off);
}

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations are
// complete (lgkmcnt(0)), its global loads and stores may stay in flight.
// (__syncthreads() also waits for every outstanding global store -- a round
// trip to memory per barrier in a kernel that streams its output.)  The
// asm's memory clobber keeps the compiler from moving memory accesses
// across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Wave-wide reductions with DPP row shifts and row broadcasts (no LDS round
// trips: a __shfl_xor step is a ds_bpermute and a wait on it).  Every lane of
// the wave must be active; the result is lane 63's, read into every lane.
// A lane whose DPP source lies outside its row keeps `ident` (bound_ctrl off).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v, uint32_t ident) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v, uint64_t ident) {
  return (uint64_t)dpp_u32<CTRL, ROWS>((uint32_t)v, (uint32_t)ident) |
         (uint64_t)dpp_u32<CTRL, ROWS>((uint32_t)(v >> 32), (uint32_t)(ident >> 32)) << 32;
}
__device__ __forceinline__ uint32_t lane63_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t lane63_u64(uint64_t v) {
  return (uint64_t)lane63_u32((uint32_t)v) | (uint64_t)lane63_u32((uint32_t)(v >> 32)) << 32;
}
// Inclusive scan (lane i: op over lanes 0..i); T is uint32_t or uint64_t.
template <typename T, typename F>
__device__ __forceinline__ T wave_incl_dpp(T v, T ident, F op) {
  if constexpr (sizeof(T) == 4) {
    v = op(v, dpp_u32<0x111, 0xf>(v, ident));  // row_shr:1
    v = op(v, dpp_u32<0x112, 0xf>(v, ident));  // row_shr:2
    v = op(v, dpp_u32<0x114, 0xf>(v, ident));  // row_shr:4
    v = op(v, dpp_u32<0x118, 0xf>(v, ident));  // row_shr:8
    v = op(v, dpp_u32<0x142, 0xa>(v, ident));  // row_bcast:15
    v = op(v, dpp_u32<0x143, 0xc>(v, ident));  // row_bcast:31
  } else {
    v = op(v, dpp_u64<0x111, 0xf>(v, ident));
    v = op(v, dpp_u64<0x112, 0xf>(v, ident));
    v = op(v, dpp_u64<0x114, 0xf>(v, ident));
    v = op(v, dpp_u64<0x118, 0xf>(v, ident));
    v = op(v, dpp_u64<0x142, 0xa>(v, ident));
    v = op(v, dpp_u64<0x143, 0xc>(v, ident));
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_add_u32(uint32_t v) {
  return wave_incl_dpp<uint32_t>(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint64_t wave_scan_add_u64(uint64_t v) {
  return wave_incl_dpp<uint64_t>(v, 0ull, [](uint64_t a, uint64_t b) { return a + b; });
}
__device__ __forceinline__ uint64_t wave_add_u64(uint64_t v) {
  return lane63_u64(wave_incl_dpp<uint64_t>(v, 0ull, [](uint64_t a, uint64_t b) { return a + b; }));
}
__device__ __forceinline__ uint32_t wave_add_u32(uint32_t v) {
  return lane63_u32(wave_scan_add_u32(v));
}
__device__ __forceinline__ uint32_t wave_max_u32_all(uint32_t v) {
  return lane63_u32(wave_incl_dpp<uint32_t>(v, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; }));
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  return lane63_u64(wave_incl_dpp<uint64_t>(v, ~0ull, [](uint64_t a, uint64_t b) { return a < b ? a : b; }));
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  return lane63_u64(wave_incl_dpp<uint64_t>(v, 0ull, [](uint64_t a, uint64_t b) { return a > b ? a : b; }));
}

// Block-level sum of per-thread counters -> one atomic per block.
__device__ __forceinline__ void block_add(unsigned long long *dst,
                                          unsigned long long v,
                                          unsigned long long *lds4) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds4[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += lds4[w];
    if (s) atomicAdd(dst, s);
  }
  __syncthreads();
}

// Fetch the 16 bytes at p + pos where fewer than 16 may belong to the
// string (tail): the last 16 bytes of the string are loaded and shifted so
// that byte 0 of the result is byte `pos` of the string.  Strings shorter
// than 16 bytes are gathered bytewise.  Bytes past the string are zero.
__device__ __forceinline__ u32x4 load_tail(const uint8_t *p, uint32_t pos,
                                           uint32_t len) {
  const uint32_t rem = len - pos;  // 0 < rem < 16
  u32x4 v = {0, 0, 0, 0};
  if (len >= 16) {
    const u32x4 w = *reinterpret_cast<const u32x4_ua *>(p + len - 16);
    // move bytes [16 - rem, 16) of w down to [0, rem): 128-bit shift right
    const uint32_t s = 8 * (16 - rem);  // 8..120 bits
    const uint64_t lo64 = (uint64_t)w.x | ((uint64_t)w.y << 32);
    const uint64_t hi64 = (uint64_t)w.z | ((uint64_t)w.w << 32);
    uint64_t rlo, rhi;
    if (s >= 64) {
      rlo = hi64 >> (s - 64);
      rhi = 0;
    } else {
      rlo = (lo64 >> s) | (hi64 << (64 - s));
      rhi = hi64 >> s;
    }
    v.x = (uint32_t)rlo; v.y = (uint32_t)(rlo >> 32);
    v.z = (uint32_t)rhi; v.w = (uint32_t)(rhi >> 32);
  } else {
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
      if (k < rem) o[k >> 2] |= (uint32_t)p[pos + k] << (8 * (k & 3));
    v.x = o[0]; v.y = o[1]; v.z = o[2]; v.w = o[3];
  }
  return v;
}

// ---------------------------------------------------------------------------
// decoupled look-back (single-pass prefix over tiles)
// ---------------------------------------------------------------------------
// Lane-path scan words: {flag:2, value:62}, zeroed by a memset per launch.
constexpr uint64_t kStA = 1ull << 62;
constexpr uint64_t kStP = 2ull << 62;
constexpr uint64_t kStMask = (1ull << 62) - 1;

// Output slot of a string of `len` encoded bytes in a batch decode
// (include/qhuff.h): the reference's estimate_decode_length
// (huffman.h:113-115) + 16 spare bytes, rounded up to 64 bytes so that every
// slot starts 64-byte aligned (decoders write whole 64-byte sectors).
__host__ __device__ __forceinline__ uint64_t qh_dec_slot(uint32_t len) {
  return ((uint64_t)len * 8 / 5 + 16 + 63) & ~(uint64_t)63;
}

// LDS image of the decode FSM (qh_lane_dec.inc): rows padded to 17 dwords so
// that entry (row r, nibble v) lies in bank (17 r + v) mod 32 -- with
// 16-dword rows every lane reading nibble v would hit one of two banks, and
// header text has a few dominant high nibbles (0x4-0x7).
constexpr uint32_t kFsmRowWords = 17;
constexpr uint32_t kFsmLdsWords = QH_NSTATE * kFsmRowWords;  // 17,476 B

}  // namespace qhk
