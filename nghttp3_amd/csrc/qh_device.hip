// qh_device.hip -- QPACK Huffman batch engine for MI355X (gfx950, CDNA4).
//
// Replaces the hot loops of nghttp3's lib/nghttp3_qpack_huffman.c
// (encode_count :34-43, encode :45-78, decode :87-124) for batches of whole
// header-field strings.  Integer/byte work only: no MFMA.  Design notes and
// the roofline accounting are in DESIGN.md.
//
// Kernels (all launched on the context's stream):
//   qh_k_scan<SLOTS>     decoupled look-back exclusive scan over strings:
//                        decode slot offsets (sum of len*8/5, the reference's
//                        rcbuf sizing, huffman.h:113-115).
//   qh_k_decode          one lane per string; 4-bit FSM (huffman.c:103-114)
//                        with the 257x16 table in LDS; 16-B input fetches;
//                        dword-aligned output stores.
//   qh_k_count           hlen = encode_count per string (huffman.c:34-43).
//   qh_k_scan<HLEN>      dense encode offsets (prefix sum of hlen).
//   qh_k_encode          one lane per string; 64-bit accumulator with
//                        big-endian 32-bit flushes and EOS-prefix padding
//                        (huffman.c:53-75).
//   qh_k_synth_*         deterministic synthetic inputs (bench/tests only).

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/qhuff.h"
#include "qh_tables.h"

#define QH_VERSION "0.1.0"

namespace qhk {

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
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16-byte vector with 1-byte alignment: gfx950 runs global_load_dwordx4 on
// unaligned addresses (unaligned access mode), so a string can be fetched
// from its own first byte without a head-alignment loop.
typedef u32x4 u32x4_ua __attribute__((aligned(1)));

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

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
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

// Byte-exact output stream built from aligned dword stores.  The first and
// the last partial dword of a string are written byte by byte so that
// neighbouring strings (owned by other lanes) are never touched.
struct Sink {
  uint32_t *wp;      // current aligned dword
  uint64_t acc;      // pending bytes, stream order = little-endian
  uint32_t nb;       // pending bits (multiple of 8), includes head gap
  uint32_t head;     // leading bytes of *wp that belong to someone else
};

// Pointer arithmetic (not integer casts) keeps the global address space, so
// stores stay global_store_* rather than flat_* (flat ops also count on
// lgkmcnt and would make every LDS lookup of the FSM wait for them).
__device__ __forceinline__ void sink_init(Sink &s, uint8_t *p) {
  s.head = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  s.wp = reinterpret_cast<uint32_t *>(p - s.head);
  s.acc = 0;
  s.nb = s.head * 8;
}

__device__ __forceinline__ void sink_flush(Sink &s) {  // needs nb >= 32
  const uint32_t w = (uint32_t)s.acc;
  if (s.head) {
    uint8_t *b = reinterpret_cast<uint8_t *>(s.wp);
    for (uint32_t k = s.head; k < 4; ++k) b[k] = (uint8_t)(w >> (8 * k));
    s.head = 0;
  } else {
    *s.wp = w;
  }
  ++s.wp;
  s.acc >>= 32;
  s.nb -= 32;
}

__device__ __forceinline__ void sink_finish(Sink &s) {
  const uint32_t nbytes = s.nb >> 3;
  uint8_t *b = reinterpret_cast<uint8_t *>(s.wp);
  for (uint32_t k = s.head; k < nbytes; ++k)
    b[k] = (uint8_t)(s.acc >> (8 * k));
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
// decoupled look-back exclusive scan over strings
// ---------------------------------------------------------------------------

// Decode slot of a string with `len` encoded bytes: the reference's
// estimate_decode_length (huffman.h:113-115) rounded up to 16 bytes.
__host__ __device__ __forceinline__ uint64_t qh_slot_size(uint32_t len) {
  return (((uint64_t)len * 8 / 5) + 15) & ~uint64_t(15);
}

constexpr int kScanItems = 8;
constexpr int kScanTile = kBlock * kScanItems;  // 2048 strings per tile
constexpr uint64_t kStA = 1ull << 62;           // aggregate available
constexpr uint64_t kStP = 2ull << 62;           // inclusive prefix available
constexpr uint64_t kStMask = (1ull << 62) - 1;

enum ScanMode { SCAN_SLOTS = 0, SCAN_HLEN = 1 };

// SCAN_SLOTS: value(i) = in[i].len * 8 / 5, result -> out[i].off
// SCAN_HLEN:  value(i) = out[i].len (hlen from qh_k_count), result -> out[i].off
template <int MODE>
__global__ __launch_bounds__(kBlock) void qh_k_scan(
    const SpanIn *__restrict__ in, SpanOut *__restrict__ out, uint64_t n,
    uint64_t *__restrict__ tile_state, uint32_t *__restrict__ tile_ctr,
    DevStats *__restrict__ stats) {
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_wave[kBlock / 64];
  __shared__ uint64_t s_prefix;
  if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t base = (uint64_t)tile * kScanTile + threadIdx.x * kScanItems;

  uint64_t local[kScanItems];
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const uint64_t i = base + k;
    uint64_t v = 0;
    if (i < n) {
      if (MODE == SCAN_SLOTS)
        v = qh_slot_size(in[i].len);
      else
        v = out[i].len;
    }
    local[k] = sum;
    sum += v;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(incl, o);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wave[wid] = incl;
  __syncthreads();
  uint64_t wave_off = 0, agg = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w) {
    if (w < wid) wave_off += s_wave[w];
    agg += s_wave[w];
  }
  if (threadIdx.x == 0) {
    uint64_t prefix = 0;
    if (tile == 0) {
      st_relaxed(&tile_state[0], kStP | agg);
    } else {
      st_relaxed(&tile_state[tile], kStA | agg);
      int64_t j = (int64_t)tile - 1;
      uint32_t spins = 0;
      while (j >= 0) {
        const uint64_t s = ld_relaxed(&tile_state[j]);
        const uint64_t flag = s & ~kStMask;
        if (flag == 0) {
          // predecessor has not published yet; its tile id was drawn
          // before ours, so it is running.  Bounded for safety.
          if (++spins > (1u << 26)) {
            atomicAdd(&stats->scan_timeouts, 1ull);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        prefix += s & kStMask;
        if (flag == kStP) break;
        --j;
      }
      st_relaxed(&tile_state[tile], kStP | (prefix + agg));
    }
    s_prefix = prefix;
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    if (MODE == SCAN_SLOTS && tile == ntiles - 1) {
      stats->dst_bytes = prefix + agg;
    }
  }
  __syncthreads();
  const uint64_t thread_off = s_prefix + wave_off + incl - sum;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const uint64_t i = base + k;
    if (i < n) out[i].off = thread_off + local[k];
  }
}

// ---------------------------------------------------------------------------
// tile scheduling: one block = 256 strings, one lane each, ranked by length
// ---------------------------------------------------------------------------

struct TileLds {
  uint32_t hist[kBlock];
  uint32_t order[kBlock];
  uint32_t wsum[kBlock / 64];
};

// Counting-sort the tile's strings by length (longest first, 16-byte
// buckets) so that the 64 lanes of a wave get similar trip counts; returns
// the tile-relative index of the string this thread processes.  The
// permutation only changes which lane decodes a string, never its output.
__device__ __forceinline__ uint32_t tile_rank_by_len(uint32_t len, TileLds &t) {
  const uint32_t tid = threadIdx.x;
  const uint32_t key = 255u - min(len >> 4, 255u);
  t.hist[tid] = 0;
  __syncthreads();
  const uint32_t r = atomicAdd(&t.hist[key], 1u);
  __syncthreads();
  const uint32_t h = t.hist[tid];
  uint32_t incl = h;
  const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o);
    if (lane >= o) incl += x;
  }
  if (lane == 63) t.wsum[wid] = incl;
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; ++w)
    if (w < wid) base += t.wsum[w];
  t.hist[tid] = base + incl - h;  // bucket start
  __syncthreads();
  t.order[t.hist[key] + r] = tid;
  __syncthreads();
  return t.order[tid];
}

// ---------------------------------------------------------------------------
// decode: one lane per string, FSM in LDS
// ---------------------------------------------------------------------------

// LDS image of the decode FSM.  Rows are padded to 17 dwords so that entry
// (row r, nibble v) lies in bank (17 r + v) mod 32: with 16-dword rows every
// lane reading nibble v would hit one of two banks, and header text has a
// few dominant high nibbles (0x4-0x7).
constexpr uint32_t kFsmRowWords = 17;
constexpr uint32_t kFsmLdsWords = QH_NSTATE * kFsmRowWords;  // 17,476 B

// One FSM step for the byte in bits [8b, 8b+8) of word w (huffman.c:103-114).
// LDS word = (state * 68) | flags << 16 | sym << 24: the reference node
// {fstate, flags, sym} with fstate pre-multiplied into its row's byte offset.
#define QH_DECODE_BYTE(w, b)                                                  \
  do {                                                                        \
    const uint32_t hi4 = ((w) >> (8 * (b) + 2)) & 0x3Cu;                      \
    const uint32_t e1 = lds_word(fsm, st + hi4);                              \
    acc |= (uint64_t)(e1 >> 24) << nb;                                        \
    nb += (e1 >> (kFlagSymBit - 3)) & 8u;                                     \
    const uint32_t lo4 = (8 * (b) >= 2) ? (((w) >> (8 * (b) - 2)) & 0x3Cu)    \
                                        : (((w) << 2) & 0x3Cu);               \
    const uint32_t e2 = lds_word(fsm, (e1 & 0xFFFFu) + lo4);                  \
    acc |= (uint64_t)(e2 >> 24) << nb;                                        \
    nb += (e2 >> (kFlagSymBit - 3)) & 8u;                                     \
    st = e2 & 0xFFFFu;                                                        \
    last = e2;                                                                \
  } while (0)

#define QH_FLUSH()                                                            \
  do {                                                                        \
    if (nb >= 32) {                                                           \
      wp[nout++] = (uint32_t)acc;                                             \
      acc >>= 32;                                                             \
      nb -= 32;                                                               \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(kBlock) void qh_k_decode(
    const uint8_t *__restrict__ src, const SpanIn *__restrict__ in,
    SpanOut *__restrict__ out, uint64_t n, uint8_t *__restrict__ dst,
    uint64_t dst_cap, const uint32_t *__restrict__ g_fsm,
    DevStats *__restrict__ stats) {
  __shared__ uint32_t fsm[kFsmLdsWords];
  __shared__ TileLds tl;
  __shared__ unsigned long long red[kBlock / 64];
  for (uint32_t i = threadIdx.x; i < kFsmWords; i += kBlock) {
    const uint32_t w = g_fsm[i];
    fsm[(i >> 4) * kFsmRowWords + (i & 15)] =
        ((w & 0xFFFFu) * (kFsmRowWords * 4)) | (w & 0xFFFF0000u);
  }
  __syncthreads();

  unsigned long long my_in = 0, my_out = 0, my_err = 0;
  for (uint64_t tile0 = (uint64_t)blockIdx.x * kBlock; tile0 < n;
       tile0 += (uint64_t)gridDim.x * kBlock) {
    const uint64_t mine = tile0 + threadIdx.x;
    const uint32_t mylen = mine < n ? in[mine].len : 0u;
    const uint64_t s = tile0 + tile_rank_by_len(mylen, tl);
    if (s >= n) continue;
    const SpanIn sp = in[s];
    const uint64_t slot = out[s].off;
    const uint32_t len = sp.len;
    my_in += len;
    if (slot + qh_slot_size(len) > dst_cap) {
      out[s].len = 0;
      out[s].status = QH_ERR_NOMEM;
      ++my_err;
      continue;
    }
    const uint8_t *p = src + sp.off;
    // Slots are 16-byte aligned (qh_slot_size), so the string's output is
    // written with whole aligned dwords only: no head bytes, and the last
    // partial dword spills garbage into the string's own slot padding.
    uint32_t *wp = reinterpret_cast<uint32_t *>(dst + slot);
    uint64_t acc = 0;
    uint32_t nb = 0;
    uint32_t nout = 0;                       // dwords stored
    uint32_t st = 0;
    uint32_t last = QH_FLAG_ACCEPTED << 16;  // huffman.c:80-85

    const uint32_t body = len & ~15u;
    u32x4 nxt = {0, 0, 0, 0};
    if (body) nxt = *reinterpret_cast<const u32x4_ua *>(p);
    for (uint32_t pos = 0; pos < body; pos += 16) {
      const u32x4 v = nxt;
      if (pos + 16 < body)  // prefetch the next chunk before the FSM chain
        nxt = *reinterpret_cast<const u32x4_ua *>(p + pos + 16);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t w = v[d];
        QH_DECODE_BYTE(w, 0);
        QH_DECODE_BYTE(w, 1);
        QH_FLUSH();
        QH_DECODE_BYTE(w, 2);
        QH_DECODE_BYTE(w, 3);
        QH_FLUSH();
      }
    }
    if (body < len) {
      const u32x4 v = load_tail(p, body, len);
      const uint32_t rem = len - body;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t w = v[d];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if ((uint32_t)(4 * d + b) < rem) {
            QH_DECODE_BYTE(w, b);
            QH_FLUSH();
          }
        }
      }
    }
    const uint32_t dec_len = nout * 4 + (nb >> 3);
    // huffman.c:119-121: fin && !ACCEPTED -> -108.  The absorbing failure
    // state 256 carries no flags, so it fails here too (qpack.c:2756).
    const bool ok = (last >> 16) & QH_FLAG_ACCEPTED;
    if (ok) {
      if (nb) wp[nout] = (uint32_t)acc;
      out[s].len = dec_len;
      out[s].status = 0;
      my_out += dec_len;
    } else {
      out[s].len = 0;
      out[s].status = QH_ERR_QPACK_FATAL;
      ++my_err;
    }
  }
  block_add(&stats->in_bytes, my_in, red);
  block_add(&stats->out_bytes, my_out, red);
  block_add(&stats->n_errors, my_err, red);
}
#undef QH_FLUSH

// ---------------------------------------------------------------------------
// encode_count and encode: one lane per string, symbol table in LDS
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void qh_k_count(
    const uint8_t *__restrict__ src, const SpanIn *__restrict__ in,
    SpanOut *__restrict__ out, uint32_t *__restrict__ hlen_out, uint64_t n,
    const uint32_t *__restrict__ g_sym, DevStats *__restrict__ stats) {
  __shared__ uint8_t nbits[256];
  __shared__ TileLds tl;
  __shared__ unsigned long long red[kBlock / 64];
  nbits[threadIdx.x] = (uint8_t)g_sym[2 * threadIdx.x];
  __syncthreads();
  unsigned long long my_in = 0;
  for (uint64_t tile0 = (uint64_t)blockIdx.x * kBlock; tile0 < n;
       tile0 += (uint64_t)gridDim.x * kBlock) {
    const uint64_t mine = tile0 + threadIdx.x;
    const uint32_t mylen = mine < n ? in[mine].len : 0u;
    const uint64_t s = tile0 + tile_rank_by_len(mylen, tl);
    if (s >= n) continue;
    const SpanIn sp = in[s];
    const uint8_t *p = src + sp.off;
    const uint32_t len = sp.len;
    my_in += len;
    uint32_t bits = 0;
    const uint32_t body = len & ~15u;
    u32x4 nxt = {0, 0, 0, 0};
    if (body) nxt = *reinterpret_cast<const u32x4_ua *>(p);
    for (uint32_t pos = 0; pos < body; pos += 16) {
      const u32x4 v = nxt;
      if (pos + 16 < body) nxt = *reinterpret_cast<const u32x4_ua *>(p + pos + 16);
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int b = 0; b < 4; ++b) bits += nbits[(v[d] >> (8 * b)) & 0xFFu];
    }
    if (body < len) {
      const u32x4 v = load_tail(p, body, len);
      const uint32_t rem = len - body;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((uint32_t)(4 * d + b) < rem)
            bits += nbits[(v[d] >> (8 * b)) & 0xFFu];
    }
    const uint32_t h = (bits + 7) / 8;  // huffman.c:42
    if (hlen_out) hlen_out[s] = h;
    if (out) {
      out[s].len = h;
      out[s].status = 0;
    }
  }
  block_add(&stats->in_bytes, my_in, red);
}

// The bit accumulator is pre-loaded with `head` dummy bytes (the bytes of
// the first aligned dword that belong to the previous string), so every
// 32-bit word it emits is an aligned dword of dst.  The first word is shared
// with the previous string and is kept in a register; all later words are
// stored whole.  Only the two edge dwords are written bytewise, once.
#define QH_ENCODE_SYM(c)                                                      \
  do {                                                                        \
    const uint2 e = symtab[(c)];                                              \
    code |= (uint64_t)e.y << (32 - nbits);                                    \
    nbits += e.x;                                                             \
    if (nbits >= 32) {                                                        \
      const uint32_t x = (uint32_t)(code >> 32);                              \
      if (k == 0) first = x;                                                  \
      if (k != 0 || head == 0) wp[k] = __builtin_bswap32(x);                  \
      ++k;                                                                    \
      code <<= 32;                                                            \
      nbits -= 32;                                                            \
    }                                                                         \
  } while (0)

__global__ __launch_bounds__(kBlock) void qh_k_encode(
    const uint8_t *__restrict__ src, const SpanIn *__restrict__ in,
    SpanOut *__restrict__ out, uint64_t n, uint8_t *__restrict__ dst,
    uint64_t dst_cap, const uint32_t *__restrict__ g_sym,
    DevStats *__restrict__ stats) {
  __shared__ uint2 symtab[256];
  __shared__ TileLds tl;
  __shared__ unsigned long long red[kBlock / 64];
  symtab[threadIdx.x] = make_uint2(g_sym[2 * threadIdx.x], g_sym[2 * threadIdx.x + 1]);
  __syncthreads();
  unsigned long long my_out = 0, my_err = 0;
  for (uint64_t tile0 = (uint64_t)blockIdx.x * kBlock; tile0 < n;
       tile0 += (uint64_t)gridDim.x * kBlock) {
    const uint64_t mine = tile0 + threadIdx.x;
    const uint32_t mylen = mine < n ? in[mine].len : 0u;
    const uint64_t s = tile0 + tile_rank_by_len(mylen, tl);
    if (s >= n) continue;
    const SpanIn sp = in[s];
    const SpanOut so = out[s];
    if (so.off + so.len > dst_cap) {
      out[s].len = 0;
      out[s].status = QH_ERR_NOMEM;
      ++my_err;
      continue;
    }
    const uint8_t *p = src + sp.off;
    const uint32_t len = sp.len;
    const uint32_t head = (uint32_t)(so.off & 3);
    uint32_t *wp = reinterpret_cast<uint32_t *>(dst + so.off - head);
    uint64_t code = 0;
    uint32_t nbits = head * 8;  // dummy leading bits, never stored
    uint32_t k = 0;             // aligned dwords emitted
    uint32_t first = 0;         // big-endian image of dword 0
    const uint32_t body = len & ~15u;
    u32x4 nxt = {0, 0, 0, 0};
    if (body) nxt = *reinterpret_cast<const u32x4_ua *>(p);
    for (uint32_t pos = 0; pos < body; pos += 16) {
      const u32x4 v = nxt;
      if (pos + 16 < body) nxt = *reinterpret_cast<const u32x4_ua *>(p + pos + 16);
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int b = 0; b < 4; ++b) QH_ENCODE_SYM((v[d] >> (8 * b)) & 0xFFu);
    }
    if (body < len) {
      const u32x4 v = load_tail(p, body, len);
      const uint32_t rem = len - body;
#pragma unroll
      for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if ((uint32_t)(4 * d + b) < rem)
            QH_ENCODE_SYM((v[d] >> (8 * b)) & 0xFFu);
    }
    // huffman.c:67-75: pad the last partial byte with the leading (all-one)
    // bits of EOS; nbits < 32 here.
    const uint32_t padded = (nbits + 7) & ~7u;
    if (padded != nbits)
      code |= ((1ull << (padded - nbits)) - 1) << (64 - padded);
    const uint32_t tail = (uint32_t)(code >> 32);  // bytes [0, padded/8)
    uint8_t *b0 = reinterpret_cast<uint8_t *>(wp);
    if (k == 0) {
      // the whole string lies inside dword 0: bytes [head, padded/8)
      for (uint32_t j = head; j < padded / 8; ++j)
        b0[j] = (uint8_t)(tail >> (24 - 8 * j));
    } else {
      for (uint32_t j = head; j < 4 && head; ++j)
        b0[j] = (uint8_t)(first >> (24 - 8 * j));
      uint8_t *bk = b0 + 4 * k;
      for (uint32_t j = 0; j < padded / 8; ++j)
        bk[j] = (uint8_t)(tail >> (24 - 8 * j));
    }
    my_out += so.len;
  }
  block_add(&stats->out_bytes, my_out, red);
  block_add(&stats->n_errors, my_err, red);
}

// ---------------------------------------------------------------------------
// synthetic inputs (splitmix64, counter-based)
// ---------------------------------------------------------------------------

__host__ __device__ __forceinline__ uint64_t sm64_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// k-th output (k = 0, 1, ...) of the splitmix64 generator seeded with `seed`.
__host__ __device__ __forceinline__ uint64_t sm64_at(uint64_t seed,
                                                     uint64_t k) {
  return sm64_mix(seed + (k + 1) * 0x9E3779B97F4A7C15ull);
}
constexpr uint64_t kLenStream = 0x4C454E47544853ull;   // "LENGTHS"
constexpr uint64_t kByteStream = 0x4259544553ull;      // "BYTES"

__global__ __launch_bounds__(kBlock) void qh_k_synth_lens(
    uint64_t seed, uint64_t n, uint32_t lo, uint32_t span, SpanIn *in) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s >= n) return;
  const uint64_t r = sm64_at(seed ^ kLenStream, s);
  in[s].len = lo + (uint32_t)(r % span);
  in[s].flags = 0;
}

// offsets: exclusive scan of len into in[i].off (reuses the scan machinery
// through a small adapter kernel pair: lens are copied into out[].len).
__global__ __launch_bounds__(kBlock) void qh_k_copy_len(const SpanIn *in,
                                                        SpanOut *tmp,
                                                        uint64_t n) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s < n) tmp[s].len = in[s].len;
}
__global__ __launch_bounds__(kBlock) void qh_k_set_off(SpanIn *in,
                                                       const SpanOut *tmp,
                                                       uint64_t n,
                                                       uint64_t *total) {
  const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (s < n) {
    in[s].off = tmp[s].off;
    if (s == n - 1) *total = tmp[s].off + in[s].len;
  }
}

__global__ __launch_bounds__(kBlock) void qh_k_synth_fill(
    uint64_t seed, uint8_t *dst, uint64_t nbytes, const uint8_t *alph,
    uint32_t alen) {
  __shared__ uint8_t a[256];
  if (threadIdx.x < alen) a[threadIdx.x] = alph[threadIdx.x];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * 4;
  for (uint64_t k = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
       k < nbytes; k += stride) {
    uint32_t w = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      w |= (uint32_t)a[sm64_at(seed ^ kByteStream, k + b) % alen] << (8 * b);
    if (k + 4 <= nbytes) {
      *reinterpret_cast<uint32_t *>(dst + k) = w;
    } else {
      for (int b = 0; k + b < nbytes; ++b) dst[k + b] = (uint8_t)(w >> (8 * b));
    }
  }
}

}  // namespace qhk

using namespace qhk;

// ---------------------------------------------------------------------------
// host side: context, scratch, timing
// ---------------------------------------------------------------------------

struct qh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  uint32_t *d_fsm = nullptr;  // 257*16 words
  uint32_t *d_sym = nullptr;  // 257*2 words
  DevStats *d_stats = nullptr;
  uint64_t *d_tile_state = nullptr;
  size_t tile_state_cap = 0;  // entries (+1 word for the tile counter)
  uint64_t last_n = 0;
  int num_cus = 256;
  // host-mode staging
  void *h_buf[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t h_cap[4] = {0, 0, 0, 0};
  // timing
  bool timing = false;
  struct Ev {
    const char *name;
    hipEvent_t a, b;
  };
  std::vector<Ev> events;
  std::vector<hipEvent_t> pool;
};

namespace {

#define QH_HIP(call)                                                           \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "qhuff: %s failed: %s (%s:%d)\n", #call,                 \
              hipGetErrorString(e_), __FILE__, __LINE__);                      \
      return QH_ERR_FATAL;                                                     \
    }                                                                          \
  } while (0)

hipEvent_t take_event(qh_ctx *c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct Timed {
  qh_ctx *c;
  const char *name;
  hipEvent_t a = nullptr, b = nullptr;
  Timed(qh_ctx *c_, const char *n) : c(c_), name(n) {
    if (c->timing) {
      a = take_event(c);
      b = take_event(c);
      if (a) hipEventRecord(a, c->stream);
    }
  }
  ~Timed() {
    if (c->timing && a && b) {
      hipEventRecord(b, c->stream);
      c->events.push_back({name, a, b});
    }
  }
};

int ensure_tile_state(qh_ctx *c, uint64_t n) {
  const size_t tiles = (size_t)((n + kScanTile - 1) / kScanTile) + 1;
  if (tiles + 2 > c->tile_state_cap) {
    if (c->d_tile_state) hipFree(c->d_tile_state);
    c->d_tile_state = nullptr;
    size_t cap = 1024;
    while (cap < tiles + 2) cap *= 2;
    QH_HIP(hipMalloc(&c->d_tile_state, cap * sizeof(uint64_t)));
    c->tile_state_cap = cap;
  }
  return 0;
}

int grid_for(qh_ctx *c, uint64_t n) {
  uint64_t g = (n + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)c->num_cus * 8;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

int launch_scan(qh_ctx *c, int mode, const SpanIn *in, SpanOut *out,
                uint64_t n) {
  if (n == 0) return 0;
  int rv = ensure_tile_state(c, n);
  if (rv) return rv;
  const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
  // word 0 = tile counter (as u32), words 1.. = tile states
  QH_HIP(hipMemsetAsync(c->d_tile_state, 0, (tiles + 1) * sizeof(uint64_t),
                        c->stream));
  uint32_t *ctr = reinterpret_cast<uint32_t *>(c->d_tile_state);
  uint64_t *states = c->d_tile_state + 1;
  Timed t(c, mode == SCAN_SLOTS ? "qh_k_scan_slots" : "qh_k_scan_hlen");
  if (mode == SCAN_SLOTS)
    hipLaunchKernelGGL(qh_k_scan<SCAN_SLOTS>, dim3((unsigned)tiles),
                       dim3(kBlock), 0, c->stream, in, out, n, states, ctr,
                       c->d_stats);
  else
    hipLaunchKernelGGL(qh_k_scan<SCAN_HLEN>, dim3((unsigned)tiles),
                       dim3(kBlock), 0, c->stream, in, out, n, states, ctr,
                       c->d_stats);
  QH_HIP(hipGetLastError());
  return 0;
}

int reset_stats(qh_ctx *c, uint64_t n) {
  QH_HIP(hipMemsetAsync(c->d_stats, 0, sizeof(DevStats), c->stream));
  c->last_n = n;
  return 0;
}

int check_ctx(qh_ctx *c) {
  if (!c) return QH_ERR_INVALID_ARGUMENT;
  QH_HIP(hipSetDevice(c->device));
  return 0;
}

// Device-resident decode pipeline.
int decode_device(qh_ctx *c, const uint8_t *src, const SpanIn *in, uint64_t n,
                  uint8_t *dst, uint64_t dst_cap, SpanOut *out) {
  int rv = reset_stats(c, n);
  if (rv || n == 0) return rv;
  rv = launch_scan(c, SCAN_SLOTS, in, out, n);
  if (rv) return rv;
  {
    Timed t(c, "qh_k_decode");
    hipLaunchKernelGGL(qh_k_decode, dim3(grid_for(c, n)), dim3(kBlock), 0,
                       c->stream, src, in, out, n, dst, dst_cap, c->d_fsm,
                       c->d_stats);
  }
  QH_HIP(hipGetLastError());
  return 0;
}

int count_device(qh_ctx *c, const uint8_t *src, const SpanIn *in, uint64_t n,
                 uint32_t *hlen, SpanOut *out) {
  Timed t(c, "qh_k_count");
  hipLaunchKernelGGL(qh_k_count, dim3(grid_for(c, n)), dim3(kBlock), 0,
                     c->stream, src, in, out, hlen, n, c->d_sym, c->d_stats);
  QH_HIP(hipGetLastError());
  return 0;
}

int encode_device(qh_ctx *c, const uint8_t *src, const SpanIn *in, uint64_t n,
                  uint8_t *dst, uint64_t dst_cap, SpanOut *out) {
  int rv = reset_stats(c, n);
  if (rv || n == 0) return rv;
  rv = count_device(c, src, in, n, nullptr, out);
  if (rv) return rv;
  rv = launch_scan(c, SCAN_HLEN, in, out, n);
  if (rv) return rv;
  {
    Timed t(c, "qh_k_encode");
    hipLaunchKernelGGL(qh_k_encode, dim3(grid_for(c, n)), dim3(kBlock), 0,
                       c->stream, src, in, out, n, dst, dst_cap, c->d_sym,
                       c->d_stats);
  }
  QH_HIP(hipGetLastError());
  return 0;
}

// host-mode staging buffer k (0 = src, 1 = spans in, 2 = dst, 3 = spans out)
int stage(qh_ctx *c, int k, size_t bytes, void **p) {
  if (bytes == 0) bytes = 16;
  if (c->h_cap[k] < bytes) {
    if (c->h_buf[k]) hipFree(c->h_buf[k]);
    c->h_buf[k] = nullptr;
    c->h_cap[k] = 0;
    QH_HIP(hipMalloc(&c->h_buf[k], bytes));
    c->h_cap[k] = bytes;
  }
  *p = c->h_buf[k];
  return 0;
}

uint64_t src_extent(const qh_span_in *in, size_t n) {
  uint64_t e = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t x = in[i].off + in[i].len;
    if (x > e) e = x;
  }
  return e;
}

}  // namespace

// ---------------------------------------------------------------------------
// exported C ABI
// ---------------------------------------------------------------------------

extern "C" {

QH_EXPORT const char *qh_version(void) { return QH_VERSION; }

QH_EXPORT int qh_ctx_new(qh_ctx **pctx, int device, void *stream) {
  if (!pctx) return QH_ERR_INVALID_ARGUMENT;
  *pctx = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fprintf(stderr, "qhuff: no HIP device available (batch API needs one)\n");
    return QH_ERR_FATAL;
  }
  if (device < 0 || device >= ndev) return QH_ERR_INVALID_ARGUMENT;
  qh_ctx *c = new (std::nothrow) qh_ctx();
  if (!c) return QH_ERR_NOMEM;
  c->device = device;
  auto fail = [&](int rv) {
    qh_ctx_del(c);
    return rv;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(QH_ERR_FATAL);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess &&
      prop.multiProcessorCount > 0)
    c->num_cus = prop.multiProcessorCount;
  // NULL selects the HIP default (null) stream, as HIP/ROCm libraries do.
  c->stream = (hipStream_t)stream;
  if (hipMalloc(&c->d_fsm, sizeof(kFsmPacked)) != hipSuccess ||
      hipMalloc(&c->d_sym, sizeof(kSymPacked)) != hipSuccess ||
      hipMalloc(&c->d_stats, sizeof(DevStats)) != hipSuccess)
    return fail(QH_ERR_NOMEM);
  if (hipMemcpy(c->d_fsm, kFsmPacked, sizeof(kFsmPacked),
                hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_sym, kSymPacked, sizeof(kSymPacked),
                hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_stats, 0, sizeof(DevStats)) != hipSuccess)
    return fail(QH_ERR_FATAL);
  *pctx = c;
  return 0;
}

QH_EXPORT void qh_ctx_del(qh_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  for (auto &e : c->events) {
    hipEventDestroy(e.a);
    hipEventDestroy(e.b);
  }
  for (auto e : c->pool) hipEventDestroy(e);
  if (c->d_fsm) hipFree(c->d_fsm);
  if (c->d_sym) hipFree(c->d_sym);
  if (c->d_stats) hipFree(c->d_stats);
  if (c->d_tile_state) hipFree(c->d_tile_state);
  for (int k = 0; k < 4; ++k)
    if (c->h_buf[k]) hipFree(c->h_buf[k]);
  if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
  delete c;
}

QH_EXPORT int qh_ctx_set_stream(qh_ctx *c, void *stream) {
  if (!c) return QH_ERR_INVALID_ARGUMENT;
  if (c->own_stream && c->stream) {
    QH_HIP(hipStreamSynchronize(c->stream));
    QH_HIP(hipStreamDestroy(c->stream));
  }
  c->own_stream = false;
  c->stream = (hipStream_t)stream;
  return 0;
}

QH_EXPORT void *qh_ctx_stream(qh_ctx *c) { return c ? (void *)c->stream : nullptr; }

QH_EXPORT int qh_ctx_sync(qh_ctx *c) {
  int rv = check_ctx(c);
  if (rv) return rv;
  QH_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

QH_EXPORT int qh_ctx_last_stats(qh_ctx *c, qh_batch_stats *st) {
  int rv = check_ctx(c);
  if (rv) return rv;
  if (!st) return QH_ERR_INVALID_ARGUMENT;
  DevStats d;
  QH_HIP(hipMemcpyAsync(&d, c->d_stats, sizeof(d), hipMemcpyDeviceToHost,
                        c->stream));
  QH_HIP(hipStreamSynchronize(c->stream));
  if (d.scan_timeouts) {
    fprintf(stderr, "qhuff: scan look-back timed out (%llu tiles)\n",
            d.scan_timeouts);
    return QH_ERR_FATAL;
  }
  st->n = c->last_n;
  st->in_bytes = d.in_bytes;
  st->out_bytes = d.out_bytes;
  st->dst_bytes = d.dst_bytes;
  st->n_errors = d.n_errors;
  return 0;
}

QH_EXPORT uint64_t qh_decode_dst_size(const qh_span_in *in, size_t n) {
  uint64_t s = 0;
  for (size_t i = 0; i < n; ++i) s += qh_slot_size(in[i].len);
  return s;
}

QH_EXPORT uint64_t qh_encode_dst_bound(const qh_span_in *in, size_t n) {
  uint64_t s = 0;
  for (size_t i = 0; i < n; ++i) s += ((uint64_t)in[i].len * 30 + 7) / 8;
  return s;
}

QH_EXPORT int qh_decode_batch(qh_ctx *c, const uint8_t *src,
                              const qh_span_in *in, size_t n, uint8_t *dst,
                              uint64_t dst_cap, qh_span_out *out, int where) {
  int rv = check_ctx(c);
  if (rv) return rv;
  if (n && (!src || !in || !out || (!dst && dst_cap))) return QH_ERR_INVALID_ARGUMENT;
  if (where == QH_WHERE_DEVICE)
    return decode_device(c, src, (const SpanIn *)in, n, dst, dst_cap,
                         (SpanOut *)out);
  if (where != QH_WHERE_HOST) return QH_ERR_INVALID_ARGUMENT;
  // host mode: stage through device buffers
  const uint64_t extent = src_extent(in, n);
  const uint64_t need = qh_decode_dst_size(in, n);
  const uint64_t dcap = dst_cap < need ? dst_cap : need;
  void *d_src, *d_in, *d_dst, *d_out;
  if ((rv = stage(c, 0, extent, &d_src)) || (rv = stage(c, 1, n * 16, &d_in)) ||
      (rv = stage(c, 2, dcap, &d_dst)) || (rv = stage(c, 3, n * 16, &d_out)))
    return rv;
  QH_HIP(hipMemcpyAsync(d_src, src, extent, hipMemcpyHostToDevice, c->stream));
  QH_HIP(hipMemcpyAsync(d_in, in, n * 16, hipMemcpyHostToDevice, c->stream));
  rv = decode_device(c, (const uint8_t *)d_src, (const SpanIn *)d_in, n,
                     (uint8_t *)d_dst, dcap, (SpanOut *)d_out);
  if (rv) return rv;
  QH_HIP(hipMemcpyAsync(out, d_out, n * 16, hipMemcpyDeviceToHost, c->stream));
  if (dcap)
    QH_HIP(hipMemcpyAsync(dst, d_dst, dcap, hipMemcpyDeviceToHost, c->stream));
  QH_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

QH_EXPORT int qh_encode_count_batch(qh_ctx *c, const uint8_t *src,
                                    const qh_span_in *in, size_t n,
                                    uint32_t *hlen, int where) {
  int rv = check_ctx(c);
  if (rv) return rv;
  if (n && (!src || !in || !hlen)) return QH_ERR_INVALID_ARGUMENT;
  if (where == QH_WHERE_DEVICE) {
    if ((rv = reset_stats(c, n)) || n == 0) return rv;
    return count_device(c, src, (const SpanIn *)in, n, hlen, nullptr);
  }
  if (where != QH_WHERE_HOST) return QH_ERR_INVALID_ARGUMENT;
  const uint64_t extent = src_extent(in, n);
  void *d_src, *d_in, *d_h;
  if ((rv = stage(c, 0, extent, &d_src)) || (rv = stage(c, 1, n * 16, &d_in)) ||
      (rv = stage(c, 3, n * 4, &d_h)))
    return rv;
  QH_HIP(hipMemcpyAsync(d_src, src, extent, hipMemcpyHostToDevice, c->stream));
  QH_HIP(hipMemcpyAsync(d_in, in, n * 16, hipMemcpyHostToDevice, c->stream));
  if ((rv = reset_stats(c, n))) return rv;
  if (n) {
    rv = count_device(c, (const uint8_t *)d_src, (const SpanIn *)d_in, n,
                      (uint32_t *)d_h, nullptr);
    if (rv) return rv;
    QH_HIP(hipMemcpyAsync(hlen, d_h, n * 4, hipMemcpyDeviceToHost, c->stream));
  }
  QH_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

QH_EXPORT int qh_encode_batch(qh_ctx *c, const uint8_t *src,
                              const qh_span_in *in, size_t n, uint8_t *dst,
                              uint64_t dst_cap, qh_span_out *out, int where) {
  int rv = check_ctx(c);
  if (rv) return rv;
  if (n && (!src || !in || !out || (!dst && dst_cap))) return QH_ERR_INVALID_ARGUMENT;
  if (where == QH_WHERE_DEVICE)
    return encode_device(c, src, (const SpanIn *)in, n, dst, dst_cap,
                         (SpanOut *)out);
  if (where != QH_WHERE_HOST) return QH_ERR_INVALID_ARGUMENT;
  const uint64_t extent = src_extent(in, n);
  const uint64_t bound = qh_encode_dst_bound(in, n);
  const uint64_t dcap = dst_cap < bound ? dst_cap : bound;
  void *d_src, *d_in, *d_dst, *d_out;
  if ((rv = stage(c, 0, extent, &d_src)) || (rv = stage(c, 1, n * 16, &d_in)) ||
      (rv = stage(c, 2, dcap, &d_dst)) || (rv = stage(c, 3, n * 16, &d_out)))
    return rv;
  QH_HIP(hipMemcpyAsync(d_src, src, extent, hipMemcpyHostToDevice, c->stream));
  QH_HIP(hipMemcpyAsync(d_in, in, n * 16, hipMemcpyHostToDevice, c->stream));
  rv = encode_device(c, (const uint8_t *)d_src, (const SpanIn *)d_in, n,
                     (uint8_t *)d_dst, dcap, (SpanOut *)d_out);
  if (rv) return rv;
  QH_HIP(hipMemcpyAsync(out, d_out, n * 16, hipMemcpyDeviceToHost, c->stream));
  QH_HIP(hipStreamSynchronize(c->stream));
  // copy back only the bytes the dense layout occupies
  uint64_t used = 0;
  for (size_t i = 0; i < n; ++i)
    if (out[i].status == 0 && out[i].off + out[i].len > used)
      used = out[i].off + out[i].len;
  if (used)
    QH_HIP(hipMemcpy(dst, d_dst, used, hipMemcpyDeviceToHost));
  return 0;
}

QH_EXPORT int qh_ctx_enable_timing(qh_ctx *c, int on) {
  if (!c) return QH_ERR_INVALID_ARGUMENT;
  c->timing = on != 0;
  return 0;
}

QH_EXPORT int qh_ctx_kernel_times(qh_ctx *c, const char **names,
                                  uint64_t *counts, double *ms, int cap) {
  int rv = check_ctx(c);
  if (rv) return rv;
  QH_HIP(hipStreamSynchronize(c->stream));
  std::vector<std::string> keys;
  std::vector<uint64_t> cnt;
  std::vector<double> tot;
  for (auto &e : c->events) {
    float t = 0;
    hipEventElapsedTime(&t, e.a, e.b);
    size_t k = 0;
    for (; k < keys.size(); ++k)
      if (keys[k] == e.name) break;
    if (k == keys.size()) {
      keys.push_back(e.name);
      cnt.push_back(0);
      tot.push_back(0);
    }
    cnt[k] += 1;
    tot[k] += t;
    c->pool.push_back(e.a);
    c->pool.push_back(e.b);
  }
  int m = 0;
  for (size_t k = 0; k < keys.size() && m < cap; ++k, ++m) {
    // names point at the string literals recorded with the events
    for (auto &e : c->events)
      if (keys[k] == e.name) {
        names[m] = e.name;
        break;
      }
    counts[m] = cnt[k];
    ms[m] = tot[k];
  }
  c->events.clear();
  return m;
}

QH_EXPORT int qh_synth_spans(qh_ctx *c, uint64_t seed, size_t n, uint32_t lo,
                             uint32_t hi, int dist, double zipf_s,
                             qh_span_in *in_dev, uint64_t *total_dev) {
  (void)zipf_s;
  int rv = check_ctx(c);
  if (rv) return rv;
  if (hi < lo || !in_dev || !total_dev || dist != 0) return QH_ERR_INVALID_ARGUMENT;
  if (n == 0) {
    QH_HIP(hipMemsetAsync(total_dev, 0, 8, c->stream));
    return 0;
  }
  SpanIn *in = (SpanIn *)in_dev;
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(qh_k_synth_lens, dim3(blocks), dim3(kBlock), 0, c->stream,
                     seed, (uint64_t)n, lo, hi - lo + 1, in);
  QH_HIP(hipGetLastError());
  void *tmp;
  if ((rv = stage(c, 3, n * 16, &tmp))) return rv;
  hipLaunchKernelGGL(qh_k_copy_len, dim3(blocks), dim3(kBlock), 0, c->stream,
                     in, (SpanOut *)tmp, (uint64_t)n);
  if ((rv = launch_scan(c, SCAN_HLEN, in, (SpanOut *)tmp, n))) return rv;
  hipLaunchKernelGGL(qh_k_set_off, dim3(blocks), dim3(kBlock), 0, c->stream,
                     in, (const SpanOut *)tmp, (uint64_t)n, total_dev);
  QH_HIP(hipGetLastError());
  return 0;
}

QH_EXPORT int qh_synth_fill(qh_ctx *c, uint64_t seed, uint8_t *dst_dev,
                            uint64_t nbytes, const uint8_t *alphabet,
                            uint32_t alphabet_len) {
  int rv = check_ctx(c);
  if (rv) return rv;
  if (!alphabet || alphabet_len == 0 || alphabet_len > 256 || (!dst_dev && nbytes))
    return QH_ERR_INVALID_ARGUMENT;
  if (nbytes == 0) return 0;
  void *d_alph;
  if ((rv = stage(c, 1, 256, &d_alph))) return rv;
  QH_HIP(hipMemcpyAsync(d_alph, alphabet, alphabet_len, hipMemcpyHostToDevice,
                        c->stream));
  uint64_t blocks = (nbytes / 4 + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(qh_k_synth_fill, dim3((unsigned)blocks), dim3(kBlock), 0,
                     c->stream, seed, dst_dev, nbytes, (const uint8_t *)d_alph,
                     alphabet_len);
  QH_HIP(hipGetLastError());
  // the alphabet staging buffer is reused by later host-mode calls: wait
  QH_HIP(hipStreamSynchronize(c->stream));
  return 0;
}

}  // extern "C"
