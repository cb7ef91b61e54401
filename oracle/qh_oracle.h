/*
 * qh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of nghttp3's QPACK Huffman codec
 * (lib/nghttp3_qpack_huffman.c:34-129, lib/nghttp3_qpack_huffman.h:35-115).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline: the product
 * (nghttp3_amd/, include/qhuff.h) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - the tables this file builds are compared byte-for-byte with the
 *     reference tables in lib/nghttp3_qpack_huffman_data.c (SHA-256 digests
 *     committed in tests/golden/tables.json, re-derived from the reference
 *     text when /root/reference is present);
 *   - RFC 7541 Appendix C known-answer vectors (tests/golden/kat.json);
 *   - the reference's own unit tests tests/nghttp3_qpack_test.c:856-899
 *     (random round trip, failure-state streaming) restated in tests/.
 * The reference C cannot be compiled here (nghttp3.h needs the generated
 * nghttp3/version.h), so there is no oracle/_ref build.
 */
#ifndef QH_ORACLE_H
#define QH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint16_t fstate;
  uint8_t flags;
} qho_decode_ctx;

#define QHO_FLAG_ACCEPTED 0x01u
#define QHO_FLAG_SYM 0x02u
#define QHO_ERR_QPACK_FATAL (-108)

/* Tables as built by the oracle (sym: 257 x {nbits, code}; fsm: 257 x 16 u32
 * words fstate | flags << 16 | sym << 24). */
void qho_tables(uint32_t sym[257][2], uint32_t fsm[257][16]);

/* huffman.c:34-43 */
size_t qho_encode_count(const uint8_t *src, size_t len);
/* huffman.c:45-78 */
uint8_t *qho_encode(uint8_t *dest, const uint8_t *src, size_t srclen);
/* huffman.c:80-85 */
void qho_decode_context_init(qho_decode_ctx *ctx);
/* huffman.c:87-124 */
ptrdiff_t qho_decode(qho_decode_ctx *ctx, uint8_t *dest, const uint8_t *src,
                     size_t srclen, int fin);
/* huffman.c:126-129 */
int qho_decode_failure_state(const qho_decode_ctx *ctx);

/* Batch helpers over packed strings (string i = src[off[i] .. off[i]+len[i])).
 * encode: writes encoded strings densely into dst; out_off/out_len per string
 *   (out_off = exclusive prefix sum of encode_count). Returns total bytes.
 * decode (fin = 1 per string): string i written at dst + slot_off[i] where
 *   slot_off is the exclusive prefix sum of the batch API's slot size,
 *   round_up(len*8/5, 16) (huffman.h:113-115 estimate, include/qhuff.h);
 *   out_len = decoded length (0 on error), status 0 or -108. Returns the
 *   number of failed strings. */
uint64_t qho_encode_batch(const uint8_t *src, const uint64_t *off,
                          const uint32_t *len, size_t n, uint8_t *dst,
                          uint64_t *out_off, uint32_t *out_len);
uint64_t qho_decode_batch(const uint8_t *src, const uint64_t *off,
                          const uint32_t *len, size_t n, uint8_t *dst,
                          uint64_t *slot_off, uint32_t *out_len,
                          int32_t *status);

/* CPU baseline: round trip (encode_count + encode, then decode) of the n
 * strings on a pool of `nthreads` threads created once, thread t pinned to
 * cpus[t] (cpus may be NULL) and owning a contiguous shard.  Each of `reps`
 * encode and decode passes starts and ends at a barrier and runs the shard
 * inner[0] (encode) / inner[1] (decode) times, calibrated so that a pass
 * takes >= min_seconds; enc_seconds[r] / dec_seconds[r] are the pass times
 * divided by those counts (seconds per round over the n strings).  Decoded
 * bytes are verified after the timed passes.  Returns 0 if every string
 * round-tripped. */
int qho_bench_roundtrip(const uint8_t *src, const uint64_t *off,
                        const uint32_t *len, size_t n, int nthreads,
                        const int *cpus, int reps, double min_seconds,
                        double *enc_seconds, double *dec_seconds,
                        int *inner_out);

#ifdef __cplusplus
}
#endif

#endif /* QH_ORACLE_H */
