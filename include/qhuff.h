/*
 * qhuff.h -- C ABI of the MI355X QPACK Huffman engine (libqhuff.so).
 *
 * Two families of entry points:
 *
 * 1. Exact-signature drop-ins for nghttp3's private Huffman codec
 *    (lib/nghttp3_qpack_huffman.h:42-107; implementation
 *    lib/nghttp3_qpack_huffman.c:34-129; data
 *    lib/nghttp3_qpack_huffman_data.c:30-96,98-4982).  They keep the
 *    reference names, argument meaning and error behaviour so that
 *    lib/nghttp3_qpack.c links against libqhuff instead of
 *    nghttp3_qpack_huffman.o / nghttp3_qpack_huffman_data.o (the symbols are
 *    hidden inside libnghttp3, so the replacement is at link time; see
 *    INTEGRATION.md).  These serve the streaming case the reference decoder
 *    has: a Huffman string split across nghttp3_qpack_decoder_read_request
 *    calls (qpack.c:2737-2763, fin = 0 until the last chunk).  They run on
 *    the host: a partial chunk of a few bytes cannot amortise a launch.
 *
 * 2. The batch API (qh_*): whole strings gathered by the QPACK layer
 *    (qpack.c call sites :1861,1882,1953,1961,1980,1993 for encode,
 *    :2750,2756 reached from :2992,3083,3606,3694 for decode) are encoded or
 *    decoded by HIP kernels on gfx950.  There is no host fallback: without a
 *    usable HIP device every batch entry point returns QH_ERR_FATAL.
 *
 * Plain C types only; no torch or HIP types appear in any signature
 * (streams are passed as `void *` = hipStream_t).
 */
#ifndef QHUFF_H
#define QHUFF_H

#include <stddef.h>
#include <stdint.h>

#if defined(_WIN32)
#define QH_EXPORT
#else
#define QH_EXPORT __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* 1. Exact-signature drop-ins (reference: lib/nghttp3_qpack_huffman.h)      */
/* ------------------------------------------------------------------------ */

/* nghttp3.h:82 */
typedef ptrdiff_t nghttp3_ssize;

#ifndef NGHTTP3_QPACK_HUFFMAN_H
/* huffman.h:35-40 -- code is MSB-aligned in 32 bits. */
typedef struct nghttp3_qpack_huffman_sym {
  uint32_t nbits;
  uint32_t code;
} nghttp3_qpack_huffman_sym;

/* huffman.h:51,54 */
#define NGHTTP3_QPACK_HUFFMAN_FLAG_ACCEPTED 0x01U
#define NGHTTP3_QPACK_HUFFMAN_FLAG_SYM 0x02U

/* huffman.h:56-68 */
typedef struct nghttp3_qpack_huffman_decode_node {
  uint16_t fstate;
  uint8_t flags;
  uint8_t sym;
} nghttp3_qpack_huffman_decode_node;

/* huffman.h:70-74 */
typedef struct nghttp3_qpack_huffman_decode_context {
  uint16_t fstate;
  uint8_t flags;
} nghttp3_qpack_huffman_decode_context;

/* huffman.h:113-115 */
static inline size_t nghttp3_qpack_huffman_estimate_decode_length(size_t len) {
  return len * 8 / 5;
}
#endif /* !NGHTTP3_QPACK_HUFFMAN_H */

/* huffman.h:42 / huffman_data.c:30-96 */
QH_EXPORT extern const nghttp3_qpack_huffman_sym huffman_sym_table[];
/* huffman.h:76 / huffman_data.c:98-4982 */
QH_EXPORT extern const nghttp3_qpack_huffman_decode_node
    qpack_huffman_decode_table[][16];

/* huffman.h:44 (huffman.c:34-43): ceil(sum of code lengths / 8). */
QH_EXPORT size_t nghttp3_qpack_huffman_encode_count(const uint8_t *src,
                                                    size_t len);
/* huffman.h:46-47 (huffman.c:45-78): writes exactly encode_count bytes,
 * returns dest + that count. */
QH_EXPORT uint8_t *nghttp3_qpack_huffman_encode(uint8_t *dest,
                                                const uint8_t *src,
                                                size_t srclen);
/* huffman.h:78-79 (huffman.c:80-85) */
QH_EXPORT void nghttp3_qpack_huffman_decode_context_init(
    nghttp3_qpack_huffman_decode_context *ctx);
/* huffman.h:97-100 (huffman.c:87-124): bytes written, or -108
 * (NGHTTP3_ERR_QPACK_FATAL) when fin && the final state is not accepting. */
QH_EXPORT nghttp3_ssize nghttp3_qpack_huffman_decode(
    nghttp3_qpack_huffman_decode_context *ctx, uint8_t *dest,
    const uint8_t *src, size_t srclen, int fin);
/* huffman.h:106-107 (huffman.c:126-129) */
QH_EXPORT int nghttp3_qpack_huffman_decode_failure_state(
    const nghttp3_qpack_huffman_decode_context *ctx);

/* ------------------------------------------------------------------------ */
/* 2. Batch API (HIP, gfx950)                                                */
/* ------------------------------------------------------------------------ */

/* Return codes (values follow lib/includes/nghttp3/nghttp3.h). */
#define QH_OK 0
#define QH_ERR_INVALID_ARGUMENT (-101) /* NGHTTP3_ERR_INVALID_ARGUMENT */
#define QH_ERR_QPACK_FATAL (-108)      /* NGHTTP3_ERR_QPACK_FATAL      */
#define QH_ERR_FATAL (-900)            /* NGHTTP3_ERR_FATAL: HIP failure */
#define QH_ERR_NOMEM (-901)            /* NGHTTP3_ERR_NOMEM            */

/* Where the pointers handed to a batch call live. */
#define QH_WHERE_HOST 0   /* host memory; the call copies H2D/D2H, blocks */
#define QH_WHERE_DEVICE 1 /* HBM; the call is asynchronous on ctx stream */

/* One string: bytes [off, off + len) of the batch's source buffer. */
typedef struct qh_span_in {
  uint64_t off;
  uint32_t len;
  uint32_t flags; /* reserved, must be 0 */
} qh_span_in;

/* One result string: bytes [off, off + len) of the batch's destination
 * buffer.  status is 0, QH_ERR_QPACK_FATAL (invalid Huffman string, same
 * verdict as nghttp3_qpack_huffman_decode(..., fin = 1) plus the
 * failure-state check at qpack.c:2756), or QH_ERR_NOMEM (the string's slot
 * does not fit in dst_cap; nothing written). */
typedef struct qh_span_out {
  uint64_t off;
  uint32_t len;
  int32_t status;
} qh_span_out;

/* Totals of the most recent batch call on a context. */
typedef struct qh_batch_stats {
  uint64_t n;          /* strings                                    */
  uint64_t in_bytes;   /* sum of input lengths                       */
  uint64_t out_bytes;  /* sum of output lengths (successful strings) */
  uint64_t dst_bytes;  /* destination bytes the layout occupies      */
  uint64_t n_errors;   /* strings with status != 0                   */
} qh_batch_stats;

typedef struct qh_ctx qh_ctx;

/* Bind a context to HIP device `device` and stream `stream` (a hipStream_t;
 * NULL = the device's default stream, as in other HIP libraries).  Every
 * batch call is ordered on that stream. */
QH_EXPORT int qh_ctx_new(qh_ctx **pctx, int device, void *stream);
QH_EXPORT void qh_ctx_del(qh_ctx *ctx);
QH_EXPORT int qh_ctx_set_stream(qh_ctx *ctx, void *stream);
QH_EXPORT void *qh_ctx_stream(qh_ctx *ctx);
/* Wait for all work queued on the context's stream. */
QH_EXPORT int qh_ctx_sync(qh_ctx *ctx);
/* Totals of the last batch call (synchronises the stream). */
QH_EXPORT int qh_ctx_last_stats(qh_ctx *ctx, qh_batch_stats *stats);

/* Destination sizing.  A decoded string never exceeds the reference's
 * estimate_decode_length(len) = len * 8 / 5 (huffman.h:113-115; the caller
 * of the reference sizes its rcbuf from it, qpack.c:2977,3065,3591,3677).
 * Batch decode gives string i a slot of round_up(len_i * 8 / 5 + 16, 64)
 * bytes, slots in string order and back to back (so every slot starts
 * 64-byte aligned relative to dst), so qh_decode_dst_size(in, n) = the sum
 * of the slots is what a batch needs; out[i].off is the start of the slot
 * and out[i].len the decoded length.  The other bytes of a slot are
 * unspecified.  A string whose slot does not fit in dst_cap gets
 * QH_ERR_NOMEM; nothing is written at or past dst_cap.
 * Encode output is dense: out[i].off = sum_{j<i} encode_count(string j);
 * qh_encode_dst_bound() is an upper bound. */
QH_EXPORT uint64_t qh_decode_dst_size(const qh_span_in *in, size_t n);
QH_EXPORT uint64_t qh_encode_dst_bound(const qh_span_in *in, size_t n);

/* Decode n complete Huffman strings (fin = 1 each). */
QH_EXPORT int qh_decode_batch(qh_ctx *ctx, const uint8_t *src,
                              const qh_span_in *in, size_t n, uint8_t *dst,
                              uint64_t dst_cap, qh_span_out *out, int where);

/* hlen[i] = nghttp3_qpack_huffman_encode_count(string i). */
QH_EXPORT int qh_encode_count_batch(qh_ctx *ctx, const uint8_t *src,
                                    const qh_span_in *in, size_t n,
                                    uint32_t *hlen, int where);

/* Huffman-encode n strings densely into dst (byte-identical to
 * nghttp3_qpack_huffman_encode per string). */
QH_EXPORT int qh_encode_batch(qh_ctx *ctx, const uint8_t *src,
                              const qh_span_in *in, size_t n, uint8_t *dst,
                              uint64_t dst_cap, qh_span_out *out, int where);

/* Per-kernel HIP-event timing of batch calls (off by default).  When on,
 * every kernel launch is bracketed by events on the context stream;
 * qh_ctx_kernel_times() synchronises and returns, for up to `cap` kernels,
 * their names, launch counts and summed milliseconds, then resets. */
QH_EXPORT int qh_ctx_enable_timing(qh_ctx *ctx, int on);
QH_EXPORT int qh_ctx_kernel_times(qh_ctx *ctx, const char **names,
                                  uint64_t *counts, double *ms, int cap);

/* Deterministic synthetic workloads generated on the device (bench/tests):
 * string i has length lo + splitmix64-draw % (hi - lo + 1) (dist 0, uniform)
 * or a Zipf(s)-distributed length in [lo, hi] (dist 1); strings are packed
 * back to back (in[i].off = prefix sum of lengths) and byte k of the packed
 * buffer is alphabet[draw(k) % alphabet_len].  See nghttp3_amd/synth.py for
 * the bit-exact host restatement. */
QH_EXPORT int qh_synth_spans(qh_ctx *ctx, uint64_t seed, size_t n, uint32_t lo,
                             uint32_t hi, int dist, double zipf_s,
                             qh_span_in *in_dev, uint64_t *total_dev);
QH_EXPORT int qh_synth_fill(qh_ctx *ctx, uint64_t seed, uint8_t *dst_dev,
                            uint64_t nbytes, const uint8_t *alphabet,
                            uint32_t alphabet_len);

/* Library version string. */
QH_EXPORT const char *qh_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QHUFF_H */
