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
/* qh_decode_batch only: HBM, asynchronous, the decoded strings packed back
 * to back in dst as with QH_WHERE_HOST (out[i].off = the decoded bytes
 * before string i); the strings are decoded into a context scratch buffer of
 * dst_cap bytes first, then packed (one more pass over the decoded bytes). */
#define QH_WHERE_DEVICE_DENSE 2

/* One string: bytes [off, off + len) of the batch's source buffer. */
typedef struct qh_span_in {
  uint64_t off;
  uint32_t len;
  uint32_t flags; /* QH_SPAN_* bits as written by the QPACK scanners below;
                     ignored by the Huffman batch calls */
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
  /* decode with QH_DECODER_WINDOWS / _SORTED: lock-step iterations (16
   * table lookups each) run by lanes, and by waves (each wave counts its
   * longest lane per window); lane_steps / (64 * wave_steps) is the active-
   * lane fraction.  Counted only by the instrumented development build
   * (make stamps: the counter slows the decoder); 0 otherwise. */
  uint64_t lane_steps;
  uint64_t wave_steps;
} qh_batch_stats;

typedef struct qh_ctx qh_ctx;

/* Bind a context to HIP device `device` and stream `stream` (a hipStream_t;
 * NULL = the device's default stream, as in other HIP libraries).  Every
 * batch call is ordered on that stream. */
QH_EXPORT int qh_ctx_new(qh_ctx **pctx, int device, void *stream);
QH_EXPORT void qh_ctx_del(qh_ctx *ctx);
QH_EXPORT int qh_ctx_set_stream(qh_ctx *ctx, void *stream);
/* Decoder kernel of qh_decode_batch (results are identical; speed is not):
 * QH_DECODER_WINDOWS (default) sorts each 256-string window by length and
 * decodes a window per workgroup -- fastest for header strings of similar
 * length (8-256 B, and the 1-128 B strings of whole field sections);
 * QH_DECODER_WAVES lets every wave sort and decode its own chunks of 256
 * strings with no workgroup barrier, its input staged through LDS in
 * 64-byte groups. */
#define QH_DECODER_WINDOWS 0
#define QH_DECODER_WAVES 1
/* QH_DECODER_SORTED: the window decoder over a batch-wide schedule --
 * three short passes over the spans sort the strings into 16-byte length
 * classes, longest first, so every 256-string window holds strings of one
 * class (same output layout).  For skewed lengths and binary text: on one
 * MI355X, Zipf lengths to 4 KiB decode 2.3x the wave decoder and 6x the
 * window decoder, binary text 1.3x; 8-256 B headers ~5% slower than
 * QH_DECODER_WINDOWS (the schedule's ~25 us). */
#define QH_DECODER_SORTED 2
QH_EXPORT int qh_ctx_set_decoder(qh_ctx *ctx, int kind);
/* Codes kernel of qh_encode_batch (results are identical; speed is not):
 * QH_ENCODER_AUTO (default) runs one of the two below per batch, chosen
 * from the strings of the context's previous encode (their lengths' spread
 * and mean, their encoded size; the first encode of a context uses the
 * window encoder): QH_ENCODER_FUSED for skewed, long or binary strings,
 * else QH_ENCODER_WINDOWS.
 * QH_ENCODER_WINDOWS encodes a sorted window of up to 256 strings
 * per workgroup into an LDS stage copied out with coalesced stores --
 * fastest for strings of similar length; QH_ENCODER_WAVES lets every wave
 * sort and encode its own chunks of 256 strings with no workgroup barrier,
 * each lane writing its string's 16-byte output chunks from an LDS ring --
 * fastest for skewed or long strings (Zipf up to 4 KiB: 2.3x). */
#define QH_ENCODER_WINDOWS 0
#define QH_ENCODER_WAVES 1
/* QH_ENCODER_FUSED: one pass over the plaintext -- every lane takes 16 bytes
 * of one string, whatever the string lengths; code bits are summed per
 * string, a decoupled look-back over 4 KiB tiles places each tile in the dense
 * output, and the codes go out through an LDS stage. */
#define QH_ENCODER_FUSED 2
#define QH_ENCODER_AUTO 3
/* QH_ENCODER_REGION: the length pass, then a codes pass that streams the
 * plaintext region of every 64 strings lying back to back in memory (lane j
 * of a wave: bytes [16 j, 16 j + 16) of each 1 KiB round, codes placed by a
 * prefix sum of their lengths and the strings' pads); strings in any other
 * layout a lane each.  QH_ENCODER_AUTO's choice for header text. */
#define QH_ENCODER_REGION 4
QH_EXPORT int qh_ctx_set_encoder(qh_ctx *ctx, int kind);
/* Tuning options (results are identical; speed is not).  The library reads
 * no environment variable that changes what it computes or which kernels
 * run: these are set explicitly, per context.
 * QH_OPT_LONG_MIN: QH_DECODER_SORTED decodes strings of at least `value`
 *   encoded bytes (their 16-byte length class and longer) with a workgroup
 *   per string; 0 turns that path off (default 4096; at most 2^30).
 * QH_OPT_LENS_LANE_PASS: 1 counts every string's encoded length a lane per
 *   string (the path the length kernel takes for scattered spans) instead
 *   of streaming the strings' region; 0 (default) chooses per window.
 * No reference counterpart (the reference codec has no batch kernels). */
#define QH_OPT_LONG_MIN 1
#define QH_OPT_LENS_LANE_PASS 2
QH_EXPORT int qh_ctx_set_option(qh_ctx *ctx, int option, int64_t value);
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
 * QH_ERR_NOMEM; nothing is written at or past dst_cap.  With QH_WHERE_HOST
 * the decoded strings come back packed: dst holds them back to back and
 * out[i].off = the sum of the decoded lengths before string i (only decoded
 * bytes cross PCIe; the batch is pipelined in slices over copy and compute
 * streams); dst_cap >= qh_decode_dst_size(in, n) still always suffices, and a
 * string whose bytes would pass dst_cap gets QH_ERR_NOMEM.
 * Encode output is dense: out[i].off = sum_{j<i} encode_count(string j);
 * qh_encode_dst_bound() is an upper bound. */
QH_EXPORT uint64_t qh_decode_dst_size(const qh_span_in *in, size_t n);
QH_EXPORT uint64_t qh_encode_dst_bound(const qh_span_in *in, size_t n);

/* Decode n complete Huffman strings (fin = 1 each). */
QH_EXPORT int qh_decode_batch(qh_ctx *ctx, const uint8_t *src,
                              const qh_span_in *in, size_t n, uint8_t *dst,
                              uint64_t dst_cap, qh_span_out *out, int where);

/* One host-memory batch (as qh_decode_batch with QH_WHERE_HOST) fanned out
 * over n_ctx contexts -- one per GPU, or several on one GPU with their own
 * streams: the strings are cut into n_ctx ranges of about equal encoded
 * bytes, in string order, and context k decodes range k from its own host
 * thread through its own H2D / decode / D2H pipeline (SURVEY.md section
 * 8(e): each GPU receives its shard by its own H2D; the reference has no
 * parallel path).  Range k's decoded strings are packed back to back from
 * dst + B_k, B_k = the sum of len * 8 / 5 (the reference's
 * estimate_decode_length, huffman.h:113-115) over the strings of the ranges
 * before it, so the strings are in global order with a gap between ranges
 * that never exceeds that estimate's slack; out[i].off is the offset in dst.
 * dst_cap >= qh_decode_dst_size(in, n) suffices.  Blocks until every range
 * is done; returns 0 or the first range's error. */
QH_EXPORT int qh_decode_batch_multi(qh_ctx *const *ctxs, int n_ctx, const uint8_t *src,
                                    const qh_span_in *in, size_t n, uint8_t *dst,
                                    uint64_t dst_cap, qh_span_out *out);

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
/* dst_dev[j] = byte first + j of that packed buffer (a rank generates its
 * own shard of a batch). */
QH_EXPORT int qh_synth_fill(qh_ctx *ctx, uint64_t seed, uint64_t first,
                            uint8_t *dst_dev, uint64_t nbytes,
                            const uint8_t *alphabet, uint32_t alphabet_len);

/* ---- QPACK field-line framing ---------
 * Host C (nghttp3_amd/csrc/qh_qpack.c).  The scanners turn whole encoded
 * field sections (request-stream header blocks) and encoder-stream bytes
 * into field lines plus (off, len, flags) string spans, ready for
 * qh_decode_batch (pass only the spans with QH_SPAN_HUFFMAN; the others are
 * raw octets).  Indices are returned as encoded (static, base-relative or
 * post-base); resolving them against the tables is the QPACK layer's job.
 * Replaces the framing of nghttp3_qpack_decoder_read_request
 * (lib/nghttp3_qpack.c:3347-3800) and nghttp3_qpack_decoder_read_encoder
 * (:2815-3150) around the per-string Huffman calls (:2737-2763). */
#define QH_ERR_QPACK_HEADER_TOO_LARGE (-109)     /* nghttp3.h:224 */
#define QH_ERR_QPACK_DECOMPRESSION_FAILED (-401) /* nghttp3.h:252 */
#define QH_ERR_QPACK_ENCODER_STREAM_ERROR (-402) /* nghttp3.h:259 */

#define QH_SPAN_HUFFMAN 0x1u /* H bit set: Huffman-coded string       */
#define QH_SPAN_NAME 0x2u    /* the string is a field name (else value) */

/* Field-line opcodes (qpack.c:3439-3495) and encoder-stream instructions
 * (qpack.c:2837-2875). */
#define QH_FL_INDEXED 1         /* 1Txxxxxx                           */
#define QH_FL_INDEXED_PB 2      /* 0001xxxx  post-base index           */
#define QH_FL_INDEXED_NAME 3    /* 01NTxxxx  name ref + value literal  */
#define QH_FL_INDEXED_NAME_PB 4 /* 0000Nxxx  post-base name ref + value */
#define QH_FL_LITERAL 5         /* 001NHxxx  name literal + value      */
#define QH_ES_INSERT_INDEXED 6  /* 1Txxxxxx  insert with name ref      */
#define QH_ES_INSERT 7          /* 01Hxxxxx  insert with literal name  */
#define QH_ES_SET_DTABLE_CAP 8  /* 001xxxxx                            */
#define QH_ES_DUPLICATE 9       /* 000xxxxx                            */

#define QH_FL_DYNAMIC 0x1u /* index refers to the dynamic table (T = 0) */
#define QH_FL_NEVER 0x2u   /* N bit: never index                        */

/* One field line or encoder instruction (24 B).  name / value are indices
 * into the span array of the same call, or -1. */
typedef struct qh_field_line {
  uint64_t index; /* table index / capacity as encoded; 0 for literals */
  uint8_t opcode; /* QH_FL_* or QH_ES_*                                */
  uint8_t flags;  /* QH_FL_DYNAMIC | QH_FL_NEVER                        */
  uint16_t reserved;
  int32_t name;
  int32_t value;
  uint32_t reserved2;
} qh_field_line;

/* Encoded field section prefix (RFC 9204 4.5.1, qpack.c:3369-3437). */
typedef struct qh_section_prefix {
  uint64_t ricnt;      /* Encoded Required Insert Count (not reconstructed) */
  uint64_t delta_base;
  uint32_t sign;
  uint32_t reserved;
} qh_section_prefix;

/* Scans one complete field section (fin = 1).  Returns 0, or the error
 * nghttp3_qpack_decoder_read_request would return for it:
 * QH_ERR_QPACK_DECOMPRESSION_FAILED (integer overflow, a representation cut
 * by the end of the section, :3780-3784, or an index no table state can
 * make valid: a static index >= 99, :3992 -> :2796-2797; with Required
 * Insert Count 0 a negative Delta Base, :3414-3418, or any dynamic
 * reference, :3985-3987, :4009-4011), QH_ERR_QPACK_HEADER_TOO_LARGE
 * (name > 256 / value > 65536 bytes, Huffman ones by their len*8/5
 * estimate, :3575-3588, :3661-3674), or QH_ERR_NOMEM when lines_cap /
 * spans_cap is too small.  On an error *nlines is 0 and *nspans counts the
 * strings read before it (the reference decodes those first, so a Huffman
 * failure among them takes precedence: -401).  Span offsets are src_off +
 * position in src.  Indices are not resolved: a section with a non-zero
 * Required Insert Count frames fine whatever the dynamic table holds. */
QH_EXPORT int qh_qpack_scan_field_section(
    const uint8_t *src, size_t srclen, uint64_t src_off,
    qh_section_prefix *prefix, qh_field_line *lines, size_t lines_cap,
    size_t *nlines, qh_span_in *spans, size_t spans_cap, size_t *nspans);

/* Batch of field sections: block i is src[blocks[i].off, +len).  Lines and
 * spans of block i are [line_start[i], line_start[i+1]) and likewise for
 * spans (both arrays hold nblocks + 1 entries); status[i] is block i's
 * framing verdict (a failed block contributes no lines, and the spans it
 * read before the error).  Returns 0, or QH_ERR_NOMEM when the caps are
 * exceeded. */
QH_EXPORT int qh_qpack_scan_blocks(const uint8_t *src,
                                   const qh_span_in *blocks, size_t nblocks,
                                   qh_field_line *lines, size_t lines_cap,
                                   qh_span_in *spans, size_t spans_cap,
                                   uint32_t *line_start, uint32_t *span_start,
                                   int32_t *status);

/* The same batch scan on the GPU (blocks, lines, spans, line_start,
 * span_start, status and huff in HBM; where must be QH_WHERE_DEVICE): same
 * parser source, same outputs and verdicts as qh_qpack_scan_blocks.  If
 * huff is not NULL it also receives the Huffman-coded spans alone, in
 * order, ready for qh_decode_batch.  totals (host, may be NULL) receives
 * {lines, spans, Huffman spans}.  Synchronises once (to check the totals
 * against the caps); returns 0, QH_ERR_NOMEM or QH_ERR_FATAL. */
QH_EXPORT int qh_scan_blocks_batch(qh_ctx *ctx, const uint8_t *src,
                                   const qh_span_in *blocks, size_t nblocks,
                                   qh_field_line *lines, size_t lines_cap,
                                   qh_span_in *spans, size_t spans_cap,
                                   uint32_t *line_start, uint32_t *span_start,
                                   int32_t *status, qh_span_in *huff,
                                   size_t huff_cap, uint64_t *totals,
                                   int where);

/* ---- Whole field sections in one call (decoder side of config 4) -------
 * Replaces the request-stream decode loop of nghttp3_qpack_decoder_read_request
 * (lib/nghttp3_qpack.c:3347-3805) for a batch of complete, independent field
 * sections (fin = 1 each): framing (the parser above), every Huffman string
 * decoded by the batch kernels (qpack_read_huffman_string, :2737-2763), a
 * Huffman failure turned into the block's DECOMPRESSION_FAILED (:3604-3609,
 * :3693-3698), then per string the field name / value check of
 * nghttp3_check_header_name / _value (http.c:691-709, :798-838) and, for
 * names, the token of qpack_lookup_token (qpack.c:342; the reference
 * computes it on emit, :4130).
 *
 * Outputs are caller-allocated (HBM for QH_WHERE_DEVICE, host memory for
 * QH_WHERE_HOST, where the call stages through the device and blocks):
 *   lines / spans / line_start / span_start / status -- as qh_qpack_scan_blocks
 *     (lines_cap, spans_cap >= total block bytes + 1 always suffice);
 *   strs[k]    -- string k: a Huffman string decoded into dst (off, len in
 *                 dst, status 0 or QH_ERR_QPACK_FATAL); a raw string is not
 *                 copied (off, len in src, status 0);
 *   verdict[k] -- 1 valid / 0 not (0 for a failed Huffman string); optional;
 *   token[k]   -- nghttp3_qpack_token of a name, -1 otherwise; optional;
 *   dst        -- decoded Huffman strings, qh_decode_batch's slot layout in
 *                 Huffman-string order; dst_cap >= the `dst_need` total.
 * status[b] is 0 or the reference's error for the block: its first framing
 * error, unless a Huffman string before it fails (-401).  A block whose
 * framing failed has no lines (its line_start range is empty) and keeps the
 * spans read before the error; a block that framed cleanly but whose
 * Huffman string failed (-401) keeps all its lines and spans -- the framing
 * is valid, the string's strs[k].status says which one failed -- where the
 * reference emits no field of it (the callers drop such a block's lines).
 * On QH_ERR_NOMEM the framing may have written lines and spans below the
 * caps; nothing else is written.
 * Totals (nlines, nspans, nhuff, dst_need) are filled in on return, also on
 * QH_ERR_NOMEM (caps or dst_cap too small: nothing was decoded; resize and
 * call again).  opts: QH_SECTIONS_DTABLE0 decodes as a decoder whose
 * dynamic table capacity is 0 (qpack_decode -s 0): any Required Insert
 * Count but 0 fails the block (reconstruct_ricnt, :3915-3950). */
#define QH_SECTIONS_DTABLE0 0x1u

typedef struct qh_sections {
  qh_field_line *lines;
  size_t lines_cap;
  qh_span_in *spans;
  size_t spans_cap;
  qh_span_out *strs;
  int8_t *verdict;
  int32_t *token;
  uint32_t *line_start; /* nblocks + 1 */
  uint32_t *span_start; /* nblocks + 1 */
  int32_t *status;      /* nblocks     */
  qh_section_prefix *prefixes; /* nblocks, optional: each block's prefix as
                                  encoded (zero for a block whose prefix
                                  does not parse) */
  uint8_t *dst;
  uint64_t dst_cap;
  /* filled in by the call */
  uint64_t nlines, nspans, nhuff, dst_need;
} qh_sections;

QH_EXPORT int qh_decode_sections_batch(qh_ctx *ctx, const uint8_t *src,
                                       const qh_span_in *blocks,
                                       size_t nblocks, uint32_t opts,
                                       qh_sections *out, int where);

/* Scans encoder-stream bytes.  Returns the number of bytes of complete
 * instructions (a trailing partial instruction is left for the next call,
 * like the streaming decoder), QH_ERR_QPACK_ENCODER_STREAM_ERROR (also for
 * a static name reference >= 99, qpack.c:2916 -> :3965-3966),
 * QH_ERR_QPACK_HEADER_TOO_LARGE or QH_ERR_NOMEM. */
QH_EXPORT nghttp3_ssize qh_qpack_scan_encoder_stream(
    const uint8_t *src, size_t srclen, uint64_t src_off, qh_field_line *insts,
    size_t insts_cap, size_t *ninsts, qh_span_in *spans, size_t spans_cap,
    size_t *nspans);

/* Prefixed integers, qpack.c:2643-2682 (nghttp3_qpack_put_varint_len /
 * nghttp3_qpack_put_varint). */
QH_EXPORT size_t qh_qpack_put_varint_len(uint64_t n, size_t prefix);
QH_EXPORT uint8_t *qh_qpack_put_varint(uint8_t *buf, uint64_t n,
                                       size_t prefix);

/* Representation writers; each returns the bytes written at dst.  fb is the
 * first byte's fixed bits and prefix the index / name-length prefix, as the
 * reference's callers pass them (qpack.c:1898-2069): indexed static 0xc0/6,
 * dynamic 0x80/6, post-base 0x10/4; name ref static 0x50/4 (| 0x20 never),
 * dynamic 0x40/4, post-base 0x00/3 (| 0x08); literal 0x20/3 (| 0x10);
 * inserts 0xc0/6, 0x80/6 (name ref) and 0x40/5 (literal name).  Strings
 * are Huffman-coded iff that is strictly shorter (:1862, :1954, :1962).
 * dst must hold qh_qpack_literal_bound(namelen, valuelen) bytes. */
QH_EXPORT size_t qh_qpack_write_indexed(uint8_t *dst, uint8_t fb,
                                        uint64_t idx, size_t prefix);
/* qpack_encoder_write_indexed_name, qpack.c:1851-1896 */
QH_EXPORT size_t qh_qpack_write_indexed_name(uint8_t *dst, uint8_t fb,
                                             uint64_t nameidx, size_t prefix,
                                             const uint8_t *value,
                                             size_t valuelen);
/* qpack_encoder_write_literal, qpack.c:1944-2006 */
QH_EXPORT size_t qh_qpack_write_literal(uint8_t *dst, uint8_t fb,
                                        size_t prefix, const uint8_t *name,
                                        size_t namelen, const uint8_t *value,
                                        size_t valuelen);
QH_EXPORT size_t qh_qpack_literal_bound(size_t namelen, size_t valuelen);

/* Batch writer of whole field sections (the encoder side of config 4):
 * section b is lines [line_start[b], line_start[b + 1]) (QH_FL_* opcodes;
 * name / value index `strs`, spans of `plain`) after its prefix (all zero
 * if prefixes is NULL).  sections[b] receives the section's (off, len) in
 * dst.  Returns 0, QH_ERR_NOMEM (dst_cap too small) or
 * QH_ERR_INVALID_ARGUMENT (unknown opcode / missing string). */
QH_EXPORT int qh_qpack_write_sections(const uint8_t *plain,
                                      const qh_span_in *strs,
                                      const qh_field_line *lines,
                                      const uint32_t *line_start,
                                      size_t nsections,
                                      const qh_section_prefix *prefixes,
                                      uint8_t *dst, size_t dst_cap,
                                      qh_span_in *sections);

/* ---- The encoder side of whole field sections (SURVEY.md section 8(a)
 * rows a9 / a10, 8(f) row 2) ----------------------------------------------
 * The static table (RFC 9204 Appendix A; the reference's stable[],
 * qpack.c:189-291): entry idx's name and value (static storage). */
QH_EXPORT int qh_qpack_static_entry(size_t idx, const uint8_t **name,
                                    size_t *namelen, const uint8_t **value,
                                    size_t *valuelen);

/* The representation nghttp3_qpack_encoder_encode_nv (qpack.c:1455-1628)
 * chooses for each of nfields fields when the dynamic table is not used
 * (capacity 0; qpack_encode -s 0): field i is strs[2i] (name) and
 * strs[2i + 1] (value), spans of `plain`; never[i] (optional) is its
 * NGHTTP3_NV_FLAG_NEVER_INDEX.  lines[i] becomes an Indexed Field Line
 * (static entry with that name and value), a Literal With (static) Name
 * Reference, or a Literal With Literal Name, with name / value = 2i / 2i + 1
 * where used and QH_FL_NEVER from never[i] (the static lookup also skips the
 * value match for authorization and cookie values under 20 bytes,
 * :1307-1321, :1643-1645).  Host C. */
QH_EXPORT int qh_qpack_plan_fields(const uint8_t *plain, const qh_span_in *strs,
                                   size_t nfields, const uint8_t *never,
                                   qh_field_line *lines);

/* Batch writer of whole field sections on the GPU: the encoder batch
 * adapter of the Huffman call sites (qpack.c:1851-2006).  Section b is
 * lines [line_start[b], line_start[b + 1]) after its prefix (prefixes[b], or
 * all zero when prefixes is NULL: no dynamic-table references); a line's
 * name / value index strs, spans of plain.  Steps: hlen of every string
 * (the count kernels), Huffman iff hlen < len (:1862, :1954, :1962), the
 * picked strings encoded densely (the encode kernels), then the sections
 * written (first bytes and prefixes as qh_qpack_write_sections; byte for
 * byte its output).  sections[b] receives (off, len) in dst, sections back
 * to back from 0; *dst_need the total.  All pointers in HBM
 * (QH_WHERE_DEVICE; one sync, for the caps check) or in host memory
 * (QH_WHERE_HOST: staged, blocking).  Returns 0, QH_ERR_NOMEM (dst_cap <
 * *dst_need; nothing written), QH_ERR_INVALID_ARGUMENT (unknown opcode or
 * missing string) or QH_ERR_FATAL. */
QH_EXPORT int qh_encode_sections_batch(qh_ctx *ctx, const uint8_t *plain,
                                       const qh_span_in *strs, size_t nstrs,
                                       const qh_field_line *lines,
                                       const uint32_t *line_start,
                                       size_t nsections,
                                       const qh_section_prefix *prefixes,
                                       uint8_t *dst, uint64_t dst_cap,
                                       qh_span_in *sections,
                                       uint64_t *dst_need, int where);

/* ---- Field name / value validation -------
 * Scalar drop-ins for the public functions (nghttp3.h:3443, :3452;
 * lib/nghttp3_http.c:691-709, :798-838), nghttp3_amd/csrc/qh_http.c. */
QH_EXPORT int nghttp3_check_header_name(const uint8_t *name, size_t len);
QH_EXPORT int nghttp3_check_header_value(const uint8_t *value, size_t len);

/* Batch form on the GPU: verdict[i] = nghttp3_check_header_name of string i
 * if in[i].flags has QH_SPAN_NAME, else nghttp3_check_header_value (1 valid,
 * 0 not), e.g. over the decode destination right after qh_decode_batch.
 * Device strings are read in aligned 16-byte chunks that each hold a byte
 * of the string (so no load leaves the string's pages; no padding is
 * needed).  Host batches are staged. */
QH_EXPORT int qh_check_fields_batch(qh_ctx *ctx, const uint8_t *src,
                                    const qh_span_in *in, size_t n,
                                    int8_t *verdict, int where);

/* ---- Header-name tokens ------------------
 * qh_qpack_lookup_token replaces the static qpack_lookup_token
 * (lib/nghttp3_qpack.c:342, generated by genlibtokenlookup.py): the
 * nghttp3_qpack_token of a field name (nghttp3.h:840-1131), or -1.  The
 * batch form looks up every string of a batch on the GPU (names decoded by
 * qh_decode_batch stay in HBM). */
QH_EXPORT int32_t qh_qpack_lookup_token(const uint8_t *name, size_t namelen);
QH_EXPORT int qh_lookup_tokens_batch(qh_ctx *ctx, const uint8_t *src,
                                     const qh_span_in *in, size_t n,
                                     int32_t *token, int where);

/* Library version string. */
QH_EXPORT const char *qh_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QHUFF_H */
