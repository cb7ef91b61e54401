/*
 * qh_scalar.c -- exact-signature drop-ins for nghttp3's private Huffman
 * codec (lib/nghttp3_qpack_huffman.h:42-107), linked into libqhuff.so.
 *
 * These are the streaming entry points: lib/nghttp3_qpack.c calls them per
 * chunk of a string that may still be arriving (qpack_read_huffman_string,
 * qpack.c:2737-2763, fin = 0 until the chunk reaching the string's end) and
 * per field while encoding (qpack.c:1861-1882, 1953-1993).  A chunk is a
 * handful of bytes, so they run on the host; whole strings go to the HIP
 * batch API (qh_decode_batch / qh_encode_batch) instead, which never calls
 * back into this file.
 *
 * The tables are the generated lists in qh_tables.h expanded into the
 * reference layouts and exported under the reference names
 * (lib/nghttp3_qpack_huffman_data.c:30,98).
 */
#include <string.h>

#include "../../include/qhuff.h"
#include "qh_tables.h"

#define QH_SYM_ENTRY(nbits, code) {nbits, code},
const nghttp3_qpack_huffman_sym huffman_sym_table[QH_NSYM] = {
    QH_SYM_LIST(QH_SYM_ENTRY)};

#define QH_NODE_ENTRY(w)                                                       \
  {(uint16_t)((w) & 0xFFFFu), (uint8_t)(((w) >> 16) & 0xFFu),                  \
   (uint8_t)((w) >> 24)},
#define QH_NODE_ROW(...) {__VA_ARGS__},
const nghttp3_qpack_huffman_decode_node qpack_huffman_decode_table[QH_NSTATE]
                                                                  [16] = {
    QH_FSM_ROWS(QH_NODE_ROW, QH_NODE_ENTRY)};

size_t nghttp3_qpack_huffman_encode_count(const uint8_t *src, size_t len) {
  size_t bits = 0;
  const uint8_t *end = src + len;
  while (src != end) bits += huffman_sym_table[*src++].nbits;
  return (bits + 7) / 8; /* trailing bits are EOS-prefix padding */
}

uint8_t *nghttp3_qpack_huffman_encode(uint8_t *dest, const uint8_t *src,
                                      size_t srclen) {
  uint64_t acc = 0; /* pending bits, MSB-first from bit 63 */
  size_t pending = 0;
  size_t i;
  for (i = 0; i < srclen; ++i) {
    const nghttp3_qpack_huffman_sym *s = &huffman_sym_table[src[i]];
    acc |= (uint64_t)s->code << (32 - pending);
    pending += s->nbits;
    if (pending >= 32) {
      const uint32_t word = (uint32_t)(acc >> 32);
      dest[0] = (uint8_t)(word >> 24); /* network byte order */
      dest[1] = (uint8_t)(word >> 16);
      dest[2] = (uint8_t)(word >> 8);
      dest[3] = (uint8_t)word;
      dest += 4;
      acc <<= 32;
      pending -= 32;
    }
  }
  while (pending >= 8) {
    *dest++ = (uint8_t)(acc >> 56);
    acc <<= 8;
    pending -= 8;
  }
  if (pending) {
    const uint8_t pad = (uint8_t)((1u << (8 - pending)) - 1);
    *dest++ = (uint8_t)((uint8_t)(acc >> 56) | pad);
  }
  return dest;
}

void nghttp3_qpack_huffman_decode_context_init(
    nghttp3_qpack_huffman_decode_context *ctx) {
  ctx->fstate = 0;
  ctx->flags = NGHTTP3_QPACK_HUFFMAN_FLAG_ACCEPTED;
}

nghttp3_ssize nghttp3_qpack_huffman_decode(
    nghttp3_qpack_huffman_decode_context *ctx, uint8_t *dest,
    const uint8_t *src, size_t srclen, int fin) {
  uint8_t *out = dest;
  uint16_t state = ctx->fstate;
  uint8_t flags = ctx->flags;
  size_t i;
  for (i = 0; i < srclen; ++i) {
    const uint8_t c = src[i];
    const nghttp3_qpack_huffman_decode_node *hi =
        &qpack_huffman_decode_table[state][c >> 4];
    if (hi->flags & NGHTTP3_QPACK_HUFFMAN_FLAG_SYM) *out++ = hi->sym;
    const nghttp3_qpack_huffman_decode_node *lo =
        &qpack_huffman_decode_table[hi->fstate][c & 0x0Fu];
    if (lo->flags & NGHTTP3_QPACK_HUFFMAN_FLAG_SYM) *out++ = lo->sym;
    state = lo->fstate;
    flags = lo->flags;
  }
  ctx->fstate = state;
  ctx->flags = flags;
  if (fin && !(flags & NGHTTP3_QPACK_HUFFMAN_FLAG_ACCEPTED))
    return QH_ERR_QPACK_FATAL;
  return out - dest;
}

int nghttp3_qpack_huffman_decode_failure_state(
    const nghttp3_qpack_huffman_decode_context *ctx) {
  return ctx->fstate == QH_FAIL_STATE;
}
