/*
 * QPACK field-line framing around the Huffman strings (SURVEY.md section
 * 8(f) rows 1 and 2): host-side scanners that turn whole encoded field
 * sections and encoder-stream bytes into (offset, length, H) string spans
 * for the batch Huffman decoder, and the representation writers that emit
 * field lines around the batch encoder's output.
 *
 * Reference behaviour restated here (lib/nghttp3_qpack.c):
 *   - prefixed integers: qpack_read_varint :2481-2543 (limit 2^62-1,
 *     NGHTTP3_QPACK_INT_MAX, lib/nghttp3_qpack.h:43), put_varint_len /
 *     put_varint :2643-2682;
 *   - request-stream field section: nghttp3_qpack_decoder_read_request
 *     :3347-3800 (section prefix :3369-3437, opcodes :3439-3495, name and
 *     value length checks :3562-3602 / :3648-3691, fin on an unfinished
 *     representation :3780-3784);
 *   - encoder stream: nghttp3_qpack_decoder_read_encoder :2815-3150
 *     (opcodes :2837-2875);
 *   - representation writers: qpack_encoder_write_indexed_name :1851-1896,
 *     qpack_encoder_write_literal :1944-2006 and their callers'
 *     first bytes and prefixes :1898-2069.
 *
 * The scanners only frame: they do not resolve table indices (the dynamic
 * table lives in the QPACK layer, out of scope) and do not decode strings
 * (the GPU batch does).  Everything here is plain C on the host: parsing
 * is a serial byte walk per section, and sections shard across threads or
 * ranks by block.
 */
#include <string.h>

#include "../../include/qhuff.h"

#include "qh_qpack_core.h"

QH_EXPORT int qh_qpack_scan_field_section(
  const uint8_t *src, size_t srclen, uint64_t src_off,
  qh_section_prefix *prefix, qh_field_line *lines, size_t lines_cap,
  size_t *nlines, qh_span_in *spans, size_t spans_cap, size_t *nspans) {
  scan_out o = {.lines = lines, .lines_cap = lines_cap, .spans = spans, .spans_cap = spans_cap};
  int rv;

  if ((src == NULL && srclen) || nlines == NULL || nspans == NULL ||
      (lines == NULL && lines_cap) || (spans == NULL && spans_cap)) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  rv = scan_section(&o, src, srclen, src_off, prefix);
  *nlines = rv ? 0 : o.nlines; /* on error: no lines, the strings read so far */
  *nspans = o.nspans;
  return rv;
}

QH_EXPORT int qh_qpack_scan_blocks(const uint8_t *src,
                                   const qh_span_in *blocks, size_t nblocks,
                                   qh_field_line *lines, size_t lines_cap,
                                   qh_span_in *spans, size_t spans_cap,
                                   uint32_t *line_start, uint32_t *span_start,
                                   int32_t *status) {
  scan_out o = {.lines = lines, .lines_cap = lines_cap, .spans = spans, .spans_cap = spans_cap};
  size_t i;

  if ((src == NULL && nblocks) || (blocks == NULL && nblocks) ||
      line_start == NULL || span_start == NULL ||
      (status == NULL && nblocks) || lines_cap > UINT32_MAX ||
      spans_cap > UINT32_MAX) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  for (i = 0; i < nblocks; ++i) {
    size_t l0 = o.nlines, s0 = o.nspans;
    int rv;
    line_start[i] = (uint32_t)l0;
    span_start[i] = (uint32_t)s0;
    rv = scan_section(&o, src + blocks[i].off, blocks[i].len, blocks[i].off,
                      NULL);
    if (rv == QH_ERR_NOMEM) {
      line_start[nblocks] = (uint32_t)l0;
      span_start[nblocks] = (uint32_t)s0;
      return QH_ERR_NOMEM;
    }
    status[i] = rv;
    if (rv != 0) { /* a bad section keeps the strings read before the error,
                      and no lines */
      o.nlines = l0;
    }
  }
  line_start[nblocks] = (uint32_t)o.nlines;
  span_start[nblocks] = (uint32_t)o.nspans;
  return 0;
}

QH_EXPORT nghttp3_ssize qh_qpack_scan_encoder_stream(
  const uint8_t *src, size_t srclen, uint64_t src_off, qh_field_line *insts,
  size_t insts_cap, size_t *ninsts, qh_span_in *spans, size_t spans_cap,
  size_t *nspans) {
  scan_out o = {.lines = insts, .lines_cap = insts_cap, .spans = spans, .spans_cap = spans_cap};
  const uint8_t *p = src, *end = src + srclen, *done = src;
  const int bad = QH_ERR_QPACK_ENCODER_STREAM_ERROR;
  const int big = QH_ERR_QPACK_HEADER_TOO_LARGE; /* qpack.c:2962-2972 */
  int rv = 0;

  if ((src == NULL && srclen) || ninsts == NULL || nspans == NULL ||
      (insts == NULL && insts_cap) || (spans == NULL && spans_cap)) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  /* qpack.c:2837-2875.  An instruction cut by the end of the input is left
   * for the next call: the return value counts complete instructions. */
  while (p != end) {
    uint8_t b = *p;
    size_t l0 = o.nlines, s0 = o.nspans;
    qh_field_line *l;

    if (b & 0x80u) {
      l = new_line(&o, QH_ES_INSERT_INDEXED, (b & 0x40u) ? 0 : QH_FL_DYNAMIC);
      if (l == NULL) {
        rv = QH_ERR_NOMEM;
        break;
      }
      rv = read_varint(&l->index, &p, end, 6);
      /* rel2abs -> validate_index (qpack.c:3952-3969, :2796-2797): a
       * static name reference must be < 99, whatever the table holds */
      if (rv > 0 && !(l->flags & QH_FL_DYNAMIC) &&
          l->index >= QH_QPACK_STATIC_ENTRIES) {
        rv = bad;
      }
      if (rv > 0) {
        rv = read_string(&o, &l->value, src, src_off, &p, end, 7,
                         QH_QPACK_MAX_VALUELEN, 0, big, bad);
      }
    } else if (b & 0x40u) {
      l = new_line(&o, QH_ES_INSERT, 0);
      if (l == NULL) {
        rv = QH_ERR_NOMEM;
        break;
      }
      rv = read_string(&o, &l->name, src, src_off, &p, end, 5,
                       QH_QPACK_MAX_NAMELEN, QH_SPAN_NAME, big, bad);
      if (rv > 0) {
        rv = read_string(&o, &l->value, src, src_off, &p, end, 7,
                         QH_QPACK_MAX_VALUELEN, 0, big, bad);
      }
    } else {
      l = new_line(&o, (b & 0x20u) ? QH_ES_SET_DTABLE_CAP : QH_ES_DUPLICATE,
                   (b & 0x20u) ? 0 : QH_FL_DYNAMIC);
      if (l == NULL) {
        rv = QH_ERR_NOMEM;
        break;
      }
      rv = read_varint(&l->index, &p, end, 5);
    }
    if (rv < 0) {
      if (rv == QH_ERR_QPACK_FATAL) {
        rv = bad;
      }
      o.nlines = l0;
      o.nspans = s0;
      break;
    }
    if (rv == 0) { /* truncated: roll back this instruction */
      o.nlines = l0;
      o.nspans = s0;
      break;
    }
    done = p;
    rv = 0;
  }
  *ninsts = o.nlines;
  *nspans = o.nspans;
  if (rv < 0) {
    return rv;
  }
  return (nghttp3_ssize)(done - src);
}

/* ---- representation writers ---- */

QH_EXPORT size_t qh_qpack_put_varint_len(uint64_t n, size_t prefix) {
  size_t k = (size_t)((1 << prefix) - 1);
  size_t len = 0;
  if (n < k) {
    return 1;
  }
  n -= k;
  ++len;
  for (; n >= 128; n >>= 7, ++len)
    ;
  return len + 1;
}

QH_EXPORT uint8_t *qh_qpack_put_varint(uint8_t *buf, uint64_t n,
                                       size_t prefix) {
  size_t k = (size_t)((1 << prefix) - 1);
  *buf = (uint8_t)(*buf & ~k);
  if (n < k) {
    *buf = (uint8_t)(*buf | n);
    return buf + 1;
  }
  *buf = (uint8_t)(*buf | k);
  ++buf;
  n -= k;
  for (; n >= 128; n >>= 7) {
    *buf++ = (uint8_t)((1 << 7) | (n & 0x7f));
  }
  *buf++ = (uint8_t)n;
  return buf;
}

/* A string literal whose H flag sits at bit `prefix` of the first byte
 * (already holding the caller's high bits): Huffman iff it is strictly
 * shorter (qpack.c:1862, :1954, :1962). */
static uint8_t *put_string(uint8_t *p, size_t prefix, const uint8_t *s,
                           size_t len) {
  size_t hlen = nghttp3_qpack_huffman_encode_count(s, len);
  if (hlen < len) {
    *p = (uint8_t)(*p | (1u << prefix));
    p = qh_qpack_put_varint(p, hlen, prefix);
    return nghttp3_qpack_huffman_encode(p, s, len);
  }
  p = qh_qpack_put_varint(p, len, prefix);
  if (len) {
    memcpy(p, s, len);
  }
  return p + len;
}

QH_EXPORT size_t qh_qpack_write_indexed(uint8_t *dst, uint8_t fb,
                                        uint64_t idx, size_t prefix) {
  *dst = fb;
  return (size_t)(qh_qpack_put_varint(dst, idx, prefix) - dst);
}

QH_EXPORT size_t qh_qpack_write_indexed_name(uint8_t *dst, uint8_t fb,
                                             uint64_t nameidx, size_t prefix,
                                             const uint8_t *value,
                                             size_t valuelen) {
  uint8_t *p;
  *dst = fb;
  p = qh_qpack_put_varint(dst, nameidx, prefix);
  *p = 0;
  p = put_string(p, 7, value, valuelen);
  return (size_t)(p - dst);
}

QH_EXPORT size_t qh_qpack_write_literal(uint8_t *dst, uint8_t fb,
                                        size_t prefix, const uint8_t *name,
                                        size_t namelen, const uint8_t *value,
                                        size_t valuelen) {
  uint8_t *p;
  *dst = fb;
  p = put_string(dst, prefix, name, namelen);
  *p = 0;
  p = put_string(p, 7, value, valuelen);
  return (size_t)(p - dst);
}

QH_EXPORT size_t qh_qpack_literal_bound(size_t namelen, size_t valuelen) {
  return 10 + namelen + 10 + valuelen;
}

/* Batch representation writer: section b is field lines
 * [line_start[b], line_start[b + 1]) written after its prefix (encoded
 * Required Insert Count, sign, Delta Base; all zero when prefixes is NULL,
 * i.e. no dynamic-table references).  Each line's strings are spans of
 * `plain` (strs[line.name], strs[line.value]); first bytes and prefixes
 * follow the reference encoder for the opcode and flags (qpack.c:1898-2069,
 * static vs dynamic by QH_FL_DYNAMIC, N bit by QH_FL_NEVER). */
QH_EXPORT int qh_qpack_write_sections(const uint8_t *plain,
                                      const qh_span_in *strs,
                                      const qh_field_line *lines,
                                      const uint32_t *line_start,
                                      size_t nsections,
                                      const qh_section_prefix *prefixes,
                                      uint8_t *dst, size_t dst_cap,
                                      qh_span_in *sections) {
  uint8_t *p = dst, *end = dst + dst_cap;
  size_t b;
  uint32_t i;

  if ((nsections && (line_start == NULL || sections == NULL)) ||
      (dst == NULL && dst_cap)) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  for (b = 0; b < nsections; ++b) {
    uint8_t *s0 = p;
    uint64_t ricnt = prefixes ? prefixes[b].ricnt : 0;
    uint64_t dbase = prefixes ? prefixes[b].delta_base : 0;
    if ((size_t)(end - p) < 20) {
      return QH_ERR_NOMEM;
    }
    *p = 0;
    p = qh_qpack_put_varint(p, ricnt, 8);
    *p = (prefixes && prefixes[b].sign) ? 0x80 : 0;
    p = qh_qpack_put_varint(p, dbase, 7);
    for (i = line_start[b]; i < line_start[b + 1]; ++i) {
      const qh_field_line *l = &lines[i];
      int dyn = (l->flags & QH_FL_DYNAMIC) != 0;
      int never = (l->flags & QH_FL_NEVER) != 0;
      const qh_span_in *nm = l->name >= 0 ? &strs[l->name] : NULL;
      const qh_span_in *v = l->value >= 0 ? &strs[l->value] : NULL;
      size_t need = qh_qpack_literal_bound(nm ? nm->len : 0, v ? v->len : 0);
      if ((size_t)(end - p) < need) {
        return QH_ERR_NOMEM;
      }
      switch (l->opcode) {
      case QH_FL_INDEXED:
        p += qh_qpack_write_indexed(p, dyn ? 0x80 : 0xc0, l->index, 6);
        break;
      case QH_FL_INDEXED_PB:
        p += qh_qpack_write_indexed(p, 0x10, l->index, 4);
        break;
      case QH_FL_INDEXED_NAME:
      case QH_FL_INDEXED_NAME_PB:
        if (v == NULL) {
          return QH_ERR_INVALID_ARGUMENT;
        }
        if (l->opcode == QH_FL_INDEXED_NAME) {
          p += qh_qpack_write_indexed_name(
            p, (uint8_t)(0x40 | (never ? 0x20 : 0) | (dyn ? 0 : 0x10)),
            l->index, 4, plain + v->off, v->len);
        } else {
          p += qh_qpack_write_indexed_name(p, never ? 0x08 : 0, l->index, 3,
                                           plain + v->off, v->len);
        }
        break;
      case QH_FL_LITERAL:
        if (v == NULL || nm == NULL) {
          return QH_ERR_INVALID_ARGUMENT;
        }
        p += qh_qpack_write_literal(p, never ? 0x30 : 0x20, 3,
                                    plain + nm->off, nm->len, plain + v->off,
                                    v->len);
        break;
      default:
        return QH_ERR_INVALID_ARGUMENT;
      }
    }
    sections[b].off = (uint64_t)(s0 - dst);
    sections[b].len = (uint32_t)(p - s0);
    sections[b].flags = 0;
  }
  return 0;
}
