/*
 * QPACK field-section parser core, shared by the host library (qh_qpack.c)
 * and the GPU framing kernel (qh_frame.inc): one source, so the two paths
 * cannot drift.  QH_HD is empty for C and __host__ __device__ for HIP.
 * Counting mode: a scan_out with lines == NULL / spans == NULL counts lines
 * and spans without storing them.  See qh_qpack.c for the reference lines.
 */
#ifndef QH_QPACK_CORE_H
#define QH_QPACK_CORE_H

#ifndef QH_HD
#define QH_HD
#endif

#define QH_QPACK_INT_MAX ((1ull << 62) - 1) /* nghttp3_qpack.h:43 */
#define QH_QPACK_MAX_NAMELEN 256            /* nghttp3_qpack.h:47 */
#define QH_QPACK_MAX_VALUELEN 65536         /* nghttp3_qpack.h:50 */
#define QH_QPACK_STATIC_ENTRIES 99          /* stable[], qpack.c:52-189 */

/* Reads an N-bit-prefix integer starting at *pp (the first byte's prefix
 * bits).  Returns 1 when complete, 0 when the input ends first, or
 * QH_ERR_QPACK_FATAL on overflow -- the same verdicts as
 * qpack_read_varint (qpack.c:2481-2543) given the whole input at once. */
QH_HD static inline int read_varint(uint64_t *res, const uint8_t **pp, const uint8_t *end,
                       unsigned prefix) {
  const uint8_t *p = *pp;
  uint64_t k = (uint8_t)((1u << prefix) - 1);
  uint64_t n, add;
  unsigned shift = 0;

  if (p == end) {
    return 0;
  }
  if ((*p & k) != k) {
    *res = *p & k;
    *pp = p + 1;
    return 1;
  }
  n = k;
  for (++p; p != end; ++p, shift += 7) {
    add = *p & 0x7fu;
    if (shift > 62) {
      return QH_ERR_QPACK_FATAL;
    }
    if ((QH_QPACK_INT_MAX >> shift) < add) {
      return QH_ERR_QPACK_FATAL;
    }
    add <<= shift;
    if (QH_QPACK_INT_MAX - add < n) {
      return QH_ERR_QPACK_FATAL;
    }
    n += add;
    if ((*p & 0x80u) == 0) {
      *res = n;
      *pp = p + 1;
      return 1;
    }
  }
  return 0;
}

#ifndef QH_LONG_MIN
#define QH_LONG_MIN 4096u /* qh_peek_dec.inc kDeferMin */
#endif

typedef struct scan_out {
  qh_field_line *lines;
  size_t lines_cap, nlines;
  qh_span_in *spans;
  size_t spans_cap, nspans;
  qh_field_line scratch;
  size_t nhuff;    /* Huffman-coded strings seen */
  uint64_t hslots; /* their batch-decode slot bytes (include/qhuff.h) */
  uint32_t opts; /* QH_SECTIONS_DTABLE0: the decoder's table capacity is 0 */
  /* (the GPU framing's write pass; zero elsewhere) lines name batch-global
   * spans (span_base + the block's own index); every span's record goes to
   * aux[] (block << 32 | its Huffman index, ~0u for a raw string) and every
   * Huffman span also to huff[huff_base + its index among them] */
  qh_span_in *huff;
  uint64_t *aux;
  uint64_t span_base, huff_base, block;
  /* Huffman strings of at least QH_LONG_MIN encoded bytes (the GPU
   * pipeline decodes them a workgroup each, qh_k_dec_long_list) */
  uint64_t nlong;
  /* (the GPU framing's count pass) where each line starts, as an offset
   * into the section, for its first lstarts_cap lines */
  uint16_t *lstarts;
  uint32_t lstarts_cap;
} scan_out;

/* One string literal: H bit at bit `prefix` of the first byte, then the
 * prefixed length, then the bytes.  Checks the decoder's size limits on
 * the (estimated, for Huffman) decoded length (qpack.c:3575-3588,
 * :3661-3674).  Returns 1, 0 (truncated), or a negative error. */
QH_HD static inline int read_string(scan_out *o, int32_t *span_idx, const uint8_t *base,
                       uint64_t base_off, const uint8_t **pp,
                       const uint8_t *end, unsigned prefix, uint64_t limit,
                       uint32_t kind, int too_large_rv, int bad_rv) {
  const uint8_t *p = *pp;
  uint64_t len;
  uint32_t h;
  int rv;
  qh_span_in *s;

  if (p == end) {
    return 0;
  }
  h = (*p & (1u << prefix)) ? QH_SPAN_HUFFMAN : 0;
  rv = read_varint(&len, &p, end, prefix);
  if (rv < 0) {
    return bad_rv;
  }
  if (rv == 0) {
    return 0;
  }
  if (len > limit) {
    return too_large_rv;
  }
  if (h && len * 8 / 5 > limit) { /* nghttp3_qpack_huffman.h:113-115 */
    return too_large_rv;
  }
  if ((uint64_t)(end - p) < len) {
    return 0;
  }
  if (o->nspans == o->spans_cap) {
    return QH_ERR_NOMEM;
  }
  if (o->spans) { /* one whole-record store (the GPU framing kernel) */
    qh_span_in rec;
    rec.off = base_off + (uint64_t)(p - base);
    rec.len = (uint32_t)len;
    rec.flags = h | kind;
    s = &o->spans[o->nspans];
    *s = rec;
  }
  if (o->aux) {
    o->aux[o->nspans] = (o->block << 32) | (h ? (uint32_t)(o->huff_base + o->nhuff) : 0xFFFFFFFFu);
  }
  if (h && o->huff && o->spans) {
    o->huff[o->huff_base + o->nhuff] = o->spans[o->nspans];
  }
  *span_idx = (int32_t)(o->span_base + o->nspans++);
  o->nhuff += h ? 1 : 0;
  /* the slot qh_decode_batch gives it: len * 8 / 5 + 16, rounded up to 64 */
  o->hslots += h ? ((len * 8 / 5 + 16 + 63) & ~(uint64_t)63) : 0;
  o->nlong += h && len >= QH_LONG_MIN ? 1 : 0;
  *pp = p + len;
  return 1;
}

QH_HD static inline qh_field_line *new_line(scan_out *o, uint8_t opcode, uint8_t flags) {
  qh_field_line *l;
  if (o->nlines == o->lines_cap) {
    return NULL;
  }
  /* counting mode: lines land in a scratch slot */
  l = o->lines ? &o->lines[o->nlines] : &o->scratch;
  ++o->nlines;
  l->index = 0;
  l->reserved = 0;
  l->reserved2 = 0;
  l->opcode = opcode;
  l->flags = flags;
  l->name = -1;
  l->value = -1;
  return l;
}

QH_HD static inline int scan_section(scan_out *o, const uint8_t *src, size_t srclen,
                        uint64_t src_off, qh_section_prefix *prefix) {
  const uint8_t *p = src, *end = src + srclen;
  const int bad = QH_ERR_QPACK_DECOMPRESSION_FAILED;
  const int big = QH_ERR_QPACK_HEADER_TOO_LARGE;
  qh_section_prefix pf;
  int rv;

  /* Section prefix, qpack.c:3369-3437: Required Insert Count (8-bit
   * prefix), then sign bit + Delta Base (7-bit prefix). */
  rv = read_varint(&pf.ricnt, &p, end, 8);
  if (rv <= 0) {
    return bad;
  }
  /* nghttp3_qpack_decoder_reconstruct_ricnt (qpack.c:3915-3950): with a
   * hard table capacity of 0 there are no entries (full = 0), so any
   * encoded count but 0 fails. */
  if ((o->opts & QH_SECTIONS_DTABLE0) && pf.ricnt != 0) {
    return bad;
  }
  if (p == end) {
    return bad;
  }
  pf.sign = (*p & 0x80u) ? 1 : 0;
  pf.reserved = 0;
  rv = read_varint(&pf.delta_base, &p, end, 7);
  if (rv <= 0) {
    return bad;
  }
  /* qpack.c:3414-3418: a negative Delta Base needs ricnt > delta_base; an
   * encoded count of 0 is a reconstructed count of 0 (:3919-3921), whatever
   * the table holds. */
  if (pf.sign && pf.ricnt == 0) {
    return bad;
  }
  if (prefix) {
    *prefix = pf;
  }

  while (p != end) {
    uint8_t b = *p, opcode, flags = 0;
    unsigned iprefix;
    int has_name_idx = 1, has_value = 1;
    qh_field_line cur, *l = &cur; /* built here, stored whole at its end */
    size_t li;

    /* qpack.c:3439-3495 */
    if (b & 0x80u) {
      opcode = QH_FL_INDEXED;
      flags = (b & 0x40u) ? 0 : QH_FL_DYNAMIC;
      iprefix = 6;
      has_value = 0;
    } else if (b & 0x40u) {
      opcode = QH_FL_INDEXED_NAME;
      flags = (uint8_t)(((b & 0x20u) ? QH_FL_NEVER : 0) |
                        ((b & 0x10u) ? 0 : QH_FL_DYNAMIC));
      iprefix = 4;
    } else if (b & 0x20u) {
      opcode = QH_FL_LITERAL;
      flags = (b & 0x10u) ? QH_FL_NEVER : 0;
      iprefix = 3;
      has_name_idx = 0;
    } else if (b & 0x10u) {
      opcode = QH_FL_INDEXED_PB;
      flags = QH_FL_DYNAMIC;
      iprefix = 4;
      has_value = 0;
    } else {
      opcode = QH_FL_INDEXED_NAME_PB;
      flags = (uint8_t)(QH_FL_DYNAMIC | ((b & 0x08u) ? QH_FL_NEVER : 0));
      iprefix = 3;
    }
    if (o->nlines == o->lines_cap) {
      return QH_ERR_NOMEM;
    }
    li = o->nlines++; /* (a line cut short by an error is never stored: the
                          callers drop a failed block's lines) */
    if (o->lstarts && li < o->lstarts_cap) {
      o->lstarts[li] = (uint16_t)(p - src);
    }
    cur.index = 0;
    cur.reserved = 0;
    cur.reserved2 = 0;
    cur.opcode = opcode;
    cur.flags = flags;
    cur.name = -1;
    cur.value = -1;
    if (has_name_idx) {
      rv = read_varint(&l->index, &p, end, iprefix);
      if (rv <= 0) {
        return bad; /* overflow, or unfinished at fin (:3780-3784) */
      }
      /* brel2abs / pbrel2abs (qpack.c:3971-4017), the checks that need no
       * table state: a static index must be < 99 (validate_index,
       * :2796-2797); with Required Insert Count 0 every dynamic reference
       * has absidx >= ricnt = 0 (:3985-3987, :4009-4011). */
      if (flags & QH_FL_DYNAMIC) {
        if (pf.ricnt == 0) {
          return bad;
        }
      } else if (l->index >= QH_QPACK_STATIC_ENTRIES) {
        return bad;
      }
    } else {
      rv = read_string(o, &l->name, src, src_off, &p, end, 3,
                       QH_QPACK_MAX_NAMELEN, QH_SPAN_NAME, big, bad);
      if (rv <= 0) {
        return rv < 0 ? rv : bad;
      }
    }
    if (has_value) {
      rv = read_string(o, &l->value, src, src_off, &p, end, 7,
                       QH_QPACK_MAX_VALUELEN, 0, big, bad);
      if (rv <= 0) {
        return rv < 0 ? rv : bad;
      }
    }
    if (o->lines) {
      o->lines[li] = cur;
    }
  }
  return 0;
}

#endif /* QH_QPACK_CORE_H */
