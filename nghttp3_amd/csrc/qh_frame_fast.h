/*
 * The GPU framing count pass's parse of one staged block (qh_frame.inc's
 * qh_k_frame_count; a restatement of qh_qpack_core.h's scan_section in
 * counting mode for a lane of a wave whose lanes parse different blocks).
 * Host-and-device code (QH_HD), so tests/test_frame_fast.py compiles it on
 * the host and compares it with scan_section block by block.
 */
#ifndef QH_FRAME_FAST_H
#define QH_FRAME_FAST_H

#ifndef QH_HD
#define QH_HD
#endif

QH_HD inline uint32_t fr_min(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Line starts the count pass keeps per block (offsets into the block, u16):
// the write pass parses the lines of a block with at most this many lines
// (and under 64 KiB) a lane each, kFrLines lanes per block.
static constexpr uint32_t kFrLines = 32;

// The count pass's parse of a staged block (qh_qpack_core.h's scan_section
// in counting mode, restated for a lane of a wave whose 64 lanes parse 64
// different blocks): each field line is read as at most two windows of four
// bytes whose loads issue together (the line's first bytes; its value's
// first bytes), and the line's kind, prefixes and lengths are selects rather
// than branches.  It only ever answers for a block it finds clean: any
// check scan_section would fail, an integer past four bytes, or a section
// that ends inside a line returns false, and the caller parses that block
// with scan_section, whose verdicts (and counts up to the error) are the
// reference's.
struct FrCounts {
  uint32_t lines, spans, huff, nlong;
  uint64_t slots;
};
// Eight bytes of the stage from offset o: three aligned dword reads issued
// together, funnel-shifted (the stage has 16 bytes of slack; bytes past the
// block are its neighbour's and never decide a verdict: every use below is
// bounded by the block's length).
QH_HD inline uint64_t fr_win8(const uint8_t *stage, uint32_t o) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(stage + (o & ~3u));
  const uint64_t lo = (uint64_t)w[0] | (uint64_t)w[1] << 32;
  const uint32_t hi = w[2], sh = 8u * (o & 3u);
  return sh ? (lo >> sh) | ((uint64_t)hi << (64u - sh)) : lo;
}
// An integer with a k-bit prefix at the start of window w: its value and
// the bytes it takes (0: longer than the window).  Arithmetic, no branches.
QH_HD inline uint32_t fr_varint(uint32_t w, uint32_t k, uint32_t &used) {
  const uint32_t m = (1u << k) - 1u, b0 = w & m;
  const uint32_t c1 = b0 == m ? 1u : 0u;          // a second byte
  const uint32_t c2 = c1 & ((w >> 15) & 1u);      // a third
  const uint32_t c3 = c2 & ((w >> 23) & 1u);      // a fourth
  const uint32_t c4 = c3 & (w >> 31);             // more: not answered here
  used = c4 ? 0u : 1u + c1 + c2 + c3;
  return b0 + (c1 ? (w >> 8) & 0x7Fu : 0u) + (c2 ? ((w >> 16) & 0x7Fu) << 7 : 0u) +
         (c3 ? ((w >> 24) & 0x7Fu) << 14 : 0u);
}
// Decode-slot bytes of a Huffman string of len encoded bytes (include/qhuff.h).
QH_HD inline uint32_t fr_slot(uint32_t len) { return (len * 8 / 5 + 16 + 63) & ~63u; }
QH_HD inline bool frame_count_fast(const uint8_t *stage, uint32_t at, uint32_t len,
                                                 uint32_t opts, FrCounts &o, qh_section_prefix &pf,
                                                 uint16_t *lstarts) {
  o = FrCounts{0, 0, 0, 0, 0};
  if (len < 2) return false;
  // section prefix (qpack.c:3369-3437)
  uint32_t u0, u1;
  const uint64_t w8 = fr_win8(stage, at);
  const uint32_t ric = fr_varint((uint32_t)w8, 8, u0);
  if (!u0 || u0 >= len) return false;
  const uint32_t w1 = (uint32_t)(w8 >> (8 * u0));
  const uint32_t db = fr_varint(w1, 7, u1);
  if (!u1 || u0 + u1 > len) return false;
  pf.ricnt = ric;
  pf.sign = (w1 & 0x80u) ? 1 : 0;
  pf.reserved = 0;
  pf.delta_base = db;
  if (((opts & QH_SECTIONS_DTABLE0) && ric != 0) || (pf.sign && ric == 0)) return false;
  uint32_t q = u0 + u1, prev = 0, slots = 0;
  uint32_t li = 0;
  bool bad = false;
  // (one exit: a lane leaves the loop at its block's end or at the first
  // check that fails; the line's own checks are ORed, not branched on)
  while (q < len) {
    // line starts in pairs, one 4-byte store per two lines
    if (li < kFrLines && (li & 1u)) *reinterpret_cast<uint32_t *>(lstarts + li - 1) = prev | q << 16;
    prev = q;
    const uint64_t a8 = fr_win8(stage, at + q);
    const uint32_t a = (uint32_t)a8, b = a & 0xFFu;
    // qpack.c:3439-3495: prefix bits, name literal, value, dynamic
    const bool lit = (b & 0xE0u) == 0x20u;
    const bool has_value = !(b & 0x80u) && (b & 0xF0u) != 0x10u;
    const uint32_t k = (b & 0x80u) ? 6u : (b & 0x40u) ? 4u : (b & 0x20u) ? 3u : (b & 0x10u) ? 4u : 3u;
    const bool dyn = (b & 0x80u) ? !(b & 0x40u) : (b & 0x40u) ? !(b & 0x10u) : true;
    uint32_t used;
    const uint32_t x = fr_varint(a, k, used);  // index, or the name's length
    bad |= used == 0u || len - q < used;
    uint32_t p = q + used;
    const bool hn = lit && (b & 0x08u);
    bad |= lit && (x > QH_QPACK_MAX_NAMELEN || (hn && x * 8 / 5 > QH_QPACK_MAX_NAMELEN) || len - p < x);
    bad |= !lit && (dyn ? ric == 0 : x >= QH_QPACK_STATIC_ENTRIES);
    p = bad ? len : p + (lit ? x : 0u);
    // the value's first bytes (read whether or not the line has one; from
    // the line's own window when they lie in it)
    const uint32_t r = p - q;
    const uint32_t v = r + 4 <= 8 ? (uint32_t)(a8 >> (8 * r)) : (uint32_t)fr_win8(stage, at + p);
    uint32_t vu;
    const uint32_t vl = fr_varint(v, 7, vu);
    const bool hv = has_value && (v & 0x80u);
    bad |= has_value && (p >= len || vu == 0u || len - p < vu);
    const uint32_t p2 = p + vu;
    bad |= has_value && (vl > QH_QPACK_MAX_VALUELEN || (hv && vl * 8 / 5 > QH_QPACK_MAX_VALUELEN) || len - p2 < vl);
    if (bad) break;
    o.spans += (lit ? 1u : 0u) + (has_value ? 1u : 0u);
    o.huff += (hn ? 1u : 0u) + (hv ? 1u : 0u);
    slots += (hn ? fr_slot(x) : 0u) + (hv ? fr_slot(vl) : 0u);
    o.nlong += hv && vl >= QH_LONG_MIN ? 1u : 0u;
    ++li;
    q = has_value ? p2 + vl : p;
  }
  if (bad) return false;
  if (li < kFrLines && (li & 1u)) lstarts[li - 1] = (uint16_t)prev;
  o.lines = li;
  o.slots = slots;
  return true;
}

#endif /* QH_FRAME_FAST_H */
