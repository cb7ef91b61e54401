// The GPU framing count pass's parse (nghttp3_amd/csrc/qh_frame_fast.h)
// against scan_section (qh_qpack_core.h), block by block, compiled on the
// host.  Every block is placed in a stage buffer at an alignment from 0 to
// 15 with random bytes around it (the kernel's LDS stage holds the wave's
// other blocks there).  Prints: blocks, answered, mismatches, clean blocks
// not answered.  Usage: frame_fast_check SRC BLOCKS (SRC: bytes; BLOCKS:
// (u64 offset, u64 length) pairs).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qhuff.h"
#define QH_HD
#include "qh_qpack_core.h"
#include "qh_frame_fast.h"

static uint8_t *slurp(const char *path, long *size) {
  FILE *f = fopen(path, "rb");
  if (!f) return nullptr;
  fseek(f, 0, SEEK_END);
  *size = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *b = (uint8_t *)malloc(*size + 1);
  if (fread(b, 1, *size, f) != (size_t)*size) return nullptr;
  fclose(f);
  return b;
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  long sz = 0, bz = 0;
  uint8_t *src = slurp(argv[1], &sz);
  uint64_t *bl = (uint64_t *)slurp(argv[2], &bz);
  if (!src || !bl) return 2;
  const long n = bz / 16;
  long fast = 0, mism = 0, clean_fallback = 0;
  uint8_t *stage = (uint8_t *)aligned_alloc(16, 1 << 20);
  srand(7);
  for (long i = 0; i < n; ++i) {
    const uint64_t off = bl[2 * i];
    const uint32_t len = (uint32_t)bl[2 * i + 1];
    if (len + 64 > (1u << 20)) continue;
    const uint32_t at = rand() & 15;
    for (uint32_t k = 0; k < at; ++k) stage[k] = (uint8_t)rand();
    memcpy(stage + at, src + off, len);
    for (uint32_t k = 0; k < 32; ++k) stage[at + len + k] = (uint8_t)rand();
    FrCounts c;
    qh_section_prefix pf{}, pf2{};
    uint16_t ls[kFrLines], ls2[kFrLines];
    const bool ok = frame_count_fast(stage, at, len, QH_SECTIONS_DTABLE0, c, pf, ls);
    scan_out o = {};
    o.lines_cap = (size_t)-1;
    o.spans_cap = (size_t)-1;
    o.opts = QH_SECTIONS_DTABLE0;
    o.lstarts = ls2;
    o.lstarts_cap = kFrLines;
    const int rv = scan_section(&o, src + off, len, off, &pf2);
    if (ok) {
      ++fast;
      bool bad = rv != 0 || c.lines != o.nlines || c.spans != o.nspans || c.huff != o.nhuff ||
                 c.slots != o.hslots || c.nlong != o.nlong || pf.ricnt != pf2.ricnt ||
                 pf.delta_base != pf2.delta_base || pf.sign != pf2.sign;
      for (uint32_t k = 0; k < c.lines && k < kFrLines; ++k) bad |= ls[k] != ls2[k];
      mism += bad;
    } else if (rv == 0) {
      ++clean_fallback;
    }
  }
  printf("%ld %ld %ld %ld\n", n, fast, mism, clean_fallback);
  return 0;
}
