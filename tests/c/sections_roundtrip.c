/* A C caller of the whole-section batch entries (tests/test_gpu_qif.py):
 * reads a qpack-05 wire file (u64 stream id, u32 length, big endian), takes
 * its request-stream records (field sections), decodes them all with one
 * qh_decode_sections_batch call, then re-encodes every section from its
 * field lines, prefix and decoded strings with one qh_encode_sections_batch
 * call and compares the bytes with the input.  Prints "ok <sections>
 * <lines> <huffman strings>" or the first mismatch.  Both calls use host
 * memory (the library stages through the GPU). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qhuff.h"

static uint64_t be(const uint8_t *p, int n) {
  uint64_t v = 0;
  for (int k = 0; k < n; ++k) v = v << 8 | p[k];
  return v;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t *file = malloc((size_t)sz + 1);
  if (fread(file, 1, (size_t)sz, f) != (size_t)sz) return 2;
  fclose(f);
  qh_span_in *blocks = calloc((size_t)sz / 12 + 1, sizeof(*blocks));
  size_t nb = 0;
  for (long p = 0; p + 12 <= sz;) {
    uint64_t sid = be(file + p, 8);
    uint32_t len = (uint32_t)be(file + p + 8, 4);
    p += 12;
    if (sid != 0) {
      blocks[nb].off = (uint64_t)p;
      blocks[nb].len = len;
      blocks[nb].flags = 0;
      ++nb;
    }
    p += len;
  }
  qh_ctx *ctx;
  if (qh_ctx_new(&ctx, 0, NULL) != 0) return 3;
  size_t cap = (size_t)sz + 1;
  qh_sections s;
  memset(&s, 0, sizeof(s));
  s.lines = calloc(cap, sizeof(qh_field_line));
  s.lines_cap = cap;
  s.spans = calloc(cap, sizeof(qh_span_in));
  s.spans_cap = cap;
  s.strs = calloc(cap, sizeof(qh_span_out));
  s.line_start = calloc(nb + 1, 4);
  s.span_start = calloc(nb + 1, 4);
  s.status = calloc(nb + 1, 4);
  s.prefixes = calloc(nb + 1, sizeof(qh_section_prefix));
  s.dst_cap = 16 * cap;
  s.dst = malloc(s.dst_cap);
  int rv = qh_decode_sections_batch(ctx, file, blocks, nb, 0, &s, QH_WHERE_HOST);
  if (rv != 0) {
    printf("decode %d\n", rv);
    return 4;
  }
  for (size_t b = 0; b < nb; ++b) {
    if (s.status[b] != 0) {
      printf("block %zu status %d\n", b, s.status[b]);
      return 5;
    }
  }
  /* the decoded strings, packed: Huffman ones from dst, raw ones from the file */
  size_t ns = (size_t)s.nspans, total = 0;
  for (size_t k = 0; k < ns; ++k) total += s.strs[k].len;
  uint8_t *plain = malloc(total + 1);
  qh_span_in *strs = calloc(ns + 1, sizeof(qh_span_in));
  size_t o = 0;
  for (size_t k = 0; k < ns; ++k) {
    const uint8_t *from = (s.spans[k].flags & QH_SPAN_HUFFMAN) ? s.dst : file;
    if (s.strs[k].status != 0) return 6;
    memcpy(plain + o, from + s.strs[k].off, s.strs[k].len);
    strs[k].off = o;
    strs[k].len = s.strs[k].len;
    o += s.strs[k].len;
  }
  /* lines carry batch-global string indices already */
  uint8_t *out = malloc((size_t)sz + 64);
  qh_span_in *sections = calloc(nb + 1, sizeof(qh_span_in));
  uint64_t need = 0;
  rv = qh_encode_sections_batch(ctx, plain, strs, ns, s.lines, s.line_start, nb, s.prefixes, out,
                                (uint64_t)sz + 64, sections, &need, QH_WHERE_HOST);
  if (rv != 0) {
    printf("encode %d (need %llu)\n", rv, (unsigned long long)need);
    return 7;
  }
  for (size_t b = 0; b < nb; ++b) {
    if (sections[b].len != blocks[b].len ||
        memcmp(out + sections[b].off, file + blocks[b].off, blocks[b].len) != 0) {
      printf("section %zu differs (%u vs %u bytes)\n", b, sections[b].len, blocks[b].len);
      return 8;
    }
  }
  printf("ok %zu %llu %llu\n", nb, (unsigned long long)s.nlines, (unsigned long long)s.nhuff);
  qh_ctx_del(ctx);
  return 0;
}
