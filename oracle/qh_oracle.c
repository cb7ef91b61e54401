/*
 * qh_oracle.c -- TEST INFRASTRUCTURE ONLY (see qh_oracle.h for the rules and
 * for how this restatement is pinned to the reference).
 *
 * The tables are rebuilt here at load time from the RFC 7541 Appendix B code
 * lengths with a recursive trie walk (independent of the product's Python
 * generator), then the codec restates lib/nghttp3_qpack_huffman.c line by
 * line in behaviour:
 *   encode_count  huffman.c:34-43
 *   encode        huffman.c:45-78   (64-bit accumulator, BE 32-bit flush,
 *                                    EOS-prefix 1-bit padding)
 *   decode        huffman.c:87-124  (4-bit FSM, two lookups per byte,
 *                                    -108 when fin && !ACCEPTED)
 *   failure_state huffman.c:126-129
 */
#define _GNU_SOURCE
#include "qh_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* RFC 7541 Appendix B code lengths, symbols 0..255 then EOS. */
static const uint8_t kLen[257] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, 28, 28, 28,
    28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28, 6,  10, 10, 12, 13, 6,
    8,  11, 10, 10, 8,  11, 8,  6,  6,  6,  5,  5,  5,  6,  6,  6,  6,  6,  6,
    6,  7,  8,  15, 6,  12, 10, 13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,
    7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14,
    6,  15, 5,  6,  5,  6,  5,  6,  6,  6,  5,  7,  7,  6,  6,  6,  5,  6,  7,
    6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28, 20, 22, 20, 20, 22,
    22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, 24, 24, 22, 23, 24, 23, 23, 23,
    23, 21, 22, 23, 22, 23, 23, 24, 22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22,
    24, 21, 22, 23, 23, 21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22,
    22, 23, 26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, 19,
    21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, 20, 24, 20, 21,
    22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, 26, 27, 26, 26, 27, 27, 27,
    27, 27, 28, 27, 27, 27, 27, 27, 26, 30};

typedef struct {
  uint32_t nbits;
  uint32_t code; /* MSB-aligned */
} sym_t;

typedef struct {
  uint16_t fstate;
  uint8_t flags;
  uint8_t sym;
} node_t;

static sym_t g_sym[257];
static node_t g_fsm[257][16];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* trie: up to 2*257 nodes */
static int t_child[520][2];
static int t_leaf[520];
static int t_state[520];  /* pre-order internal id, -1 for leaves */
static int t_accept[520]; /* all-ones path of <= 7 bits */
static int t_n;

static int trie_new(void) {
  t_child[t_n][0] = t_child[t_n][1] = -1;
  t_leaf[t_n] = -1;
  t_state[t_n] = -1;
  t_accept[t_n] = 0;
  return t_n++;
}

static int g_next_state;

static void number_states(int node, int depth, int all_ones) {
  if (t_leaf[node] >= 0) return;
  t_state[node] = g_next_state++;
  t_accept[node] = all_ones && depth <= 7;
  number_states(t_child[node][0], depth + 1, 0);
  number_states(t_child[node][1], depth + 1, all_ones);
}

static void build_tables(void) {
  /* canonical code assignment: sort symbols by (length, symbol) */
  int order[257];
  int i, k, n = 0;
  for (k = 1; k <= 30; ++k)
    for (i = 0; i < 257; ++i)
      if (kLen[i] == k) order[n++] = i;
  uint32_t code = 0;
  for (i = 0; i < 257; ++i) {
    int s = order[i];
    if (i) code = (code + 1) << (kLen[s] - kLen[order[i - 1]]);
    g_sym[s].nbits = kLen[s];
    g_sym[s].code = code << (32 - kLen[s]);
  }
  /* trie */
  t_n = 0;
  int root = trie_new();
  for (i = 0; i < 257; ++i) {
    int node = root;
    for (k = (int)g_sym[i].nbits - 1; k >= 0; --k) {
      int b = (int)((g_sym[i].code >> (32 - g_sym[i].nbits + (uint32_t)k)) & 1u);
      if (t_child[node][b] < 0) {
        int c = trie_new();
        t_child[node][b] = c;
      }
      node = t_child[node][b];
    }
    t_leaf[node] = i;
  }
  g_next_state = 0;
  number_states(root, 0, 1);
  /* transitions */
  int node;
  for (node = 0; node < t_n; ++node) {
    if (t_state[node] < 0) continue;
    int st = t_state[node];
    int nib;
    for (nib = 0; nib < 16; ++nib) {
      int cur = node, sym = -1, fail = 0, on_leaf = 0;
      for (k = 3; k >= 0; --k) {
        cur = t_child[cur][(nib >> k) & 1];
        on_leaf = 0;
        if (t_leaf[cur] >= 0) {
          if (t_leaf[cur] == 256)
            fail = 1;
          else
            sym = t_leaf[cur];
          cur = root;
          on_leaf = 1;
        }
      }
      node_t e;
      if (fail) {
        e.fstate = 256;
        e.flags = 0;
        e.sym = 0;
      } else {
        e.fstate = (uint16_t)(on_leaf ? 0 : t_state[cur]);
        e.flags = (uint8_t)((sym >= 0 ? QHO_FLAG_SYM : 0) |
                            ((on_leaf || t_accept[cur]) ? QHO_FLAG_ACCEPTED : 0));
        e.sym = (uint8_t)(sym >= 0 ? sym : 0);
      }
      g_fsm[st][nib] = e;
    }
  }
  for (i = 0; i < 16; ++i) {
    g_fsm[256][i].fstate = 256;
    g_fsm[256][i].flags = 0;
    g_fsm[256][i].sym = 0;
  }
}

static void init_once(void) { pthread_once(&g_once, build_tables); }

void qho_tables(uint32_t sym[257][2], uint32_t fsm[257][16]) {
  int i, j;
  init_once();
  for (i = 0; i < 257; ++i) {
    sym[i][0] = g_sym[i].nbits;
    sym[i][1] = g_sym[i].code;
    for (j = 0; j < 16; ++j)
      fsm[i][j] = (uint32_t)g_fsm[i][j].fstate |
                  ((uint32_t)g_fsm[i][j].flags << 16) |
                  ((uint32_t)g_fsm[i][j].sym << 24);
  }
}

size_t qho_encode_count(const uint8_t *src, size_t len) {
  size_t i, nbits = 0;
  init_once();
  for (i = 0; i < len; ++i) nbits += g_sym[src[i]].nbits;
  return (nbits + 7) / 8;
}

uint8_t *qho_encode(uint8_t *dest, const uint8_t *src, size_t srclen) {
  const uint8_t *end = src + srclen;
  uint64_t code = 0;
  size_t nbits = 0;
  init_once();
  while (src != end) {
    const sym_t *s = &g_sym[*src++];
    code |= (uint64_t)s->code << (32 - nbits);
    nbits += s->nbits;
    if (nbits < 32) continue;
    uint32_t x = (uint32_t)(code >> 32);
    dest[0] = (uint8_t)(x >> 24);
    dest[1] = (uint8_t)(x >> 16);
    dest[2] = (uint8_t)(x >> 8);
    dest[3] = (uint8_t)x;
    dest += 4;
    code <<= 32;
    nbits -= 32;
  }
  for (; nbits >= 8; nbits -= 8) {
    *dest++ = (uint8_t)(code >> 56);
    code <<= 8;
  }
  if (nbits) {
    *dest++ = (uint8_t)((uint8_t)(code >> 56) | ((1u << (8 - nbits)) - 1));
  }
  return dest;
}

void qho_decode_context_init(qho_decode_ctx *ctx) {
  ctx->fstate = 0;
  ctx->flags = QHO_FLAG_ACCEPTED;
}

ptrdiff_t qho_decode(qho_decode_ctx *ctx, uint8_t *dest, const uint8_t *src,
                     size_t srclen, int fin) {
  uint8_t *p = dest;
  const uint8_t *end = src + srclen;
  node_t t;
  init_once();
  t.fstate = ctx->fstate;
  t.flags = ctx->flags;
  t.sym = 0;
  while (src != end) {
    uint8_t c = *src++;
    t = g_fsm[t.fstate][c >> 4];
    if (t.flags & QHO_FLAG_SYM) *p++ = t.sym;
    t = g_fsm[t.fstate][c & 0xFu];
    if (t.flags & QHO_FLAG_SYM) *p++ = t.sym;
  }
  ctx->fstate = t.fstate;
  ctx->flags = t.flags;
  if (fin && !(ctx->flags & QHO_FLAG_ACCEPTED)) return QHO_ERR_QPACK_FATAL;
  return p - dest;
}

int qho_decode_failure_state(const qho_decode_ctx *ctx) {
  return ctx->fstate == 0x100u;
}

uint64_t qho_encode_batch(const uint8_t *src, const uint64_t *off,
                          const uint32_t *len, size_t n, uint8_t *dst,
                          uint64_t *out_off, uint32_t *out_len) {
  uint64_t pos = 0;
  size_t i;
  for (i = 0; i < n; ++i) {
    size_t h = qho_encode_count(src + off[i], len[i]);
    uint8_t *e = qho_encode(dst + pos, src + off[i], len[i]);
    (void)e;
    out_off[i] = pos;
    out_len[i] = (uint32_t)h;
    pos += h;
  }
  return pos;
}

uint64_t qho_decode_batch(const uint8_t *src, const uint64_t *off,
                          const uint32_t *len, size_t n, uint8_t *dst,
                          uint64_t *slot_off, uint32_t *out_len,
                          int32_t *status) {
  uint64_t slot = 0, nerr = 0;
  size_t i;
  for (i = 0; i < n; ++i) {
    qho_decode_ctx ctx;
    qho_decode_context_init(&ctx);
    slot_off[i] = slot;
    ptrdiff_t r = qho_decode(&ctx, dst + slot, src + off[i], len[i], 1);
    if (r < 0 || qho_decode_failure_state(&ctx)) {
      out_len[i] = 0;
      status[i] = QHO_ERR_QPACK_FATAL;
      ++nerr;
    } else {
      out_len[i] = (uint32_t)r;
      status[i] = 0;
    }
    slot += ((uint64_t)len[i] * 8 / 5 + 15) & ~(uint64_t)15; /* qhuff.h slot */
  }
  return nerr;
}

/* ---- CPU baseline harness ----
 *
 * A pool of T threads is created once, each pinned to its own CPU (the list
 * the caller passes, else left where the scheduler puts it).  Every timed
 * pass starts from a barrier and ends at one; a thread runs its contiguous
 * shard `inner` times per pass, with `inner` calibrated so that a pass takes
 * at least `min_seconds` per thread (thread wake-up and scheduling noise are
 * then a small part of the pass).  Verification (decoded bytes == source)
 * runs after the timed passes, outside them. */

typedef struct {
  const uint8_t *src;
  const uint64_t *off;
  const uint32_t *len;
  size_t begin, end;
  uint8_t *enc;      /* encoded scratch for this shard */
  uint64_t *enc_off; /* per string */
  uint8_t *dec;      /* decoded scratch for this shard */
  int ok;
  int cpu;           /* CPU to pin to, -1 = none */
  uint64_t sink;     /* decoded lengths, so the decode cannot be elided */
  struct pool *pool;
} shard_t;

struct pool {
  pthread_barrier_t start, done;
  int cmd;   /* 0 encode, 1 decode, 2 verify, -1 exit */
  int inner;
};

static void shard_encode(shard_t *s) {
  uint64_t pos = 0;
  size_t i;
  for (i = s->begin; i < s->end; ++i) {
    size_t h = qho_encode_count(s->src + s->off[i], s->len[i]);
    s->enc_off[i - s->begin] = pos;
    qho_encode(s->enc + pos, s->src + s->off[i], s->len[i]);
    pos += h;
  }
  s->enc_off[s->end - s->begin] = pos;
}

static void shard_decode(shard_t *s, int verify) {
  size_t i;
  uint64_t sink = 0; /* (a local: shard_t's of adjacent threads share lines) */
  for (i = s->begin; i < s->end; ++i) {
    size_t k = i - s->begin;
    qho_decode_ctx ctx;
    qho_decode_context_init(&ctx);
    uint64_t a = s->enc_off[k], b = s->enc_off[k + 1];
    ptrdiff_t r = qho_decode(&ctx, s->dec, s->enc + a, (size_t)(b - a), 1);
    sink += (uint64_t)r;
    if (verify && (r != (ptrdiff_t)s->len[i] ||
                   memcmp(s->dec, s->src + s->off[i], s->len[i]) != 0))
      s->ok = 0;
  }
  s->sink += sink;
}

static void *shard_main(void *arg) {
  shard_t *s = (shard_t *)arg;
  struct pool *p = s->pool;
  int it;
  if (s->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(s->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  for (;;) {
    pthread_barrier_wait(&p->start);
    if (p->cmd < 0) break;
    if (p->cmd == 0)
      for (it = 0; it < p->inner; ++it) shard_encode(s);
    else if (p->cmd == 1)
      for (it = 0; it < p->inner; ++it) shard_decode(s, 0);
    else
      shard_decode(s, 1);
    pthread_barrier_wait(&p->done);
  }
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* one pass of every thread; seconds from the start barrier to the last
 * thread's end */
static double pool_pass(struct pool *p, int cmd, int inner) {
  p->cmd = cmd;
  p->inner = inner;
  double t0 = now_s();
  pthread_barrier_wait(&p->start);
  if (cmd >= 0) pthread_barrier_wait(&p->done); /* exit: threads leave */
  return now_s() - t0;
}

static int calib_inner(double one, double min_seconds) {
  double k = one > 0 ? min_seconds / one : 1.0;
  if (k < 1.0) return 1;
  if (k > 100000.0) return 100000;
  return (int)k + 1;
}

int qho_bench_roundtrip(const uint8_t *src, const uint64_t *off,
                        const uint32_t *len, size_t n, int nthreads,
                        const int *cpus, int reps, double min_seconds,
                        double *enc_seconds, double *dec_seconds,
                        int *inner_out) {
  shard_t *sh;
  pthread_t *tid;
  struct pool p;
  int t, r, ok = 1, ie, id;
  uint32_t maxlen = 0;
  size_t i;
  init_once();
  if (nthreads < 1) nthreads = 1;
  sh = (shard_t *)calloc((size_t)nthreads, sizeof(shard_t));
  tid = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (i = 0; i < n; ++i)
    if (len[i] > maxlen) maxlen = len[i];
  pthread_barrier_init(&p.start, NULL, (unsigned)nthreads + 1);
  pthread_barrier_init(&p.done, NULL, (unsigned)nthreads + 1);
  for (t = 0; t < nthreads; ++t) {
    size_t b = n * (size_t)t / (size_t)nthreads;
    size_t e = n * (size_t)(t + 1) / (size_t)nthreads;
    uint64_t bytes = 0;
    for (i = b; i < e; ++i) bytes += len[i];
    sh[t].src = src;
    sh[t].off = off;
    sh[t].len = len;
    sh[t].begin = b;
    sh[t].end = e;
    sh[t].enc = (uint8_t *)malloc((size_t)(bytes * 30 / 8 + 16));
    sh[t].enc_off = (uint64_t *)malloc((e - b + 1) * sizeof(uint64_t));
    sh[t].dec = (uint8_t *)malloc((size_t)maxlen * 30 / 8 * 8 / 5 + 16);
    sh[t].ok = 1;
    sh[t].cpu = cpus ? cpus[t] : -1;
    sh[t].pool = &p;
    pthread_create(&tid[t], NULL, shard_main, &sh[t]);
  }
  /* calibration passes (also the warm-up; the encode leaves the encoded
   * shards the decode passes read) */
  ie = calib_inner(pool_pass(&p, 0, 1), min_seconds);
  id = calib_inner(pool_pass(&p, 1, 1), min_seconds);
  for (r = 0; r < reps; ++r) {
    enc_seconds[r] = pool_pass(&p, 0, ie) / ie;
    dec_seconds[r] = pool_pass(&p, 1, id) / id;
  }
  pool_pass(&p, 2, 1); /* verification, untimed */
  pool_pass(&p, -1, 0);
  for (t = 0; t < nthreads; ++t) {
    pthread_join(tid[t], NULL);
    ok &= sh[t].ok;
    free(sh[t].enc);
    free(sh[t].enc_off);
    free(sh[t].dec);
  }
  pthread_barrier_destroy(&p.start);
  pthread_barrier_destroy(&p.done);
  free(sh);
  free(tid);
  if (inner_out) {
    inner_out[0] = ie;
    inner_out[1] = id;
  }
  return ok ? 0 : -1;
}
