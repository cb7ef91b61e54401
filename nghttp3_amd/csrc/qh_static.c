/*
 * The QPACK static table and the encoder's choice of representation for a
 * field when the dynamic table is not used (capacity 0) -- the encoder call
 * sites of SURVEY.md section 8(a) rows a9 / a10, host C.
 *
 * Reference behaviour restated here (lib/nghttp3_qpack.c):
 *   - the 99 entries of RFC 9204 Appendix A (stable[], :189-291);
 *   - nghttp3_qpack_encoder_encode_nv :1455-1628 at capacity 0: the name's
 *     token (qpack_lookup_token :342; a static name iff token < 99, :1477),
 *     qpack_encoder_decide_indexing_mode :1307-1371 (only its NEVER outcomes
 *     matter at capacity 0: the NEVER_INDEX flag, authorization, a cookie
 *     value shorter than 20 bytes), nghttp3_qpack_lookup_stable :1630-1660
 *     (an entry with the same name and value -> Indexed Field Line; else the
 *     first entry of the name -> Literal With Name Reference; NEVER mode
 *     skips the value match), otherwise Literal With Literal Name
 *     (:1627).  The N bit comes from the field's NEVER_INDEX flag only
 *     (:1898-1910, :2008-2017), not from the indexing mode.
 * The lookup walks the entries of the name in index order, which is the
 * order of token_stable[] (:52-169; pinned in tests/test_qif.py against
 * tests/golden/static_table.json).
 */
#include <pthread.h>
#include <string.h>

#include "../../include/qhuff.h"

#define QH_NSTATIC 99

static const char *const kStaticName[QH_NSTATIC] = {
  ":authority", ":path", "age", "content-disposition", "content-length",
  "cookie", "date", "etag", "if-modified-since", "if-none-match",
  "last-modified", "link", "location", "referer", "set-cookie",
  ":method", ":method", ":method", ":method", ":method", ":method", ":method",
  ":scheme", ":scheme",
  ":status", ":status", ":status", ":status", ":status",
  "accept", "accept", "accept-encoding", "accept-ranges",
  "access-control-allow-headers", "access-control-allow-headers",
  "access-control-allow-origin",
  "cache-control", "cache-control", "cache-control", "cache-control",
  "cache-control", "cache-control",
  "content-encoding", "content-encoding",
  "content-type", "content-type", "content-type", "content-type",
  "content-type", "content-type", "content-type", "content-type",
  "content-type", "content-type", "content-type",
  "range",
  "strict-transport-security", "strict-transport-security",
  "strict-transport-security",
  "vary", "vary", "x-content-type-options", "x-xss-protection",
  ":status", ":status", ":status", ":status", ":status", ":status",
  ":status", ":status", ":status",
  "accept-language",
  "access-control-allow-credentials", "access-control-allow-credentials",
  "access-control-allow-headers",
  "access-control-allow-methods", "access-control-allow-methods",
  "access-control-allow-methods",
  "access-control-expose-headers", "access-control-request-headers",
  "access-control-request-method", "access-control-request-method",
  "alt-svc", "authorization", "content-security-policy", "early-data",
  "expect-ct", "forwarded", "if-range", "origin", "purpose", "server",
  "timing-allow-origin", "upgrade-insecure-requests", "user-agent",
  "x-forwarded-for", "x-frame-options", "x-frame-options"};

static const char *const kStaticValue[QH_NSTATIC] = {
  "", "/", "0", "", "0", "", "", "", "", "", "", "", "", "", "",
  "CONNECT", "DELETE", "GET", "HEAD", "OPTIONS", "POST", "PUT",
  "http", "https",
  "103", "200", "304", "404", "503",
  "*/*", "application/dns-message", "gzip, deflate, br", "bytes",
  "cache-control", "content-type", "*",
  "max-age=0", "max-age=2592000", "max-age=604800", "no-cache", "no-store",
  "public, max-age=31536000",
  "br", "gzip",
  "application/dns-message", "application/javascript", "application/json",
  "application/x-www-form-urlencoded", "image/gif", "image/jpeg",
  "image/png", "text/css", "text/html; charset=utf-8", "text/plain",
  "text/plain;charset=utf-8",
  "bytes=0-",
  "max-age=31536000", "max-age=31536000; includesubdomains",
  "max-age=31536000; includesubdomains; preload",
  "accept-encoding", "origin", "nosniff", "1; mode=block",
  "100", "204", "206", "302", "400", "403", "421", "425", "500",
  "",
  "FALSE", "TRUE",
  "*",
  "get", "get, post, options", "options",
  "content-length", "content-type",
  "get", "post",
  "clear", "", "script-src 'none'; object-src 'none'; base-uri 'none'", "1",
  "", "", "", "", "prefetch", "", "*", "1", "", "", "deny", "sameorigin"};

/* Per entry: its name's token, and the next entry of the same name (or -1);
 * per token < 99: the name's first entry (or -1). */
static int32_t g_tok[QH_NSTATIC], g_next[QH_NSTATIC], g_first[QH_NSTATIC];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void static_init(void) {
  int i, j;
  for (i = 0; i < QH_NSTATIC; ++i) {
    g_first[i] = -1;
    g_next[i] = -1;
  }
  for (i = 0; i < QH_NSTATIC; ++i) {
    g_tok[i] = qh_qpack_lookup_token((const uint8_t *)kStaticName[i],
                                     strlen(kStaticName[i]));
  }
  for (i = QH_NSTATIC - 1; i >= 0; --i) {
    int32_t t = g_tok[i];
    if (t < 0 || t >= QH_NSTATIC) {
      continue; /* cannot happen: every static name has a token < 99 */
    }
    for (j = i + 1; j < QH_NSTATIC && g_tok[j] != t; ++j)
      ;
    g_next[i] = j < QH_NSTATIC ? j : -1;
    g_first[t] = i;
  }
}

QH_EXPORT int qh_qpack_static_entry(size_t idx, const uint8_t **name,
                                    size_t *namelen, const uint8_t **value,
                                    size_t *valuelen) {
  if (idx >= QH_NSTATIC) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  if (name) {
    *name = (const uint8_t *)kStaticName[idx];
  }
  if (namelen) {
    *namelen = strlen(kStaticName[idx]);
  }
  if (value) {
    *value = (const uint8_t *)kStaticValue[idx];
  }
  if (valuelen) {
    *valuelen = strlen(kStaticValue[idx]);
  }
  return 0;
}

#define QH_TOKEN_AUTHORIZATION 45 /* nghttp3.h nghttp3_qpack_token */
#define QH_TOKEN_COOKIE 68

QH_EXPORT int qh_qpack_plan_fields(const uint8_t *plain, const qh_span_in *strs,
                                   size_t nfields, const uint8_t *never,
                                   qh_field_line *lines) {
  size_t i;
  if (nfields && (plain == NULL || strs == NULL || lines == NULL)) {
    return QH_ERR_INVALID_ARGUMENT;
  }
  pthread_once(&g_once, static_init);
  for (i = 0; i < nfields; ++i) {
    const qh_span_in *nm = &strs[2 * i], *v = &strs[2 * i + 1];
    const uint8_t *name = plain + nm->off, *value = plain + v->off;
    int nv_never = never && never[i];
    int32_t token = qh_qpack_lookup_token(name, nm->len);
    qh_field_line *l = &lines[i];
    memset(l, 0, sizeof(*l));
    l->flags = nv_never ? QH_FL_NEVER : 0;
    l->name = (int32_t)(2 * i);
    l->value = (int32_t)(2 * i + 1);
    if (token >= 0 && token < QH_NSTATIC && g_first[token] >= 0) {
      int mode_never = nv_never || token == QH_TOKEN_AUTHORIZATION ||
                       (token == QH_TOKEN_COOKIE && v->len < 20);
      int32_t e = g_first[token];
      if (!mode_never) {
        for (; e >= 0; e = g_next[e]) {
          size_t vl = strlen(kStaticValue[e]);
          if (vl == v->len && memcmp(kStaticValue[e], value, vl) == 0) {
            break;
          }
        }
        if (e >= 0) {
          l->opcode = QH_FL_INDEXED;
          l->index = (uint64_t)e;
          l->name = l->value = -1;
          continue;
        }
      }
      l->opcode = QH_FL_INDEXED_NAME;
      l->index = (uint64_t)g_first[token];
      l->name = -1;
      continue;
    }
    l->opcode = QH_FL_LITERAL;
  }
  return 0;
}
