/*
 * Field name / value validation, scalar
 * drop-ins for the public nghttp3_check_header_name / _value
 * (lib/includes/nghttp3/nghttp3.h:3443, :3452; lib/nghttp3_http.c:691-709,
 * :798-838, AVX2 body :771-796).  The batch form runs on the GPU
 * (qh_validate.inc, qh_check_fields_batch).
 *
 * Character classes (pinned against the reference tables by
 * tests/golden/http_chars.json):
 *   name  -- RFC 9110 tchar without upper case: DIGIT, a-z and
 *            !#$%&'*+-.^_`|~ (VALID_HD_NAME_CHARS == 1);
 *   value -- HTAB, SP..~ and 0x80..0xFF (VALID_HD_VALUE_CHARS), i.e. every
 *            byte but the controls other than HTAB and DEL; no leading or
 *            trailing SP / HTAB (is_ws, http.c:124-131).
 */
#include "../../include/qhuff.h"

static int name_char(uint8_t c) {
  if ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9')) {
    return 1;
  }
  switch (c) {
  case '!': case '#': case '$': case '%': case '&': case '\'': case '*':
  case '+': case '-': case '.': case '^': case '_': case '`': case '|':
  case '~':
    return 1;
  }
  return 0;
}

static int value_char(uint8_t c) { return c == 0x09 || (c >= 0x20 && c != 0x7f); }

static int is_ws(uint8_t c) { return c == ' ' || c == '\t'; }

QH_EXPORT int nghttp3_check_header_name(const uint8_t *name, size_t len) {
  size_t i = 0;
  if (len == 0) {
    return 0;
  }
  if (name[0] == ':') { /* pseudo header: the rest must be non-empty */
    if (len == 1) {
      return 0;
    }
    i = 1;
  }
  for (; i < len; ++i) {
    if (!name_char(name[i])) {
      return 0;
    }
  }
  return 1;
}

QH_EXPORT int nghttp3_check_header_value(const uint8_t *value, size_t len) {
  size_t i;
  if (len == 0) {
    return 1;
  }
  if (is_ws(value[0]) || is_ws(value[len - 1])) {
    return 0;
  }
  for (i = 0; i < len; ++i) {
    if (!value_char(value[i])) {
      return 0;
    }
  }
  return 1;
}
