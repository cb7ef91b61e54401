"""TEST INFRASTRUCTURE ONLY: restatement of nghttp3's field name / value
checks, driven by the reference's own character tables.

Only tests/ may import this module.  The tables are passed in from
tests/golden/http_chars.json (VALID_HD_NAME_CHARS / VALID_HD_VALUE_CHARS
parsed from lib/nghttp3_http.c:675-758 by tests/golden/gen_http_chars.py),
so the restatement is pinned to the reference's data, not to a retyped
character list.  Logic follows lib/nghttp3_http.c:691-709 (name; leading
':' of a pseudo header, which must not be alone) and :798-838 (value;
empty is valid, no leading/trailing SP or HTAB per is_ws :124-131; the AVX2
block scan :771-796 flags exactly the bytes the table rejects).
"""


def check_header_name(name: bytes, name_chars) -> int:
    if len(name) == 0:
        return 0
    if name[0] == ord(":"):
        if len(name) == 1:
            return 0
        name = name[1:]
    return int(all(name_chars[c] == 1 for c in name))


def check_header_value(value: bytes, value_chars) -> int:
    ws = (0x20, 0x09)
    if len(value) == 0:
        return 1
    if value[0] in ws or value[-1] in ws:
        return 0
    return int(all(value_chars[c] for c in value))


def lookup_token(name: bytes, tokens) -> int:
    """qpack_lookup_token (lib/nghttp3_qpack.c:342): exact, case-sensitive
    match of the whole name against the reference's token names
    (tests/golden/tokens.json, parsed from nghttp3.h's nghttp3_qpack_token),
    else -1."""
    try:
        return tokens.get(name.decode("latin-1"), -1)
    except Exception:
        return -1
