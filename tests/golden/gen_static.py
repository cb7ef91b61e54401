#!/usr/bin/env python3
"""Regenerate tests/golden/static_table.json: the reference's QPACK static
table, read as text from lib/nghttp3_qpack.c -- stable[] (:189-291, the 99
entries of RFC 9204 Appendix A: name, value, token) and token_stable[]
(:52-169, the entries in the order nghttp3_qpack_lookup_stable :1630-1660
walks them: sorted by token, entry `token` being the first entry of that
token).  Data only."""
import json
import os
import re

REF = "/root/reference/lib/nghttp3_qpack.c"
HERE = os.path.dirname(os.path.abspath(__file__))


def _c_string(s):
    return s.encode().decode("unicode_escape")


def main():
    txt = open(REF).read()
    body = txt.split("static nghttp3_qpack_static_header stable[] = {")[1].split("};")[0]
    stable = [{"name": _c_string(n), "value": _c_string(v), "token_name": t}
              for n, v, t in re.findall(
                  r'MAKE_STATIC_HD\(\s*"((?:[^"\\]|\\.)*)"\s*,\s*"((?:[^"\\]|\\.)*)"\s*,\s*(\w+)\s*\)',
                  body)]
    body = txt.split("static nghttp3_qpack_static_entry token_stable[] = {")[1].split("};")[0]
    order = [{"absidx": int(i), "token_name": t, "hash": int(h)}
             for i, t, h in re.findall(r"MAKE_STATIC_ENT\(\s*(\d+)\s*,\s*(\w+)\s*,\s*(\d+)U\s*\)", body)]
    with open(os.path.join(HERE, "static_table.json"), "w") as f:
        json.dump({"source": "lib/nghttp3_qpack.c stable[] and token_stable[] (parsed as text)",
                   "stable": stable, "token_stable": order}, f, indent=0)
    print(len(stable), "entries,", len(order), "token-ordered")


if __name__ == "__main__":
    main()
