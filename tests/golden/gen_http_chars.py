#!/usr/bin/env python3
"""Regenerate tests/golden/http_chars.json: the reference's field-name and
field-value character classes, VALID_HD_NAME_CHARS[256] and
VALID_HD_VALUE_CHARS[256] (lib/nghttp3_http.c:675-689 and :729-758), read
from the reference file as text in the build container.  Data only: the
256 class values of each table.  Also records the reference's is_ws set
(lib/nghttp3_http.c:124-131)."""
import json
import os
import re

REF = "/root/reference/lib/nghttp3_http.c"
HERE = os.path.dirname(os.path.abspath(__file__))


def table(txt, name):
    body = txt.split(f"static const int8_t {name}[256] = {{")[1].split("};")[0]
    t = [0] * 256
    for key, val in re.findall(r"\[\s*('(?:\\.|[^'])'|0x[0-9A-Fa-f]+)\s*\]\s*=\s*(-?\d+)", body):
        if key.startswith("0x"):
            c = int(key, 16)
        else:
            lit = key[1:-1]
            c = ord(lit.encode().decode("unicode_escape"))
        t[c] = int(val)
    return t


def main():
    txt = open(REF).read()
    out = {"source": "lib/nghttp3_http.c:675-758 (parsed as text)",
           "VALID_HD_NAME_CHARS": table(txt, "VALID_HD_NAME_CHARS"),
           "VALID_HD_VALUE_CHARS": table(txt, "VALID_HD_VALUE_CHARS"),
           "is_ws": [0x20, 0x09]}
    with open(os.path.join(HERE, "http_chars.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
