"""The C-ABI library loads and exports every symbol include/qhuff.h declares
(no compute calls: this runs without a GPU)."""
import os
import re
import subprocess

from conftest import ROOT


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "qhuff.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(ln for ln in text.splitlines() if not ln.lstrip().startswith("#"))
    names = set()
    for decl in re.findall(r"QH_EXPORT([^;{]*)", text):
        m = re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*(?:\(|\[)", decl)
        if m:
            names.add(m[0])
    return names


def test_header_declares_expected_entry_points():
    from nghttp3_amd import _lib
    assert declared_symbols() == set(_lib.EXPORTED_FUNCTIONS) | set(_lib.EXPORTED_DATA)


def test_library_exports_every_declared_symbol():
    from nghttp3_amd import _lib
    lib = _lib.load()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    for name in declared_symbols():
        assert name in exported, name
        assert hasattr(lib, name)


def test_library_has_gfx950_code_object():
    from nghttp3_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_oracle_is_not_linked_into_product():
    from nghttp3_amd import _lib
    out = subprocess.check_output(["nm", "-D", _lib.LIB_PATH], text=True)
    assert "qho_" not in out
    ldd = subprocess.check_output(["ldd", _lib.LIB_PATH], text=True)
    assert "qh_oracle" not in ldd


def test_static_archive_defines_every_declared_symbol():
    archive = os.path.join(ROOT, "nghttp3_amd", "lib", "libqhuff.a")
    assert os.path.exists(archive), "run make: libqhuff.a is the link-time drop-in (INTEGRATION.md section 1)"
    out = subprocess.check_output(["nm", "-g", "--defined-only", archive], text=True)
    defined = {ln.split()[-1] for ln in out.splitlines() if len(ln.split()) == 3}
    for name in declared_symbols():
        assert name in defined, name


_LINK_PROGRAM = r"""
#include <stdio.h>
#include <string.h>
#include "qhuff.h"
/* RFC 7541 C.4.1: "www.example.com" -> f1e3 c2e5 f23a 6ba0 ab90 f4ff */
static const uint8_t kat[] = {0xf1,0xe3,0xc2,0xe5,0xf2,0x3a,0x6b,0xa0,0xab,0x90,0xf4,0xff};
int main(void) {
  const char *s = "www.example.com";
  uint8_t enc[64], dec[64];
  size_t n = strlen(s);
  if (nghttp3_qpack_huffman_encode_count((const uint8_t *)s, n) != sizeof(kat)) return 1;
  uint8_t *end = nghttp3_qpack_huffman_encode(enc, (const uint8_t *)s, n);
  if ((size_t)(end - enc) != sizeof(kat) || memcmp(enc, kat, sizeof(kat))) return 2;
  nghttp3_qpack_huffman_decode_context ctx;
  nghttp3_qpack_huffman_decode_context_init(&ctx);
  nghttp3_ssize r = nghttp3_qpack_huffman_decode(&ctx, dec, kat, 5, 0);
  nghttp3_ssize r2 = nghttp3_qpack_huffman_decode(&ctx, dec + r, kat + 5, sizeof(kat) - 5, 1);
  if (r < 0 || r2 < 0 || (size_t)(r + r2) != n || memcmp(dec, s, n)) return 3;
  if (nghttp3_qpack_huffman_decode_failure_state(&ctx)) return 4;
  puts("ok");
  return 0;
}
"""


def test_c_program_links_static_archive_in_place_of_reference_objects(tmp_path):
    """What INTEGRATION.md section 1 tells a maintainer to do, done with the
    streaming (fin=0 then fin=1) decode the reference's qpack.c:2737-2763
    drives.  Runs only the host drop-ins: no GPU is touched."""
    archive = os.path.join(ROOT, "nghttp3_amd", "lib", "libqhuff.a")
    src = tmp_path / "link.c"
    src.write_text(_LINK_PROGRAM)
    exe = tmp_path / "link"
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-I", os.path.join(ROOT, "include"),
                           str(src), archive, "-L/opt/rocm/lib", "-lamdhip64", "-lstdc++",
                           "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)])
    assert subprocess.check_output([str(exe)], text=True).strip() == "ok"


def test_product_library_reads_no_development_knob():
    """The shipped libqhuff.so holds no development environment knob: the
    only QHUFF_* string is QHUFF_VERBOSE (a stderr report of the kernels'
    occupancy).  Tuning goes through qh_ctx_set_option; results never depend
    on the environment (the reference codec is pure,
    huffman.c:87-124)."""
    from nghttp3_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    found = set(m.decode() for m in re.findall(rb"QHUFF_[A-Z0-9_]+", data))
    assert found <= {"QHUFF_VERBOSE"}, found
