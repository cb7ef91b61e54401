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
