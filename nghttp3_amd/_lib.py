"""ctypes binding of libqhuff.so (include/qhuff.h).

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``)
into ``nghttp3_amd/lib/libqhuff.so``.  There is no fallback: if the library
is missing, importing the batch API raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libqhuff.so")
# Development builds (e.g. the phase-timer library of `make stamps`) are
# selected with QHUFF_LIB; there is no fallback to anything else.
LIB_PATH = os.environ.get("QHUFF_LIB", LIB_PATH)

QH_OK = 0
QH_ERR_INVALID_ARGUMENT = -101
QH_ERR_QPACK_FATAL = -108
QH_ERR_FATAL = -900
QH_ERR_NOMEM = -901

QH_WHERE_HOST = 0
QH_WHERE_DEVICE = 1
QH_WHERE_DEVICE_DENSE = 2
QH_DECODER_WINDOWS = 0
QH_DECODER_WAVES = 1
QH_DECODER_SORTED = 2
QH_ENCODER_WINDOWS = 0
QH_ENCODER_WAVES = 1
QH_ENCODER_FUSED = 2
QH_ENCODER_AUTO = 3
QH_ENCODER_REGION = 4
QH_OPT_LONG_MIN = 1
QH_OPT_LENS_LANE_PASS = 2

NGHTTP3_QPACK_HUFFMAN_FLAG_ACCEPTED = 0x01
NGHTTP3_QPACK_HUFFMAN_FLAG_SYM = 0x02


class QhError(RuntimeError):
    def __init__(self, code, what=""):
        super().__init__(f"{what} failed with {code}")
        self.code = code


class qh_span_in(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class qh_span_out(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("len", ctypes.c_uint32), ("status", ctypes.c_int32)]


class qh_batch_stats(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("in_bytes", ctypes.c_uint64),
        ("out_bytes", ctypes.c_uint64),
        ("dst_bytes", ctypes.c_uint64),
        ("n_errors", ctypes.c_uint64),
        ("lane_steps", ctypes.c_uint64),
        ("wave_steps", ctypes.c_uint64),
    ]


class nghttp3_qpack_huffman_decode_context(ctypes.Structure):
    """lib/nghttp3_qpack_huffman.h:70-74"""

    _fields_ = [("fstate", ctypes.c_uint16), ("flags", ctypes.c_uint8)]


class nghttp3_qpack_huffman_sym(ctypes.Structure):
    """lib/nghttp3_qpack_huffman.h:35-40"""

    _fields_ = [("nbits", ctypes.c_uint32), ("code", ctypes.c_uint32)]


class nghttp3_qpack_huffman_decode_node(ctypes.Structure):
    """lib/nghttp3_qpack_huffman.h:56-68"""

    _fields_ = [("fstate", ctypes.c_uint16), ("flags", ctypes.c_uint8), ("sym", ctypes.c_uint8)]


# Every symbol include/qhuff.h declares (checked by tests/test_abi.py).
EXPORTED_FUNCTIONS = (
    "nghttp3_qpack_huffman_encode_count",
    "nghttp3_qpack_huffman_encode",
    "nghttp3_qpack_huffman_decode_context_init",
    "nghttp3_qpack_huffman_decode",
    "nghttp3_qpack_huffman_decode_failure_state",
    "qh_ctx_new",
    "qh_ctx_del",
    "qh_ctx_set_stream",
    "qh_ctx_set_decoder",
    "qh_ctx_set_encoder",
    "qh_ctx_set_option",
    "qh_ctx_stream",
    "qh_ctx_sync",
    "qh_ctx_last_stats",
    "qh_decode_dst_size",
    "qh_encode_dst_bound",
    "qh_decode_batch",
    "qh_decode_batch_multi",
    "qh_encode_count_batch",
    "qh_encode_batch",
    # QPACK field-line framing (csrc/qh_qpack.c, bound in qpack.py)
    "qh_qpack_scan_field_section",
    "qh_qpack_scan_blocks",
    "qh_scan_blocks_batch",
    "qh_decode_sections_batch",
    "qh_encode_sections_batch",
    "qh_qpack_static_entry",
    "qh_qpack_plan_fields",
    "qh_qpack_scan_encoder_stream",
    "qh_qpack_put_varint_len",
    "qh_qpack_put_varint",
    "qh_qpack_write_indexed",
    "qh_qpack_write_indexed_name",
    "qh_qpack_write_literal",
    "qh_qpack_literal_bound",
    "qh_qpack_write_sections",
    # field validation (csrc/qh_http.c, csrc/qh_validate.inc)
    "nghttp3_check_header_name",
    "nghttp3_check_header_value",
    "qh_check_fields_batch",
    # header-name tokens (csrc/qh_http.c, csrc/qh_validate.inc)
    "qh_qpack_lookup_token",
    "qh_lookup_tokens_batch",
    "qh_ctx_enable_timing",
    "qh_ctx_kernel_times",
    "qh_synth_spans",
    "qh_synth_fill",
    "qh_version",
)
EXPORTED_DATA = ("huffman_sym_table", "qpack_huffman_decode_table")

_lib = None


def load():
    """Load libqhuff.so once; raise if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make` or "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch's copy when PyTorch is present
    # (libqhuff's libamdhip64.so.7 then binds to the one torch loaded).
    # Loading the system runtime first and torch's after leaves two HSA
    # runtimes in the process, and the device is then invisible to one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    c = ctypes
    vp, sz, u64, u32, i32 = c.c_void_p, c.c_size_t, c.c_uint64, c.c_uint32, c.c_int

    lib.nghttp3_qpack_huffman_encode_count.argtypes = [vp, sz]
    lib.nghttp3_qpack_huffman_encode_count.restype = sz
    lib.nghttp3_qpack_huffman_encode.argtypes = [vp, vp, sz]
    lib.nghttp3_qpack_huffman_encode.restype = vp
    lib.nghttp3_qpack_huffman_decode_context_init.argtypes = [c.POINTER(nghttp3_qpack_huffman_decode_context)]
    lib.nghttp3_qpack_huffman_decode_context_init.restype = None
    lib.nghttp3_qpack_huffman_decode.argtypes = [
        c.POINTER(nghttp3_qpack_huffman_decode_context), vp, vp, sz, i32]
    lib.nghttp3_qpack_huffman_decode.restype = c.c_ssize_t
    lib.nghttp3_qpack_huffman_decode_failure_state.argtypes = [c.POINTER(nghttp3_qpack_huffman_decode_context)]
    lib.nghttp3_qpack_huffman_decode_failure_state.restype = i32

    lib.qh_ctx_new.argtypes = [c.POINTER(vp), i32, vp]
    lib.qh_ctx_new.restype = i32
    lib.qh_ctx_del.argtypes = [vp]
    lib.qh_ctx_del.restype = None
    lib.qh_ctx_set_decoder.argtypes = [vp, i32]
    lib.qh_ctx_set_decoder.restype = i32
    lib.qh_ctx_set_encoder.argtypes = [vp, i32]
    lib.qh_ctx_set_encoder.restype = i32
    lib.qh_ctx_set_option.argtypes = [vp, i32, ctypes.c_int64]
    lib.qh_ctx_set_option.restype = i32
    lib.qh_ctx_set_stream.argtypes = [vp, vp]
    lib.qh_ctx_set_stream.restype = i32
    lib.qh_ctx_stream.argtypes = [vp]
    lib.qh_ctx_stream.restype = vp
    lib.qh_ctx_sync.argtypes = [vp]
    lib.qh_ctx_sync.restype = i32
    lib.qh_ctx_last_stats.argtypes = [vp, c.POINTER(qh_batch_stats)]
    lib.qh_ctx_last_stats.restype = i32
    lib.qh_decode_dst_size.argtypes = [vp, sz]
    lib.qh_decode_dst_size.restype = u64
    lib.qh_encode_dst_bound.argtypes = [vp, sz]
    lib.qh_encode_dst_bound.restype = u64
    lib.qh_decode_batch.argtypes = [vp, vp, vp, sz, vp, u64, vp, i32]
    lib.qh_decode_batch.restype = i32
    lib.qh_decode_batch_multi.argtypes = [vp, i32, vp, vp, sz, vp, u64, vp]
    lib.qh_decode_batch_multi.restype = i32
    lib.qh_encode_count_batch.argtypes = [vp, vp, vp, sz, vp, i32]
    lib.qh_encode_count_batch.restype = i32
    lib.qh_encode_batch.argtypes = [vp, vp, vp, sz, vp, u64, vp, i32]
    lib.qh_encode_batch.restype = i32
    lib.qh_ctx_enable_timing.argtypes = [vp, i32]
    lib.qh_ctx_enable_timing.restype = i32
    lib.qh_ctx_kernel_times.argtypes = [vp, c.POINTER(c.c_char_p), c.POINTER(u64), c.POINTER(c.c_double), i32]
    lib.qh_ctx_kernel_times.restype = i32
    lib.qh_synth_spans.argtypes = [vp, u64, sz, u32, u32, i32, c.c_double, vp, vp]
    lib.qh_synth_spans.restype = i32
    lib.qh_synth_fill.argtypes = [vp, u64, u64, vp, u64, vp, u32]
    lib.qh_synth_fill.restype = i32
    lib.qh_version.argtypes = []
    lib.qh_version.restype = c.c_char_p
    _lib = lib
    return lib


def check(rv, what):
    if rv < 0:
        raise QhError(rv, what)
    return rv
