"""nghttp3_amd -- MI355X-native QPACK Huffman engine (drop-in for nghttp3's
lib/nghttp3_qpack_huffman.c hot path).  See DESIGN.md / INTEGRATION.md."""
from ._lib import LIB_PATH, QhError, load  # noqa: F401
from .qpack_huffman import *  # noqa: F401,F403

__version__ = "0.1.0"
