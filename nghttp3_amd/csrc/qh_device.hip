// qh_device.hip -- QPACK Huffman batch engine for MI355X (gfx950, CDNA4).
//
// Replaces the hot loops of nghttp3's lib/nghttp3_qpack_huffman.c
// (encode_count :34-43, encode :45-78, decode :87-124) for batches of whole
// header-field strings.  Integer/byte work only: no MFMA.  Design notes and
// the roofline accounting are in DESIGN.md.
//
// Kernels (all launched on the context's stream):
//   qh_k_scan<SLOTS>     decoupled look-back exclusive scan over strings:
//                        decode slot offsets (sum of len*8/5, the reference's
//                        rcbuf sizing, huffman.h:113-115).
//   qh_k_decode          one lane per string; 4-bit FSM (huffman.c:103-114)
//                        with the 257x16 table in LDS; 16-B input fetches;
//                        dword-aligned output stores.
//   qh_k_count           hlen = encode_count per string (huffman.c:34-43).
//   qh_k_scan<HLEN>      dense encode offsets (prefix sum of hlen).
//   qh_k_encode          one lane per string; 64-bit accumulator with
//                        big-endian 32-bit flushes and EOS-prefix padding
//                        (huffman.c:53-75).
//   qh_k_synth_*         deterministic synthetic inputs (bench/tests only).

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/qhuff.h"
#include "qh_tables.h"

#define QH_VERSION "0.2.0"

// One translation unit, split by concern:
#include "qh_common.h"   // span/stat types, tables, LDS + scan helpers
#include "qh_lane.inc"   // lane-per-string kernels (general spans)
#include "qh_tile.inc"      // tile engine: plan, shared helpers
#include "qh_tile_enc.inc"  // tile encoder (count / scan / emit)
#include "qh_chunk.inc"     // chunk engine: block ranges, windows, rounds
#include "qh_chunk_dec.inc"  // chunk decoder (reserve / decode)
#include "qh_lane_dec.inc"   // lane-per-string decoder (4-bit FSM)
#include "qh_lut_dec.inc"    // lane-per-string decoder (12-bit table)
#include "qh_synth.inc"  // synthetic inputs for bench/tests
#include "qh_api.inc"    // host API (include/qhuff.h)

