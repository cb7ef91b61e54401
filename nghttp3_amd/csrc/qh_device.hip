// qh_device.hip -- QPACK Huffman batch engine for MI355X (gfx950, CDNA4).
//
// Replaces the hot loops of nghttp3's lib/nghttp3_qpack_huffman.c
// (encode_count :34-43, encode :45-78, decode :87-124) for batches of whole
// header-field strings.  Integer/byte work only: no MFMA.  Design notes and
// the roofline accounting are in DESIGN.md.
//
// Kernels (all launched on the context's stream):
//   qh_k_dec_reserve   per block: output slot bytes of its strings
//   qh_k_dec_lanes     decode, one string per lane, 4-bit FSM in LDS
//                      (huffman.c:103-114)
//   qh_k_dec_lut       decode, one string per lane, 12-bit multi-symbol table
//                      (opt-in: QHUFF_DECODER=lut)
//   qh_k_enc_lens      encoded length per string (huffman.c:34-43), chunk
//                      engine, + per-block totals
//   qh_k_enc_lanes     codes, one string per lane, dense output through an
//                      LDS stage (huffman.c:45-78)
//   qh_k_scan, qh_k_synth_*   synthetic inputs (bench/tests only)

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
#include "qh_common.h"      // span/stat types, tables, small helpers
#include "qh_chunk.inc"      // block ranges, windows, chunk rounds, scans
#include "qh_scan.inc"       // batch prefix sum (synthetic inputs)
#include "qh_lane_dec.inc"   // decoder: 4-bit FSM, one string per lane
#include "qh_lane_dec2.inc"  // decoder: 4-bit FSM, two strings per lane
#include "qh_lut_dec.inc"    // decoder: 12-bit table, one string per lane
#include "qh_peek_dec.inc"   // decoder: W-bit peek table, lock-step lanes
#include "qh_dec3.inc"       // decoder (default): plan + task-queue lanes
#include "qh_lane_enc.inc"   // encoder: lengths (stream, lanes, chunks), codes (lanes)
#include "qh_enc_stream.inc" // encoder (default codes): streaming region rounds
#include "qh_synth.inc"      // synthetic inputs for bench/tests
#include "qh_api.inc"    // host API (include/qhuff.h)
#include "qh_validate.inc"  // field name / value validation batch, header-name tokens
#include "qh_frame.inc"     // QPACK field-section framing on the device
#include "qh_sections.inc"  // whole field sections: frame -> decode -> fold / check / tokens

