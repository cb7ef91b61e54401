// qh_device.hip -- QPACK Huffman batch engine for MI355X (gfx950, CDNA4).
//
// Replaces the hot loops of nghttp3's lib/nghttp3_qpack_huffman.c
// (encode_count :34-43, encode :45-78, decode :87-124) for batches of whole
// header-field strings.  Integer/byte work only: no MFMA.  Design notes and
// the roofline accounting are in DESIGN.md.
//
// Shipped kernels (all launched on the context's stream):
//   qh_k_dec_reserve + qh_k_dec_peek   decode, sorted 256-string windows, a
//                      W-bit table lookup per code (huffman.c:87-124)
//   qh_k_dec_reserve + qh_k_dec_peekw  decode, per-wave sorted chunks, input
//                      through LDS rings (QH_DECODER_WAVES)
//   qh_k_enc_lens_stream / _lane       encoded lengths (huffman.c:34-43)
//   qh_k_enc_lanes     codes, one string per lane, dense output through an
//                      LDS stage (huffman.c:45-78)
//   qh_k_frame_*, qh_k_sections_post, qh_k_check_fields,
//   qh_k_lookup_tokens QPACK framing, validation and tokens
//   qh_k_encsec_*      representation writer of whole field sections
//   qh_k_scan, qh_k_synth_*   prefix sums, synthetic inputs (bench/tests)
// Development variants (decoders fsm / fsm2 / lut / run / queue / other
// peek widths and shapes, the chunk-engine and streaming encoders) build
// only with -DQH_DEV_VARIANTS (make dev -> libqhuff_dev.so); the kernels
// that exist only for them live outside the package, in dev/csrc (-I).

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <condition_variable>
#include <atomic>
#include <thread>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/qhuff.h"
#include "qh_tables.h"

#define QH_VERSION "0.2.0"

// One translation unit, split by concern:
#include "qh_common.h"      // span/stat types, tables, small helpers
#include "qh_chunk.inc"      // block ranges, windows, chunk rounds, scans
#include "qh_scan.inc"       // batch prefix sum (synthetic inputs)
#include "qh_dec_common.inc"  // decode table blob, slot reservation
#include "qh_check.inc"       // field name / value checks (device)
#include "qh_sched.inc"       // batch-wide length-class schedule (QH_DECODER_SORTED)
#ifdef QH_DEV_VARIANTS         // development variants (make dev): not shipped
#include "qh_lane_dec.inc"   // (dev/csrc) decoder: 4-bit FSM, one string per lane
#include "qh_lane_dec2.inc"  // decoder: 4-bit FSM, two strings per lane
#include "qh_lut_dec.inc"    // decoder: 12-bit table, one string per lane
#endif
#include "qh_peek_dec.inc"   // decoders (windows: default; waves): W-bit peek table + leading-ones table
#ifdef QH_DEV_VARIANTS
#include "qh_pair_dec.inc"   // (dev/csrc) decoder: two codes per lookup, waves fed from a group queue
#endif
#ifdef QH_DEV_VARIANTS
#include "qh_dec3.inc"       // decoder: plan + task-queue lanes
#endif
#ifdef QH_DEV_VARIANTS
#include "qh_dec_q.inc"      // decoder: per-wave string queues
#endif
#include "qh_lane_enc.inc"   // encoder: lengths (stream, lanes), codes (lanes: the default)
#include "qh_enc_waves.inc"   // encoder codes (QH_ENCODER_WAVES): per-wave chunks, LDS rings
#include "qh_enc_fused.inc"   // encoder, lengths + codes in one pass (QH_ENCODER_FUSED)
#include "qh_enc_region.inc"  // encoder codes over each window's region (QH_ENCODER_REGION, opt-in)
#ifdef QH_DEV_VARIANTS
#include "qh_enc_seg.inc"    // (dev/csrc) encoder, one pass over equal-size segments per lane
#include "qh_enc_stream.inc" // encoder codes: streaming region rounds
#endif
#include "qh_synth.inc"      // synthetic inputs for bench/tests
#include "qh_host.inc"   // host-memory decode: dense packing kernels
#include "qh_api.inc"    // host API (include/qhuff.h)
#include "qh_validate.inc"  // field name / value validation batch, header-name tokens
#include "qh_frame.inc"     // QPACK field-section framing on the device
#include "qh_sections.inc"  // whole field sections: frame -> decode -> fold / check / tokens
#include "qh_enc_sections.inc"  // whole field sections out: count -> pick -> encode -> write

