// qpack -- the QIF bench driver (config 1; the driver half of config 4):
// the counterpart of the reference's examples/qpack.cc, qpack_encode.cc and
// qpack_decode.cc on the batch API of include/qhuff.h.
//
//   qpack [-s N] [-m N] [-a] [--scalar] [--time R] encode|decode IN OUT
//
// encode: QIF text (blocks of "name<TAB>value" lines, an empty line after
//   each; qpack_encode.cc:149-183) -> qpack-05 records (u64 stream id, u32
//   length, big endian; :88-107), one field section per block on stream
//   ids 1, 2, ... .  The whole file is one batch: qh_qpack_plan_fields picks
//   every field's representation (the encoder at dynamic table capacity 0:
//   only -s 0 is supported, so the encoder stream stays empty), then
//   qh_encode_sections_batch counts, Huffman-encodes and writes all
//   sections on the GPU.
// decode: records -> QIF (qpack_decode.cc:192-296).  The whole file is one
//   batch: every encoder-stream record and field section is framed on the
//   host (qh_qpack_scan_encoder_stream / qh_qpack_scan_field_section), every
//   Huffman string of the file is decoded by one qh_decode_batch call, then
//   the records are replayed in order against the dynamic table (the
//   decoder's table semantics, lib/nghttp3_qpack.c: set capacity
//   :2895-2910 / :3159-3185, rel2abs :3952-3969, inserts :3187-3306,
//   eviction :2071-2127, ricnt reconstruction :3915-3950, base :3419-3429,
//   blocking :3431-3436, brel2abs / pbrel2abs :3971-4017, validate_index
//   :2787-2798, emit :4020-4136) and written as QIF (write_header
//   :179-190), blocked sections released in Required-Insert-Count order
//   (qpack_decode.cc:154-174).
// --scalar runs the same batches through the library's scalar drop-ins
//   (nghttp3_qpack_huffman_*, qh_qpack_write_sections) instead of the GPU.
// --time R repeats the batch part R times and prints one JSON line of
//   timings to stderr.
#include <arpa/inet.h>
#include <getopt.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <iostream>
#include <iterator>
#include <queue>
#include <string>
#include <utility>
#include <vector>

#include "../../include/qhuff.h"


namespace {
// The text nghttp3_strerror gives these codes (lib/nghttp3_err.c:28-85),
// which the reference CLI prints after a failed call.
const char *qh_strerror(int rv) {
  switch (rv) {
  case QH_ERR_INVALID_ARGUMENT: return "ERR_INVALID_ARGUMENT";
  case QH_ERR_QPACK_FATAL: return "ERR_QPACK_FATAL";
  case QH_ERR_QPACK_HEADER_TOO_LARGE: return "ERR_QPACK_HEADER_TOO_LARGE";
  case QH_ERR_QPACK_DECOMPRESSION_FAILED: return "ERR_QPACK_DECOMPRESSION_FAILED";
  case QH_ERR_QPACK_ENCODER_STREAM_ERROR: return "ERR_QPACK_ENCODER_STREAM_ERROR";
  case QH_ERR_NOMEM: return "ERR_NOMEM";
  case QH_ERR_FATAL: return "ERR_FATAL";
  default: return "(unknown)";
  }
}
}  // namespace

namespace {

struct Config {
  size_t max_dtable = 0;
  size_t max_blocked = 0;
  bool immediate_ack = false;
  bool scalar = false;
  int time_reps = 0;
};
Config config;

constexpr size_t kMaxFields = 1024;  // qpack_encode.cc:142
constexpr size_t kEntryOverhead = 32;

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

double median(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

bool read_file(const char *path, std::vector<uint8_t> &out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) {
    std::cerr << "Could not open file " << path << ": " << strerror(errno) << std::endl;
    return false;
  }
  out.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  return true;
}

qh_ctx *g_ctx = nullptr;

qh_ctx *ctx() {
  if (!g_ctx) {
    int rv = qh_ctx_new(&g_ctx, 0, nullptr);
    if (rv != 0) {
      std::cerr << "qh_ctx_new: " << rv << " (no usable GPU; --scalar runs on the CPU)"
                << std::endl;
      exit(EXIT_FAILURE);
    }
  }
  return g_ctx;
}

void put_u64be(std::string &out, uint64_t v) {
  for (int k = 7; k >= 0; --k) out.push_back((char)(v >> (8 * k)));
}
void put_u32be(std::string &out, uint32_t v) {
  for (int k = 3; k >= 0; --k) out.push_back((char)(v >> (8 * k)));
}

// ---- encode --------------------------------------------------------------

int encode(const char *outfile, const char *infile) {
  if (config.max_dtable != 0) {
    std::cerr << "encode: only -s 0 (no dynamic table) is supported" << std::endl;
    return -1;
  }
  std::vector<uint8_t> text;
  if (!read_file(infile, text)) return -1;
  // blocks of fields: spans of the file (name, value) per field
  std::vector<qh_span_in> strs;
  std::vector<uint32_t> field_start{0};
  size_t pos = 0, srclen = 0;
  const size_t n = text.size();
  for (;;) {
    size_t nf = 0;
    while (pos < n) {
      size_t e = pos;
      while (e < n && text[e] != '\n') ++e;
      const size_t line_end = e;
      const size_t next = e < n ? e + 1 : e;
      if (line_end == pos) {  // empty line: end of the block
        pos = next;
        break;
      }
      if (nf == kMaxFields) {
        std::cerr << "Too many headers: " << nf << std::endl;
        return -1;
      }
      size_t d = pos;
      while (d < line_end && text[d] != '\t') ++d;
      if (d == line_end) {
        std::cerr << "Could not find TAB in "
                  << std::string((const char *)&text[pos], line_end - pos) << std::endl;
        return -1;
      }
      size_t v = d + 1;
      while (v < line_end && text[v] == ' ') ++v;
      strs.push_back({(uint64_t)pos, (uint32_t)(d - pos), 0});
      strs.push_back({(uint64_t)v, (uint32_t)(line_end - v), 0});
      srclen += (d - pos) + (line_end - v);
      ++nf;
      pos = next;
    }
    if (nf == 0) break;
    field_start.push_back((uint32_t)(strs.size() / 2));
  }
  const size_t nsec = field_start.size() - 1, nfields = strs.size() / 2;
  if (text.empty()) text.push_back(0);
  std::vector<qh_field_line> lines(nfields ? nfields : 1);
  std::vector<qh_span_in> sections(nsec ? nsec : 1);
  std::vector<uint8_t> dst;
  uint64_t need = 0;
  std::vector<double> t_plan, t_batch;
  const int reps = config.time_reps > 0 ? config.time_reps : 1;
  for (int r = 0; r < reps; ++r) {
    double t0 = now_ms();
    if (qh_qpack_plan_fields(text.data(), strs.data(), nfields, nullptr, lines.data()) != 0) {
      std::cerr << "qh_qpack_plan_fields failed" << std::endl;
      return -1;
    }
    double t1 = now_ms();
    int rv;
    if (config.scalar) {
      size_t cap = 16 + 20 * nsec + 20 * nfields + 2 * srclen;
      dst.resize(cap);
      rv = qh_qpack_write_sections(text.data(), strs.data(), lines.data(), field_start.data(),
                                   nsec, nullptr, dst.data(), cap, sections.data());
      need = nsec ? sections[nsec - 1].off + sections[nsec - 1].len : 0;
    } else {
      for (int k = 0; k < 2; ++k) {
        rv = qh_encode_sections_batch(ctx(), text.data(), strs.data(), strs.size(), lines.data(),
                                      field_start.data(), nsec, nullptr, dst.data(), dst.size(),
                                      sections.data(), &need, QH_WHERE_HOST);
        if (rv == QH_ERR_NOMEM && need > dst.size()) {
          dst.resize(need);
          continue;
        }
        break;
      }
    }
    if (rv != 0) {
      std::cerr << "encode: " << qh_strerror(rv) << std::endl;
      return -1;
    }
    double t2 = now_ms();
    t_plan.push_back(t1 - t0);
    t_batch.push_back(t2 - t1);
  }
  std::string out;
  out.reserve(need + 12 * nsec);
  for (size_t b = 0; b < nsec; ++b) {
    put_u64be(out, (uint64_t)(b + 1));
    put_u32be(out, sections[b].len);
    out.append((const char *)dst.data() + sections[b].off, sections[b].len);
  }
  std::ofstream of(outfile, std::ios::trunc | std::ios::binary);
  if (!of) {
    std::cerr << "Could not open file " << outfile << ": " << strerror(errno) << std::endl;
    return -1;
  }
  of.write(out.data(), (std::streamsize)out.size());
  if (srclen == 0) {
    std::cerr << "No header field processed" << std::endl;
  } else {
    char buf[160];
    snprintf(buf, sizeof(buf), "%zu -> %llu (r:%llu + e:0) %.2f%% compressed", srclen,
             (unsigned long long)need, (unsigned long long)need,
             (1. - (double)need / (double)srclen) * 100);
    std::cerr << buf << std::endl;
  }
  if (config.time_reps > 0) {
    fprintf(stderr,
            "{\"cmd\": \"encode\", \"path\": \"%s\", \"sections\": %zu, \"fields\": %zu, "
            "\"field_bytes\": %zu, \"out_bytes\": %llu, \"reps\": %d, \"plan_ms\": %.4f, "
            "\"batch_ms\": %.4f}\n",
            config.scalar ? "scalar" : "gpu", nsec, nfields, srclen, (unsigned long long)need,
            reps, median(t_plan), median(t_batch));
  }
  return 0;
}

// ---- decode --------------------------------------------------------------

struct Record {
  uint64_t stream_id;
  size_t off, len;
  int rv = 0;                     // framing verdict
  bool partial_bad = false;       // (stream 0) its cut last instruction's Huffman bytes fail
  size_t line0 = 0, nline = 0;    // its lines in `lines`
  size_t span0 = 0, nspan = 0;    // its strings in `spans`
  qh_section_prefix prefix{};
};

struct Entry {
  std::string name, value;
};

struct Blocked {
  uint64_t ricnt, seq, base;
  size_t rec;
  bool operator>(const Blocked &o) const {
    return ricnt != o.ricnt ? ricnt > o.ricnt : seq > o.seq;
  }
};

class Table {
 public:
  explicit Table(size_t hard_max) : hard_max_(hard_max), cap_(hard_max) {}
  uint64_t icnt() const { return next_; }
  bool set_cap(uint64_t cap) {
    if (cap > hard_max_) return false;
    cap_ = (size_t)cap;
    evict(0);
    return true;
  }
  bool add(const std::string &n, const std::string &v) {
    const size_t space = n.size() + v.size() + kEntryOverhead;
    if (space > cap_) return false;
    evict(space);
    ents_.push_front({n, v});
    size_ += space;
    ++next_;
    return true;
  }
  bool valid(uint64_t absidx) const {
    return absidx < next_ && next_ - absidx - 1 < ents_.size();
  }
  const Entry &get(uint64_t absidx) const { return ents_[(size_t)(next_ - absidx - 1)]; }
  // reconstruct_ricnt; false = DECOMPRESSION_FAILED
  bool ricnt(uint64_t enc, uint64_t &out) const {
    if (enc == 0) {
      out = 0;
      return true;
    }
    const uint64_t max_ents = hard_max_ / kEntryOverhead, full = 2 * max_ents;
    if (enc > full) return false;
    const uint64_t mx = next_ + max_ents;
    uint64_t r = mx / full * full + enc - 1;
    if (r > mx) {
      if (r <= full) return false;
      r -= full;
    }
    if (r == 0) return false;
    out = r;
    return true;
  }

 private:
  void evict(size_t space) {
    while (size_ + space > cap_ && !ents_.empty()) {
      size_ -= ents_.back().name.size() + ents_.back().value.size() + kEntryOverhead;
      ents_.pop_back();
    }
  }
  std::deque<Entry> ents_;
  size_t hard_max_, cap_, size_ = 0;
  uint64_t next_ = 0;
};

struct Decoded {
  const std::vector<uint8_t> *file;
  const std::vector<qh_span_in> *spans;
  const std::vector<qh_span_out> *hout;  // per span: decoded (Huffman) or unused
  const std::vector<uint8_t> *dst;
  std::string str(size_t k) const {
    const qh_span_in &s = (*spans)[k];
    if (s.flags & QH_SPAN_HUFFMAN) {
      const qh_span_out &o = (*hout)[k];
      return std::string((const char *)dst->data() + o.off, o.len);
    }
    return std::string((const char *)file->data() + s.off, s.len);
  }
};

void write_header(std::string &out, const std::vector<std::pair<std::string, std::string>> &h) {
  for (auto &nv : h) {
    out += nv.first;
    out += '\t';
    out += nv.second;
    out += '\n';
  }
  out += '\n';
}

// Emit one field section against the table (false: DECOMPRESSION_FAILED).
bool emit(const Table &t, const Record &r, uint64_t ricnt, uint64_t base,
          const std::vector<qh_field_line> &lines, const Decoded &d, std::string &out) {
  std::vector<std::pair<std::string, std::string>> h;
  for (size_t i = r.line0; i < r.line0 + r.nline; ++i) {
    const qh_field_line &l = lines[i];
    const bool dyn = (l.flags & QH_FL_DYNAMIC) != 0;
    std::string name, value;
    Entry ent;
    switch (l.opcode) {
      case QH_FL_INDEXED:
      case QH_FL_INDEXED_NAME:
        if (dyn) {
          if (base < l.index + 1) return false;
          const uint64_t a = base - l.index - 1;
          if (a >= ricnt || !t.valid(a)) return false;
          ent = t.get(a);
        } else {
          const uint8_t *n, *v;
          size_t nl, vl;
          if (qh_qpack_static_entry((size_t)l.index, &n, &nl, &v, &vl) != 0) return false;
          ent = {std::string((const char *)n, nl), std::string((const char *)v, vl)};
        }
        break;
      case QH_FL_INDEXED_PB:
      case QH_FL_INDEXED_NAME_PB: {
        const uint64_t a = l.index + base;
        if (a >= ricnt || !t.valid(a)) return false;
        ent = t.get(a);
        break;
      }
      default:
        break;
    }
    switch (l.opcode) {
      case QH_FL_INDEXED:
      case QH_FL_INDEXED_PB:
        h.emplace_back(ent.name, ent.value);
        break;
      case QH_FL_INDEXED_NAME:
      case QH_FL_INDEXED_NAME_PB:
        h.emplace_back(ent.name, d.str((size_t)l.value));
        break;
      default:
        h.emplace_back(d.str((size_t)l.name), d.str((size_t)l.value));
    }
  }
  write_header(out, h);
  return true;
}

// The bytes of an encoder instruction cut by the end of its record.  The
// reference reads them as they arrive (qpack.c:2815-3150): every Huffman
// string of the instruction that has begun is decoded over the bytes
// present (qpack_read_huffman_string, :2737-2763: fin = 1 once the whole
// string is there), and a failure there fails the record with
// ENCODER_STREAM_ERROR (:2992-2997, :3083-3088).  True if that happens.
bool partial_huffman_fails(const uint8_t *p, size_t n) {
  size_t pos = 0;
  bool bad = false;
  // prefixed integer: 1 complete, 0 cut (overflow is the scanner's verdict)
  auto varint = [&](int prefix, uint64_t &v) -> int {
    if (pos >= n) return 0;
    const uint64_t k = (1u << prefix) - 1;
    v = p[pos++] & k;
    if (v != k) return 1;
    for (int shift = 0; pos < n && shift <= 62; shift += 7) {
      const uint8_t b = p[pos++];
      v += (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return 1;
    }
    return 0;
  };
  // one string: 1 complete, 0 cut
  auto string = [&](int prefix) -> int {
    if (pos >= n) return 0;
    const bool h = (p[pos] >> prefix) & 1;
    uint64_t len = 0;
    if (varint(prefix, len) != 1) return 0;
    const size_t have = (size_t)std::min<uint64_t>(len, n - pos);
    if (h && have) {
      std::vector<uint8_t> out(nghttp3_qpack_huffman_estimate_decode_length(have) + 1);
      nghttp3_qpack_huffman_decode_context c;
      nghttp3_qpack_huffman_decode_context_init(&c);
      const nghttp3_ssize w = nghttp3_qpack_huffman_decode(&c, out.data(), p + pos, have, have == len);
      if (w < 0 || nghttp3_qpack_huffman_decode_failure_state(&c)) bad = true;
    }
    pos += have;
    return have == len ? 1 : 0;
  };
  if (n == 0) return false;
  const uint8_t b = p[0];
  uint64_t idx = 0;
  if (b & 0x80) {  // insert with name reference: index, value
    if (varint(6, idx) == 1) string(7);
  } else if (b & 0x40) {  // insert with literal name: name, value
    if (string(5) == 1 && !bad) string(7);
  }
  return bad;
}

int decode(const char *outfile, const char *infile) {
  std::vector<uint8_t> file;
  if (!read_file(infile, file)) return -1;
  const size_t n = file.size();
  // records; a framing error ends the list, and is reported after the
  // records before it were replayed and their output written, as the
  // reference CLI reads the file record by record (qpack_decode.cc:229-247)
  std::vector<Record> recs;
  std::string frame_err;
  for (size_t p = 0; p != n;) {
    if (n - p < 12) {
      frame_err = "Could not read stream ID and size";
      break;
    }
    uint64_t sid = 0;
    for (int k = 0; k < 8; ++k) sid = sid << 8 | file[p + k];
    uint32_t size = 0;
    for (int k = 0; k < 4; ++k) size = size << 8 | file[p + 8 + k];
    p += 12;
    if (n - p < size) {
      frame_err = "Insufficient input: require " + std::to_string(size) + " but " +
                  std::to_string(n - p) + " is available";
      break;
    }
    Record r;
    r.stream_id = sid;
    r.off = p;
    r.len = size;
    recs.push_back(r);
    p += size;
  }
  // An encoder instruction cut by the end of a stream-0 record continues in
  // the next stream-0 record, as the reference decoder keeps the partial
  // instruction's state between read_encoder calls (qpack.c:2815-3150): its
  // bytes move to the front of the next stream-0 record (a new region
  // appended to the file), where the instruction completes and takes effect;
  // a partial instruction at the end of the file is left pending, as there.
  {
    std::vector<qh_field_line> tl(n + 1);
    std::vector<qh_span_in> ts(n + 1);
    std::vector<uint8_t> tail;
    size_t extra = 0;
    for (auto &r : recs)
      if (r.stream_id == 0) extra += r.len;
    file.reserve(file.size() + 2 * extra + 1);
    for (auto &r : recs) {
      if (r.stream_id != 0) continue;
      if (!tail.empty()) {  // this record, behind the previous one's tail
        tail.insert(tail.end(), file.begin() + (std::ptrdiff_t)r.off,
                    file.begin() + (std::ptrdiff_t)(r.off + r.len));
        r.off = file.size();
        r.len = tail.size();
        file.insert(file.end(), tail.begin(), tail.end());
        tail.clear();
      }
      size_t nl = 0, ns = 0;
      const nghttp3_ssize done = qh_qpack_scan_encoder_stream(file.data() + r.off, r.len, r.off,
                                                              tl.data(), tl.size(), &nl, ts.data(),
                                                              ts.size(), &ns);
      if (done >= 0 && (size_t)done < r.len) {
        // the reference decodes a cut Huffman string's bytes as they arrive
        // and fails this record if they already fail
        if (partial_huffman_fails(file.data() + r.off + (size_t)done, r.len - (size_t)done))
          r.partial_bad = true;
        tail.assign(file.begin() + (std::ptrdiff_t)(r.off + (size_t)done),
                    file.begin() + (std::ptrdiff_t)(r.off + r.len));
        r.len = (size_t)done;
      }
    }
  }
  const size_t nf = file.size();
  if (file.empty()) file.push_back(0);
  std::vector<qh_field_line> lines(nf + 1);
  std::vector<qh_span_in> spans(nf + 1);
  std::vector<qh_span_in> huff;
  std::vector<size_t> huff_of;  // Huffman string j -> span index
  std::vector<qh_span_out> hout_batch, hout(nf + 1);
  std::vector<uint8_t> dst;
  std::vector<double> t_frame, t_batch;
  const int reps = config.time_reps > 0 ? config.time_reps : 1;
  size_t nl_tot = 0, ns_tot = 0;
  for (int rep = 0; rep < reps; ++rep) {
    double t0 = now_ms();
    nl_tot = ns_tot = 0;
    huff.clear();
    huff_of.clear();
    for (auto &r : recs) {
      size_t nl = 0, ns = 0;
      r.line0 = nl_tot;
      r.span0 = ns_tot;
      if (r.stream_id == 0) {
        const nghttp3_ssize rv = qh_qpack_scan_encoder_stream(
            file.data() + r.off, r.len, r.off, lines.data() + nl_tot, lines.size() - nl_tot, &nl,
            spans.data() + ns_tot, spans.size() - ns_tot, &ns);
        r.rv = rv < 0 ? (int)rv : ((size_t)rv != r.len ? QH_ERR_QPACK_ENCODER_STREAM_ERROR : 0);
        if (r.rv == 0 && r.partial_bad) r.rv = QH_ERR_QPACK_ENCODER_STREAM_ERROR;
      } else {
        r.prefix.reserved = 0xFFFFFFFFu;  // (the parser sets it to 0 once the prefix is read)
        r.rv = qh_qpack_scan_field_section(file.data() + r.off, r.len, r.off, &r.prefix,
                                           lines.data() + nl_tot, lines.size() - nl_tot, &nl,
                                           spans.data() + ns_tot, spans.size() - ns_tot, &ns);
      }
      for (size_t k = 0; k < nl; ++k) {  // make string indices file-global
        if (lines[nl_tot + k].name >= 0) lines[nl_tot + k].name += (int32_t)ns_tot;
        if (lines[nl_tot + k].value >= 0) lines[nl_tot + k].value += (int32_t)ns_tot;
      }
      for (size_t k = 0; k < ns; ++k) {
        if (spans[ns_tot + k].flags & QH_SPAN_HUFFMAN) {
          huff.push_back(spans[ns_tot + k]);
          huff_of.push_back(ns_tot + k);
        }
      }
      r.nline = nl;
      r.nspan = ns;
      nl_tot += nl;
      ns_tot += ns;
    }
    double t1 = now_ms();
    // every Huffman string of the file in one batch
    const size_t nh = huff.size();
    hout_batch.resize(nh ? nh : 1);
    if (config.scalar) {
      size_t cap = 0;
      for (auto &s : huff) cap += nghttp3_qpack_huffman_estimate_decode_length(s.len) + 1;
      dst.resize(cap + 1);
      size_t o = 0;
      for (size_t j = 0; j < nh; ++j) {
        nghttp3_qpack_huffman_decode_context c;
        nghttp3_qpack_huffman_decode_context_init(&c);
        const nghttp3_ssize w = nghttp3_qpack_huffman_decode(&c, dst.data() + o,
                                                              file.data() + huff[j].off,
                                                              huff[j].len, 1);
        const bool ok = w >= 0 && !nghttp3_qpack_huffman_decode_failure_state(&c);
        hout_batch[j] = {o, ok ? (uint32_t)w : 0u, ok ? 0 : QH_ERR_QPACK_FATAL};
        if (ok) o += (size_t)w;
      }
    } else if (nh) {
      dst.resize(qh_decode_dst_size(huff.data(), nh));
      const int rv = qh_decode_batch(ctx(), file.data(), huff.data(), nh, dst.data(), dst.size(),
                                     hout_batch.data(), QH_WHERE_HOST);
      if (rv != 0) {
        std::cerr << "qh_decode_batch: " << qh_strerror(rv) << std::endl;
        return -1;
      }
    }
    double t2 = now_ms();
    t_frame.push_back(t1 - t0);
    t_batch.push_back(t2 - t1);
  }
  for (size_t j = 0; j < huff.size(); ++j) hout[huff_of[j]] = hout_batch[j];
  Decoded d{&file, &spans, &hout, &dst};
  // replay in stream order
  double t3 = now_ms();
  Table table(config.max_dtable);
  std::string out;
  std::priority_queue<Blocked, std::vector<Blocked>, std::greater<Blocked>> blocked;
  uint64_t seq = 0;
  auto strings_ok = [&](const Record &r) {
    for (size_t k = r.span0; k < r.span0 + r.nspan; ++k)
      if ((spans[k].flags & QH_SPAN_HUFFMAN) && hout[k].status != 0) return false;
    return true;
  };
  // the output is written as the reference's streams it: what was emitted
  // before an error stays in the file
  std::ofstream of(outfile, std::ios::trunc | std::ios::binary);
  if (!of) {
    std::cerr << "Could not open file " << outfile << ": " << strerror(errno) << std::endl;
    return -1;
  }
  auto fail_out = [&]() {
    of.write(out.data(), (std::streamsize)out.size());
    return -1;
  };
  // a record's Huffman and framing verdicts, reported as read_encoder /
  // read_request would (a request's once it is not blocked)
  auto record_ok = [&](const Record &r) {
    if (!strings_ok(r)) {
      std::cerr << (r.stream_id == 0 ? "nghttp3_qpack_decoder_read_encoder: "
                                     : "nghttp3_qpack_decoder_read_request: ")
                << qh_strerror(r.stream_id == 0 ? QH_ERR_QPACK_ENCODER_STREAM_ERROR
                                                : QH_ERR_QPACK_DECOMPRESSION_FAILED)
                << std::endl;
      return false;
    }
    if (r.rv != 0) {
      std::cerr << (r.stream_id == 0 ? "nghttp3_qpack_decoder_read_encoder: "
                                     : "nghttp3_qpack_decoder_read_request: ")
                << qh_strerror(r.rv) << std::endl;
      return false;
    }
    return true;
  };
  for (size_t ri = 0; ri < recs.size(); ++ri) {
    const Record &r = recs[ri];
    // a request whose prefix was read blocks (or not) before its
    // representations are decoded (qpack.c:3419-3436): its other verdicts
    // come when it is emitted
    const bool prefix_read = r.stream_id != 0 && r.prefix.reserved == 0;
    if (!prefix_read && !record_ok(r)) return fail_out();
    if (r.stream_id == 0) {
      for (size_t i = r.line0; i < r.line0 + r.nline; ++i) {
        const qh_field_line &l = lines[i];
        bool ok = true;
        if (l.opcode == QH_ES_SET_DTABLE_CAP) {
          ok = table.set_cap(l.index);
        } else if (l.opcode == QH_ES_INSERT) {
          ok = table.add(d.str((size_t)l.name), d.str((size_t)l.value));
        } else {
          Entry ent;
          if (l.flags & QH_FL_DYNAMIC) {
            ok = table.icnt() >= l.index + 1 && table.valid(table.icnt() - l.index - 1);
            if (ok) ent = table.get(table.icnt() - l.index - 1);
          } else {
            const uint8_t *nm, *v;
            size_t nml, vl;
            ok = qh_qpack_static_entry((size_t)l.index, &nm, &nml, &v, &vl) == 0;
            if (ok) ent = {std::string((const char *)nm, nml), std::string((const char *)v, vl)};
          }
          if (ok)
            ok = l.opcode == QH_ES_DUPLICATE ? table.add(ent.name, ent.value)
                                             : table.add(ent.name, d.str((size_t)l.value));
        }
        if (!ok) {
          std::cerr << "nghttp3_qpack_decoder_read_encoder: " << qh_strerror(QH_ERR_QPACK_ENCODER_STREAM_ERROR)
                    << std::endl;
          return fail_out();
        }
      }
      while (!blocked.empty() && blocked.top().ricnt <= table.icnt()) {
        const Blocked b = blocked.top();
        blocked.pop();
        if (!record_ok(recs[b.rec])) return fail_out();
        if (!emit(table, recs[b.rec], b.ricnt, b.base, lines, d, out)) {
          std::cerr << "nghttp3_qpack_decoder_read_request: " << qh_strerror(QH_ERR_QPACK_DECOMPRESSION_FAILED)
                    << std::endl;
          return fail_out();
        }
      }
      continue;
    }
    uint64_t ricnt = 0, base = 0;
    bool ok = table.ricnt(r.prefix.ricnt, ricnt);
    if (ok && r.prefix.sign) {
      ok = ricnt > r.prefix.delta_base;
      base = ricnt - r.prefix.delta_base - 1;
    } else {
      base = ricnt + r.prefix.delta_base;
    }
    if (!ok) {
      std::cerr << "nghttp3_qpack_decoder_read_request: " << qh_strerror(QH_ERR_QPACK_DECOMPRESSION_FAILED)
                << std::endl;
      return fail_out();
    }
    if (ricnt > table.icnt()) {
      if (blocked.size() >= config.max_blocked) {
        std::cerr << "Too many blocked streams: max_blocked=" << config.max_blocked << std::endl;
        return fail_out();
      }
      blocked.push({ricnt, seq++, base, ri});
      continue;
    }
    if (!record_ok(r)) return fail_out();
    if (!emit(table, r, ricnt, base, lines, d, out)) {
      std::cerr << "nghttp3_qpack_decoder_read_request: " << qh_strerror(QH_ERR_QPACK_DECOMPRESSION_FAILED)
                << std::endl;
      return fail_out();
    }
  }
  double t4 = now_ms();
  of.write(out.data(), (std::streamsize)out.size());
  if (!frame_err.empty()) {
    std::cerr << frame_err << std::endl;
    return -1;
  }
  if (!blocked.empty()) {
    std::cerr << "Still " << blocked.size() << " stream(s) blocked" << std::endl;
    return -1;
  }
  if (config.time_reps > 0) {
    size_t hbytes = 0;
    for (auto &s : huff) hbytes += s.len;
    fprintf(stderr,
            "{\"cmd\": \"decode\", \"path\": \"%s\", \"records\": %zu, \"lines\": %zu, "
            "\"strings\": %zu, \"huffman_strings\": %zu, \"huffman_bytes\": %zu, "
            "\"qif_bytes\": %zu, \"reps\": %d, \"frame_ms\": %.4f, \"batch_ms\": %.4f, "
            "\"replay_ms\": %.4f}\n",
            config.scalar ? "scalar" : "gpu", recs.size(), nl_tot, ns_tot, huff.size(), hbytes,
            out.size(), reps, median(t_frame), median(t_batch), t4 - t3);
  }
  return 0;
}

void print_usage() {
  std::cerr << "Usage: qpack [OPTIONS] <COMMAND> <INFILE> <OUTFILE>" << std::endl;
}

}  // namespace

int main(int argc, char **argv) {
  static const option long_opts[] = {
      {"help", no_argument, nullptr, 'h'},
      {"max-blocked", required_argument, nullptr, 'm'},
      {"max-dtable-size", required_argument, nullptr, 's'},
      {"immediate-ack", no_argument, nullptr, 'a'},
      {"scalar", no_argument, nullptr, 'S'},
      {"time", required_argument, nullptr, 'T'},
      {nullptr, 0, nullptr, 0},
  };
  for (;;) {
    int idx = 0;
    const int c = getopt_long(argc, argv, "hm:s:a", long_opts, &idx);
    if (c == -1) break;
    switch (c) {
      case 'h':
        print_usage();
        std::cerr << R"(
  <COMMAND>   "encode" or "decode"
  <INFILE>    Path to an input file
  <OUTFILE>   Path to an output file
Options:
  -h, --help  Display this help and exit.
  -m, --max-blocked=<N>
              The maximum number of streams which are permitted to be blocked.
  -s, --max-dtable-size=<N>
              The maximum size of dynamic table (encode: 0 only).
  -a, --immediate-ack
              Turn on immediate acknowledgement (no effect at -s 0).
  --scalar    Run the batches through the scalar drop-ins on the CPU.
  --time=<R>  Repeat the batch part R times; print timings (JSON) to stderr.
)";
        return 0;
      case 'm':
        config.max_blocked = strtoul(optarg, nullptr, 10);
        break;
      case 's':
        config.max_dtable = strtoul(optarg, nullptr, 10);
        break;
      case 'a':
        config.immediate_ack = true;
        break;
      case 'S':
        config.scalar = true;
        break;
      case 'T':
        config.time_reps = atoi(optarg);
        break;
      default:
        print_usage();
        return EXIT_FAILURE;
    }
  }
  if (argc - optind < 3) {
    std::cerr << "Too few arguments" << std::endl;
    print_usage();
    return EXIT_FAILURE;
  }
  const std::string command = argv[optind++];
  const char *infile = argv[optind++];
  const char *outfile = argv[optind++];
  int rv;
  if (command == "encode") {
    rv = encode(outfile, infile);
  } else if (command == "decode") {
    rv = decode(outfile, infile);
  } else {
    std::cerr << "Unrecognized command: " << command << std::endl;
    print_usage();
    return EXIT_FAILURE;
  }
  if (g_ctx) qh_ctx_del(g_ctx);
  return rv != 0 ? EXIT_FAILURE : 0;
}
