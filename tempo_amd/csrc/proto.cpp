// proto.cpp — decode-to-columnar loader for proto-object v2 blocks and the host side of
// proto-object search (the device scan is proto_scan_kernel in proto_scan.hip).
//
// Reference semantics restated here (each with its file:line):
//   object framing      object.UnmarshalAndAdvanceBuffer (tempodb/encoding/v2/object.go:82-113)
//   paged iterator      pagedIterator.Next (tempodb/encoding/v2/iterator_paged.go:62-131):
//                       index records gathered into ~ChunkSizeBytes chunks, every page of a
//                       chunk read and decompressed before its first object
//   object decoders     v1 (pkg/model/v1/object_decoder.go): TraceBytes; v2
//                       (pkg/model/v2/object_decoder.go:28-89, segment_decoder.go:106-122):
//                       u32 start, u32 end (little endian) + TraceBytes, FastRange prefilter
//   proto decoding      gogo-generated Unmarshal of tempopb.TraceBytes / Trace and the OTLP
//                       messages (pkg/tempopb/tempo.pb.go, trace/v1/trace.pb.go,
//                       common/v1/common.pb.go, resource/v1/resource.pb.go)
//   matching            trace.MatchesProto / matchSpan / matchAttributes
//                       (pkg/model/trace/matches.go:33-184)
//
// Per object the loader keeps: the FastRange seconds, the object length, traceStart
// (min span start) with DurationMs and the start/end seconds MatchesProto derives from
// it, the root span's name and its batch's service.name, a parse-error flag, and for
// every attribute key the set of typed values the trace holds under it (resource
// attributes of every batch that has a resource, span attributes of every span; span
// names under "name" and span status codes under "error" and "status.code", the keys
// matchSpan reads). A tag term (k, v) is then "some value of the trace's set for key k
// matches v" — matchAttributes / matchSpan delete a key from tagsToFind on the first
// such value, so the reference's loop is exactly this existential test.
//
// Where the reference panics (nil AnyValue in an attribute, nil Status with an
// error/status.code tag, nil Resource on the root span's batch) this treats the value as
// absent / STATUS_CODE_UNSET / no resource attributes.
#include "proto.hpp"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "block.hpp"
#include "common.hpp"

namespace tsg {

// ------------------------------------------------------------------------------------
// Go strconv (ParseInt base 10, ParseFloat 64, ParseBool)
bool go_parse_int(std::string_view s, int64_t &out) {  // strconv.ParseInt(s, 10, 64)
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i == s.size()) return false;
  uint64_t v = 0;
  const uint64_t lim = neg ? (1ULL << 63) : (1ULL << 63) - 1;
  for (; i < s.size(); i++) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;  // (base 10 given: no underscores, no prefix)
    const uint64_t d = uint64_t(c - '0');
    if (v > (lim - d) / 10) return false;  // ErrRange
    v = v * 10 + d;
  }
  out = neg ? int64_t(0 - v) : int64_t(v);
  return true;
}

static bool ieq(std::string_view a, const char *b) {
  size_t n = std::strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; i++)
    if (std::tolower(static_cast<unsigned char>(a[i])) != b[i]) return false;
  return true;
}

// strconv.underscoreOK (atoi.go): underscores only between digits (or after a base prefix)
static bool underscore_ok(std::string_view s) {
  char saw = '^';
  size_t i = 0;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) s.remove_prefix(1);
  bool hex = false;
  if (s.size() >= 2 && s[0] == '0') {
    const char l = char(std::tolower(static_cast<unsigned char>(s[1])));
    if (l == 'b' || l == 'o' || l == 'x') {
      i = 2;
      saw = '0';
      hex = l == 'x';
    }
  }
  for (; i < s.size(); i++) {
    const char c = s[i], l = char(std::tolower(static_cast<unsigned char>(c)));
    if ((c >= '0' && c <= '9') || (hex && l >= 'a' && l <= 'f')) {
      saw = '0';
      continue;
    }
    if (c == '_') {
      if (saw != '0') return false;
      saw = '_';
      continue;
    }
    if (saw == '_') return false;
    saw = '!';
  }
  return saw != '_';
}

// strconv.ParseFloat(s, 64): Go float literal syntax (decimal, or hex with a mandatory p
// exponent), optional sign, "inf"/"infinity"/"nan" in any case, underscores per
// underscoreOK; correctly rounded (strtod); out of range (±Inf from a finite literal) is
// an error.
bool go_parse_float(std::string_view s, double &out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  std::string_view r = s.substr(i);
  if (ieq(r, "inf") || ieq(r, "infinity")) {
    out = neg ? -HUGE_VAL : HUGE_VAL;
    return true;
  }
  if (ieq(r, "nan")) {
    if (i) return false;  // (special: a sign is not accepted with NaN)
    out = std::nan("");
    return true;
  }
  std::string clean;
  clean.reserve(s.size());
  bool hex = r.size() >= 2 && r[0] == '0' && (r[1] == 'x' || r[1] == 'X');
  size_t j = hex ? 2 : 0;
  bool digits = false, dot = false, exp = false, underscores = false;
  clean.append(s.substr(0, i));
  clean.append(r.substr(0, j));
  for (; j < r.size(); j++) {
    const char c = r[j], l = char(std::tolower(static_cast<unsigned char>(c)));
    if (c == '_') {
      underscores = true;
      continue;
    }
    if ((c >= '0' && c <= '9') || (hex && l >= 'a' && l <= 'f')) {
      digits = true;
      clean.push_back(c);
      continue;
    }
    if (c == '.' && !dot) {
      dot = true;
      clean.push_back(c);
      continue;
    }
    if (((!hex && l == 'e') || (hex && l == 'p')) && digits) {
      exp = true;
      clean.push_back(c);
      j++;
      if (j < r.size() && (r[j] == '+' || r[j] == '-')) clean.push_back(r[j++]);
      bool ed = false;
      for (; j < r.size(); j++) {
        if (r[j] == '_') {
          underscores = true;
          continue;
        }
        if (r[j] < '0' || r[j] > '9') return false;
        ed = true;
        clean.push_back(r[j]);
      }
      if (!ed) return false;
      break;
    }
    return false;
  }
  if (!digits) return false;
  if (hex && !exp) return false;  // hexadecimal mantissa requires a 'p' exponent
  if (underscores && !underscore_ok(s)) return false;
  errno = 0;
  char *end = nullptr;
  const double v = std::strtod(clean.c_str(), &end);
  if (end != clean.c_str() + clean.size()) return false;
  if (std::isinf(v)) return false;  // ErrRange
  out = v;
  return true;
}

bool go_parse_bool(std::string_view s, bool &out) {  // strconv.ParseBool
  if (s == "1" || s == "t" || s == "T" || s == "TRUE" || s == "true" || s == "True") {
    out = true;
    return true;
  }
  if (s == "0" || s == "f" || s == "F" || s == "FALSE" || s == "false" || s == "False") {
    out = false;
    return true;
  }
  return false;
}

// ------------------------------------------------------------------------------------
// protobuf wire format with gogo Unmarshal's error behaviour
namespace {

struct Wire {
  const uint8_t *p, *e;
  bool varint(uint64_t &v) {
    v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= e) return false;  // io.ErrUnexpectedEOF
      const uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << shift;
      if (b < 0x80) return true;
    }
    return false;  // ErrIntOverflow
  }
  bool bytes(std::string_view &out) {
    uint64_t l;
    if (!varint(l)) return false;
    if (l > uint64_t(e - p)) return false;  // (negative length / past the end)
    out = std::string_view(reinterpret_cast<const char *>(p), size_t(l));
    p += l;
    return true;
  }
  bool fixed64(uint64_t &v) {
    if (e - p < 8) return false;
    v = le64(p);
    p += 8;
    return true;
  }
  // skipXxx (gogo): unknown fields, groups included
  bool skip(uint32_t wt, int depth = 0) {
    uint64_t v;
    std::string_view b;
    switch (wt) {
      case 0: return varint(v);
      case 1: if (e - p < 8) return false; p += 8; return true;
      case 2: return bytes(b);
      case 5: if (e - p < 4) return false; p += 4; return true;
      case 3: {
        if (depth > 64) return false;
        for (;;) {
          uint64_t tag;
          if (!varint(tag)) return false;
          const uint32_t w = uint32_t(tag & 7);
          if (w == 4) return true;  // the matching end group
          if ((tag >> 3) == 0) return false;
          if (!skip(w, depth + 1)) return false;
        }
      }
      default: return false;  // wire type 4 outside a group, 6, 7
    }
  }
  // next field of a message: false at the end; sets bad on an illegal tag
  bool next(uint32_t &field, uint32_t &wt, bool &bad) {
    if (p >= e) return false;
    uint64_t tag;
    if (!varint(tag)) {
      bad = true;
      return false;
    }
    wt = uint32_t(tag & 7);
    if (wt == 4 || (tag >> 3) == 0 || (tag >> 3) > 0x1fffffff) {  // end group / illegal tag
      bad = true;
      return false;
    }
    field = uint32_t(tag >> 3);
    return true;
  }
};

struct TypedVal {
  uint8_t type;
  std::string bytes;
};

struct AnyVal {
  int type = 0;  // 0 none, PV_* for the kinds matchAttributes compares, 9 array/kvlist
  std::string_view s;
  uint64_t u = 0;
};

struct KV {
  std::string_view key;
  AnyVal val;
  bool has_val = false;
};

bool parse_anyvalue(std::string_view buf, AnyVal &v, int depth);
bool parse_kv(std::string_view buf, KV &kv, int depth);

bool parse_kvlist(std::string_view buf, int depth) {  // KeyValueList / ArrayValue bodies: validated only
  if (depth > 100) return false;
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    if (f == 1) {
      std::string_view b;
      if (wt != 2 || !w.bytes(b)) return false;
      KV kv;
      if (!parse_kv(b, kv, depth + 1)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}
bool parse_array(std::string_view buf, int depth) {
  if (depth > 100) return false;
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    if (f == 1) {
      std::string_view b;
      if (wt != 2 || !w.bytes(b)) return false;
      AnyVal a;
      if (!parse_anyvalue(b, a, depth + 1)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

// AnyValue: oneof — the last member present wins (AnyValue.Unmarshal assigns m.Value)
bool parse_anyvalue(std::string_view buf, AnyVal &v, int depth) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    uint64_t x;
    switch (f) {
      case 1:
        if (wt != 2 || !w.bytes(b)) return false;
        v.type = PV_STRING;
        v.s = b;
        break;
      case 2:
        if (wt != 0 || !w.varint(x)) return false;
        v.type = PV_BOOL;
        v.u = x != 0;
        break;
      case 3:
        if (wt != 0 || !w.varint(x)) return false;
        v.type = PV_INT;
        v.u = x;
        break;
      case 4:
        if (wt != 1 || !w.fixed64(x)) return false;
        v.type = PV_DOUBLE;
        v.u = x;
        break;
      case 5:
        if (wt != 2 || !w.bytes(b) || !parse_array(b, depth + 1)) return false;
        v.type = 9;
        break;
      case 6:
        if (wt != 2 || !w.bytes(b) || !parse_kvlist(b, depth + 1)) return false;
        v.type = 9;
        break;
      default:
        if (!w.skip(wt)) return false;
    }
  }
  return !bad;
}

// KeyValue: key (last wins), value (an embedded message: repeated occurrences merge)
bool parse_kv(std::string_view buf, KV &kv, int depth) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    if (f == 1) {
      if (wt != 2 || !w.bytes(b)) return false;
      kv.key = b;
    } else if (f == 2) {
      if (wt != 2 || !w.bytes(b)) return false;
      kv.has_val = true;
      if (!parse_anyvalue(b, kv.val, depth + 1)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

bool parse_kv_into(std::string_view b, std::vector<KV> &out) {
  KV kv;
  if (!parse_kv(b, kv, 0)) return false;
  out.push_back(kv);
  return true;
}

// messages that are only validated (gogo parses them, MatchesProto does not read them)
bool parse_generic(std::string_view buf, const std::map<uint32_t, int> &fields) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    auto it = fields.find(f);
    if (it == fields.end()) {
      if (!w.skip(wt)) return false;
      continue;
    }
    const int kind = it->second;  // 0 varint, 1 fixed64, 2 bytes, 3 KeyValue
    std::string_view b;
    uint64_t x;
    if (kind == 0) {
      if (wt != 0 || !w.varint(x)) return false;
    } else if (kind == 1) {
      if (wt != 1 || !w.fixed64(x)) return false;
    } else {
      if (wt != 2 || !w.bytes(b)) return false;
      if (kind == 3) {
        KV kv;
        if (!parse_kv(b, kv, 0)) return false;
      }
    }
  }
  return !bad;
}

struct Span {
  std::string_view name;
  bool has_parent = false;  // len(ParentSpanId) != 0 (last occurrence wins)
  uint64_t start = 0, end = 0;
  int32_t code = 0;         // Status.Code (STATUS_CODE_UNSET without a Status)
  std::vector<KV> attrs;
};

bool parse_status(std::string_view buf, int32_t &code) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    uint64_t x;
    std::string_view b;
    if (f == 1) {
      if (wt != 0 || !w.varint(x)) return false;
    } else if (f == 2) {
      if (wt != 2 || !w.bytes(b)) return false;
    } else if (f == 3) {
      if (wt != 0 || !w.varint(x)) return false;
      code = int32_t(uint32_t(x));  // (enum: int32)
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

bool parse_span(std::string_view buf, Span &s) {
  static const std::map<uint32_t, int> kEvent = {{1, 1}, {2, 2}, {3, 3}, {4, 0}};
  static const std::map<uint32_t, int> kLink = {{1, 2}, {2, 2}, {3, 2}, {4, 3}, {5, 0}};
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    uint64_t x;
    switch (f) {
      case 1: case 2: case 3:
        if (wt != 2 || !w.bytes(b)) return false;
        break;
      case 4:
        if (wt != 2 || !w.bytes(b)) return false;
        s.has_parent = !b.empty();
        break;
      case 5:
        if (wt != 2 || !w.bytes(b)) return false;
        s.name = b;
        break;
      case 6: case 10: case 12: case 14:
        if (wt != 0 || !w.varint(x)) return false;
        break;
      case 7:
        if (wt != 1 || !w.fixed64(x)) return false;
        s.start = x;
        break;
      case 8:
        if (wt != 1 || !w.fixed64(x)) return false;
        s.end = x;
        break;
      case 9:
        if (wt != 2 || !w.bytes(b) || !parse_kv_into(b, s.attrs)) return false;
        break;
      case 11:
        if (wt != 2 || !w.bytes(b) || !parse_generic(b, kEvent)) return false;
        break;
      case 13:
        if (wt != 2 || !w.bytes(b) || !parse_generic(b, kLink)) return false;
        break;
      case 15:
        if (wt != 2 || !w.bytes(b) || !parse_status(b, s.code)) return false;  // (merges: last code wins)
        break;
      default:
        if (!w.skip(wt)) return false;
    }
  }
  return !bad;
}

struct Batch {
  bool has_resource = false;
  std::vector<KV> res_attrs;
  std::vector<Span> spans;  // every span of every InstrumentationLibrarySpans, in order
};

bool parse_ils(std::string_view buf, Batch &bt) {
  static const std::map<uint32_t, int> kLib = {{1, 2}, {2, 2}};
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    if (f == 1) {
      if (wt != 2 || !w.bytes(b) || !parse_generic(b, kLib)) return false;
    } else if (f == 2) {
      if (wt != 2 || !w.bytes(b)) return false;
      bt.spans.emplace_back();
      if (!parse_span(b, bt.spans.back())) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

bool parse_resource(std::string_view buf, Batch &bt) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    uint64_t x;
    if (f == 1) {
      if (wt != 2 || !w.bytes(b) || !parse_kv_into(b, bt.res_attrs)) return false;
    } else if (f == 2) {
      if (wt != 0 || !w.varint(x)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

bool parse_batch(std::string_view buf, Batch &bt) {  // ResourceSpans
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    if (f == 1) {  // Resource: an embedded message, repeated occurrences merge (attributes append)
      if (wt != 2 || !w.bytes(b)) return false;
      bt.has_resource = true;
      if (!parse_resource(b, bt)) return false;
    } else if (f == 2) {
      if (wt != 2 || !w.bytes(b) || !parse_ils(b, bt)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

bool parse_trace(std::string_view buf, std::vector<Batch> &out) {  // tempopb.Trace
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    if (f == 1) {
      if (wt != 2 || !w.bytes(b)) return false;
      out.emplace_back();
      if (!parse_batch(b, out.back())) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

// PrepareForRead: TraceBytes.traces, each a marshalled Trace; batches concatenated
bool parse_trace_bytes(std::string_view buf, std::vector<Batch> &out) {
  Wire w{reinterpret_cast<const uint8_t *>(buf.data()), reinterpret_cast<const uint8_t *>(buf.data()) + buf.size()};
  uint32_t f, wt;
  bool bad = false;
  while (w.next(f, wt, bad)) {
    std::string_view b;
    if (f == 1) {
      if (wt != 2 || !w.bytes(b)) return false;
      if (!parse_trace(b, out)) return false;
    } else if (!w.skip(wt)) return false;
  }
  return !bad;
}

std::string typed(uint8_t t, std::string_view s) {
  std::string o(1, char(t));
  o.append(s);
  return o;
}
std::string typed(uint8_t t, uint64_t v) {
  std::string o(9, '\0');
  o[0] = char(t);
  std::memcpy(&o[1], &v, 8);
  return o;
}

// one object's contribution: facts per key + the per-trace scalars
struct ObjFacts {
  std::vector<std::pair<std::string_view, std::string>> facts;  // (key, typed value), unsorted
  uint64_t tstart = ~0ULL, tend = 0;
  std::string root_name = "<root span not yet received>", root_svc = "<root span not yet received>";
  bool bad = false;
};

void object_facts(std::string_view body, ObjFacts &o) {
  std::vector<Batch> batches;
  if (!parse_trace_bytes(body, batches)) {
    o.bad = true;
    return;
  }
  const Span *root = nullptr;
  const Batch *root_batch = nullptr;
  auto attr = [&](const KV &kv) {
    if (!kv.has_val) return;  // (nil AnyValue: the reference dereferences it)
    const AnyVal &v = kv.val;
    if (v.type == PV_STRING) o.facts.emplace_back(kv.key, typed(PV_STRING, v.s));
    else if (v.type == PV_BOOL || v.type == PV_INT || v.type == PV_DOUBLE) o.facts.emplace_back(kv.key, typed(uint8_t(v.type), v.u));
  };
  for (const Batch &b : batches) {
    if (b.has_resource)
      for (const KV &kv : b.res_attrs) attr(kv);
    for (const Span &s : b.spans) {
      if (s.start < o.tstart) o.tstart = s.start;
      if (s.end > o.tend) o.tend = s.end;
      if (!root && !s.has_parent) {
        root = &s;
        root_batch = &b;
      }
      o.facts.emplace_back("name", typed(PV_SPANNAME, s.name));
      const uint64_t code = uint64_t(uint32_t(s.code));
      o.facts.emplace_back("error", typed(PV_SPANCODE, code));
      o.facts.emplace_back("status.code", typed(PV_SPANCODE, code));
      for (const KV &kv : s.attrs) attr(kv);
    }
  }
  if (root) {
    o.root_name = std::string(root->name);
    if (root_batch->has_resource)
      for (const KV &kv : root_batch->res_attrs)
        if (kv.key == "service.name") {  // a.Value.GetStringValue(): "" unless a string
          o.root_svc = kv.has_val && kv.val.type == PV_STRING ? std::string(kv.val.s) : std::string();
          break;
        }
  }
}

std::string json_get(const std::string &js, const char *name) {
  const std::string pat = std::string("\"") + name + "\"";
  size_t p = js.find(pat);
  if (p == std::string::npos) return "";
  p += pat.size();
  while (p < js.size() && (js[p] == ':' || js[p] == ' ')) p++;
  if (p < js.size() && js[p] == '"') {
    const size_t e = js.find('"', p + 1);
    return js.substr(p + 1, e - p - 1);
  }
  size_t e = p;
  while (e < js.size() && js[e] != ',' && js[e] != '}') e++;
  return js.substr(p, e - p);
}

struct PageObjs {
  uint8_t status = PP_OK;
  std::vector<std::string_view> ids, bodies;
  std::vector<ObjFacts> facts;
  std::vector<uint32_t> fr_start, fr_end;
  std::vector<uint8_t> hdr_bad;
  std::vector<uint8_t> buf;
};

}  // namespace

// ------------------------------------------------------------------------------------
void proto_load_host(ProtoBlock &b, const std::string &dir) {
  std::vector<uint8_t> meta;
  if (!read_file(dir + "/meta.json", meta)) fail(TSG_E_NOT_FOUND, "meta.json not found");
  const std::string js(meta.begin(), meta.end());
  const std::string enc = json_get(js, "encoding"), denc = json_get(js, "dataEncoding");
  b.enc = enc.empty() ? 0 : parse_encoding(enc);
  if (b.enc < 0) fail(TSG_E_UNSUPPORTED_ENCODING, "unknown encoding " + enc);
  if (denc == "v1") b.v2 = false;
  else if (denc == "v2") b.v2 = true;
  else fail(TSG_E_UNSUPPORTED, "unknown dataEncoding '" + denc + "' (model.NewObjectDecoder)");
  const std::string ips = json_get(js, "indexPageSize"), tr = json_get(js, "totalRecords");
  const uint32_t page_size = ips.empty() ? 0 : json_u32(ips, "indexPageSize");
  b.total_records = tr.empty() ? 0 : json_u32(tr, "totalRecords");
  std::vector<uint8_t> idx, data;
  if (!read_file(dir + "/index", idx)) fail(TSG_E_IO, "index missing");
  if (!read_file(dir + "/data", data)) fail(TSG_E_IO, "data missing");
  bool trunc = false;
  const std::vector<IndexRecord> recs = read_index(idx.data(), idx.size(), page_size, b.total_records, &trunc);
  b.index_err_at = uint32_t(recs.size());  // At(i) for i >= this errors (== total_records if none)
  const size_t np = recs.size();
  // every page decoded and split into objects, in parallel
  std::vector<PageObjs> pages(np);
  auto work = [&](size_t p) {
    PageObjs &po = pages[p];
    try {
      read_data_page(data.data(), data.size(), recs[p], b.enc, po.buf);
    } catch (const Error &) {
      po.status = PP_DECODE;
      return;
    }
    const uint8_t *cur = po.buf.data();
    size_t left = po.buf.size();
    while (left) {  // UnmarshalAndAdvanceBuffer
      if (left < 8) {
        po.status = PP_FRAMING;
        break;
      }
      const uint32_t total = le32(cur), il = le32(cur + 4);
      const uint32_t rest = total - 8;
      if (uint64_t(left - 8) < rest || il > rest) {
        po.status = PP_FRAMING;
        break;
      }
      std::string_view id(reinterpret_cast<const char *>(cur + 8), il);
      std::string_view obj(reinterpret_cast<const char *>(cur + 8 + il), rest - il);
      po.ids.push_back(id);
      po.bodies.push_back(obj);
      po.facts.emplace_back();
      ObjFacts &of = po.facts.back();
      uint32_t fs = 0, fe = 0;
      uint8_t hb = 0;
      std::string_view body = obj;
      if (b.v2) {
        if (obj.size() < 8) {  // stripStartEnd: "buffer too short to have start/end"
          hb = 1;
        } else {
          fs = le32(reinterpret_cast<const uint8_t *>(obj.data()));
          fe = le32(reinterpret_cast<const uint8_t *>(obj.data()) + 4);
          body = obj.substr(8);
        }
      }
      if (!hb) object_facts(body, of);
      po.fr_start.push_back(fs);
      po.fr_end.push_back(fe);
      po.hdr_bad.push_back(hb);
      cur += 8 + rest;
      left -= 8 + rest;
    }
  };
  {
    const size_t nth = std::max<size_t>(1, std::min<size_t>(np, std::max(1u, std::thread::hardware_concurrency()) / 2));
    std::vector<std::thread> th;
    std::mutex mu;
    size_t nextp = 0;
    for (size_t t = 0; t < std::min<size_t>(nth, 16); t++)
      th.emplace_back([&] {
        for (;;) {
          size_t p;
          {
            std::lock_guard<std::mutex> lk(mu);
            if (nextp >= np) return;
            p = nextp++;
          }
          work(p);
        }
      });
    for (auto &t : th) t.join();
  }
  // columns
  b.page_first.assign(1, 0);
  for (size_t p = 0; p < np; p++) {
    b.page_len.push_back(recs[p].length);
    b.page_status.push_back(pages[p].status);
    b.n += uint32_t(pages[p].ids.size());
    b.page_first.push_back(b.n);
  }
  const uint32_t n = b.n;
  b.id_off.reserve(n);
  b.obj_len.reserve(n);
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> tv(n);  // per trace: (key id, value id)
  std::vector<std::unordered_map<std::string, uint32_t>> vdict;
  uint32_t t = 0;
  for (size_t p = 0; p < np; p++) {
    PageObjs &po = pages[p];
    for (size_t j = 0; j < po.ids.size(); j++, t++) {
      b.id_off.push_back(uint32_t(b.ids.size()));
      if (b.ids.size() + po.ids[j].size() >= (1ull << 32)) fail(TSG_E_UNSUPPORTED, "object ids larger than 4 GiB in one block");
      b.id_len.push_back(uint32_t(po.ids[j].size()));
      b.ids.insert(b.ids.end(), po.ids[j].begin(), po.ids[j].end());
      b.obj_len.push_back(uint32_t(po.bodies[j].size()));
      b.fr_start.push_back(po.fr_start[j]);
      b.fr_end.push_back(po.fr_end[j]);
      ObjFacts &of = po.facts[j];
      uint8_t fl = po.hdr_bad[j] ? PF_HDRBAD : 0;
      if (of.bad) fl |= PF_BAD;
      b.flags.push_back(fl);
      // MatchesProto's derived values (matches.go:81-91)
      const uint64_t sms = of.tstart / 1000000, ems = of.tend / 1000000;
      b.start_ns.push_back(of.tstart);
      b.dur_ms.push_back(uint32_t(ems - sms));
      b.st_sec.push_back(uint32_t(sms / 1000));
      b.en_sec.push_back(uint32_t(ems / 1000));
      b.svc_off.push_back(uint32_t(b.names.size()));
      b.svc_len.push_back(uint32_t(of.root_svc.size()));
      b.names += of.root_svc;
      b.root_off.push_back(uint32_t(b.names.size()));
      b.root_len.push_back(uint32_t(of.root_name.size()));
      b.names += of.root_name;
      for (auto &fv : of.facts) {
        std::string key(fv.first);
        auto it = b.key_index.find(key);
        uint32_t kid;
        if (it == b.key_index.end()) {
          kid = uint32_t(b.keys.size());
          b.key_index.emplace(key, kid);
          b.keys.emplace_back();
          b.keys.back().name = key;
          vdict.emplace_back();
        } else {
          kid = it->second;
        }
        auto &vd = vdict[kid];
        auto vit = vd.find(fv.second);
        uint32_t vid;
        if (vit == vd.end()) {
          vid = uint32_t(b.keys[kid].vals.size());
          vd.emplace(fv.second, vid);
          b.keys[kid].vals.push_back(std::move(fv.second));
        } else {
          vid = vit->second;
        }
        tv[t].emplace_back(kid, vid);
      }
      std::vector<std::pair<std::string_view, std::string>>().swap(of.facts);
    }
    std::vector<uint8_t>().swap(po.buf);
  }
  // per key: value sets interned, one column
  const size_t nk = b.keys.size();
  std::vector<std::map<std::vector<uint32_t>, uint32_t>> sets(nk);
  std::vector<std::vector<uint32_t>> colv(nk, std::vector<uint32_t>(n, 0xffffffffu));
  for (uint32_t i = 0; i < n; i++) {
    auto &f = tv[i];
    std::sort(f.begin(), f.end());
    f.erase(std::unique(f.begin(), f.end()), f.end());
    for (size_t a = 0; a < f.size();) {
      size_t e = a;
      std::vector<uint32_t> vs;
      while (e < f.size() && f[e].first == f[a].first) vs.push_back(f[e++].second);
      const uint32_t kid = f[a].first;
      auto &sm = sets[kid];
      auto it = sm.find(vs);
      uint32_t sid;
      if (it == sm.end()) {
        sid = uint32_t(sm.size());
        ProtoKey &K = b.keys[kid];
        if (K.set_off.empty()) K.set_off.push_back(0);
        K.set_vals.insert(K.set_vals.end(), vs.begin(), vs.end());
        K.set_off.push_back(uint32_t(K.set_vals.size()));
        sm.emplace(std::move(vs), sid);
      } else {
        sid = it->second;
      }
      colv[kid][i] = sid;
      a = e;
    }
  }
  for (size_t k = 0; k < nk; k++) {
    ProtoKey &K = b.keys[k];
    const size_t nsets = sets[k].size();
    K.width = nsets < 0xff ? 1 : nsets < 0xffff ? 2 : 4;
    K.col.resize(size_t(n) * K.width);
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t v = colv[k][i];
      if (K.width == 1) K.col[i] = uint8_t(v == 0xffffffffu ? 0xff : v);
      else if (K.width == 2) {
        const uint16_t x = uint16_t(v == 0xffffffffu ? 0xffff : v);
        std::memcpy(&K.col[size_t(i) * 2], &x, 2);
      } else {
        std::memcpy(&K.col[size_t(i) * 4], &v, 4);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// query-time dictionary matching: one term (k, v) against a key's typed values
static bool value_matches(const std::string &key, const std::string &tv, std::string_view v) {
  const uint8_t t = uint8_t(tv[0]);
  std::string_view payload(tv.data() + 1, tv.size() - 1);
  uint64_t u = 0;
  if (payload.size() == 8) std::memcpy(&u, payload.data(), 8);
  switch (t) {
    case PV_STRING:  // strings.Contains
      return payload.find(v) != std::string_view::npos;
    case PV_INT: {
      int64_t n;
      return go_parse_int(v, n) && int64_t(u) == n;
    }
    case PV_DOUBLE: {
      double f, d;
      std::memcpy(&d, &u, 8);
      return go_parse_float(v, f) && d == f;
    }
    case PV_BOOL: {
      bool bv;
      return go_parse_bool(v, bv) && (u != 0) == bv;
    }
    case PV_SPANNAME:  // matchSpan: name == s.Name
      return payload == v;
    case PV_SPANCODE: {
      const int32_t code = int32_t(uint32_t(u));
      if (key == "error") return v == "true" && code == 2;  // Status_STATUS_CODE_ERROR
      // StatusCodeMapping[status] (0 for a missing key) == int(s.Status.Code)
      const int want = v == "ok" ? 1 : v == "error" ? 2 : 0;
      return code == want;
    }
  }
  return false;
}

std::vector<uint32_t> proto_term_bitmap(const ProtoBlock &b, const std::string &key, std::string_view v,
                                        bool &present) {
  auto it = b.key_index.find(key);
  present = it != b.key_index.end();
  if (!present) return {};
  const ProtoKey &K = b.keys[it->second];
  std::vector<uint8_t> vm(K.vals.size());
  for (size_t i = 0; i < K.vals.size(); i++) vm[i] = value_matches(key, K.vals[i], v);
  const size_t nsets = K.set_off.empty() ? 0 : K.set_off.size() - 1;
  std::vector<uint32_t> bm((nsets + 31) / 32 + 1, 0);
  for (size_t s = 0; s < nsets; s++)
    for (uint32_t j = K.set_off[s]; j < K.set_off[s + 1]; j++)
      if (vm[K.set_vals[j]]) {
        bm[s >> 5] |= 1u << (s & 31);
        break;
      }
  return bm;
}

}  // namespace tsg
