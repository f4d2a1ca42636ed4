// proto.hpp — proto-object backend search: the v1/v2 trace
// objects of a v2 block decoded once into per-trace columns and per-key value-set
// columns, searched with MatchesProto semantics by proto_scan_kernel (proto_scan.hip).
//
// Reference path: tempodb.Search -> v2.BackendBlock.Search (tempodb/encoding/v2/
// backend_block.go:159-231) -> ObjectDecoder.Matches (pkg/model/v2/object_decoder.go:57-89,
// pkg/model/v1/object_decoder.go) -> trace.MatchesProto (pkg/model/trace/matches.go:33-184).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "tsg.h"

namespace tsg {

struct DeviceCtx;
struct Ctx;

// value types of the per-key dictionaries: the AnyValue kinds matchAttributes compares
// (matches.go:160-178) and the span fields matchSpan compares (matches.go:125-143)
enum : uint8_t { PV_STRING = 1, PV_BOOL = 2, PV_INT = 3, PV_DOUBLE = 4, PV_SPANNAME = 5, PV_SPANCODE = 6 };
// per-trace flags
enum : uint8_t { PF_BAD = 1, PF_HDRBAD = 2 };
// per-page status
enum : uint8_t { PP_OK = 0, PP_DECODE = 1, PP_FRAMING = 2 };

struct ProtoKey {
  std::string name;
  std::vector<std::string> vals;        // typed value: type byte + payload (string bytes / 8-byte LE)
  std::vector<uint32_t> set_off;        // value sets (CSR over value ids), nsets + 1
  std::vector<uint32_t> set_vals;
  uint32_t width = 1;                   // column bytes: 1, 2, 4 (all-ones = key absent)
  std::vector<uint8_t> col;             // n * width (host copy until upload)
  const uint8_t *d_col = nullptr;
};

struct ProtoBlock {
  bool v2 = true;                       // dataEncoding "v2": objects carry start/end seconds
  int enc = 0;                          // page encoding
  uint32_t n = 0;                       // objects (traces), iterator order
  uint32_t total_records = 0;           // meta totalRecords (index records = pages)
  uint32_t index_err_at = 0;            // first record whose index At() fails (total_records if none)
  std::vector<uint32_t> page_first;     // per page: first object, npages + 1
  std::vector<uint32_t> page_len;       // record length (the iterator's chunking)
  std::vector<uint8_t> page_status;     // PP_*
  // per object (host)
  std::vector<uint8_t> ids;
  std::vector<uint32_t> id_off;
  std::vector<uint32_t> id_len;  // (object ids of any length: v2 objects are not limited to 16 bytes)
  std::vector<uint32_t> obj_len;
  std::vector<uint64_t> start_ns;       // traceStart (min span start; MaxUint64 without spans)
  std::vector<uint32_t> dur_ms, st_sec, en_sec, fr_start, fr_end;
  std::vector<uint8_t> flags;
  std::string names;
  std::vector<uint32_t> svc_off, svc_len, root_off, root_len;
  std::vector<ProtoKey> keys;
  std::unordered_map<std::string, uint32_t> key_index;
  // device
  DeviceCtx *dc = nullptr;
  std::vector<void *> allocs;
  const uint32_t *d_u32 = nullptr;      // [fr_start | fr_end | st_sec | en_sec | dur_ms | obj_len] x n
  const uint8_t *d_flags = nullptr;
  uint64_t device_bytes = 0;
};

void proto_block_open(Ctx &c, ProtoBlock &b, const std::string &dir, int device_hint);
void proto_block_free(ProtoBlock &b);

struct ProtoOut {
  std::vector<uint32_t> traces;         // object indices of the matches, in order
  uint64_t inspected_traces = 0, inspected_bytes = 0, skipped_traces = 0;
  int status = TSG_OK;
  std::string error;
  uint64_t kernel_ns = 0;
};
void proto_search(ProtoBlock &b, const tsg_proto_request &req, ProtoOut &out);

// Go strconv semantics used by matchAttributes (exposed for the tests through the ABI)
bool go_parse_int(std::string_view s, int64_t &out);
bool go_parse_float(std::string_view s, double &out);
bool go_parse_bool(std::string_view s, bool &out);

}  // namespace tsg
