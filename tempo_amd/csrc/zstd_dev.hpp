// zstd_dev.hpp — Zstandard frame decoding on the device (RFC 8878), for findOne over
// v2 data pages written with the zstd encoding (the v2 data default,
// modules/storage/config.go:39-53; reference decoder vendor/github.com/klauspost/compress/zstd,
// DecodeAll in tempodb/encoding/v2/data_reader.go:111-117).
//
// One lane decodes one page (sequential by nature: bit-serial FSE / Huffman states);
// its tables and the block's literals live in the workgroup's LDS, the output in HBM.
// Supported: any number of frames per page (skippable frames skipped), raw / RLE /
// compressed blocks, raw / RLE / Huffman (1 or 4 streams, FSE or direct weights, treeless
// reuse) literals, predefined / RLE / FSE / repeat sequence tables, repeat offsets, the
// optional content checksum (XXH64, low 32 bits, verified as DecodeAll does).
// Not supported (status TSG_E_UNSUPPORTED): dictionaries (Dictionary_ID != 0).
#pragma once
#ifndef TSG_ZSTD_HOST  // (tools/zstd_host_check.cpp builds the same decoder for the host)
#include <hip/hip_runtime.h>
#endif
#include <cstdint>

namespace tsg {
namespace zdev {

constexpr uint32_t kMaxBlock = 128 * 1024;  // Block_Maximum_Size
constexpr int kLLMax = 35, kMLMax = 52, kOFMax = 31;

__device__ __constant__ const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,   6,   7,   8,   9,    10,   11,
                                                     12, 13, 14, 15, 16, 18,  20,  22,  24,  28,   32,   40,
                                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__device__ __constant__ const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__device__ __constant__ const uint32_t kMLBase[53] = {
    3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,  18,  19,  20,  21,   22,   23,   24,   25,   26,    27,    28, 29,
    30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__device__ __constant__ const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (RFC 8878 3.1.1.3.2.2)
__device__ __constant__ const int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__device__ __constant__ const int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__device__ __constant__ const int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

__device__ __forceinline__ int hibit(uint32_t x) { return 31 - __clz(x); }  // x > 0

// ---- bit readers -----------------------------------------------------------------------
// Backward stream (FSE / Huffman bitstreams): bits are consumed from the top; bits asked
// for below the stream's first bit read as zeros (the spec's overflow rule).
struct BitsBack {
  const uint64_t *w;  // 8-byte aligned base
  int64_t start;      // absolute bit index of the stream's first bit
  int64_t pos;        // absolute bit index just above the next bit to read
  __device__ uint32_t read(int n) {
    if (n == 0) return 0;
    pos -= n;
    int64_t lo = pos;
    int k = n, under = 0;
    if (lo < start) {
      under = int(start - lo);
      if (under >= n) return 0;
      k = n - under;
      lo = start;
    }
    const uint64_t wi = uint64_t(lo) >> 6;
    const int off = int(lo & 63);
    uint64_t v = w[wi] >> off;
    if (off + k > 64) v |= w[wi + 1] << (64 - off);
    v &= (1ull << k) - 1;
    return uint32_t(v << under);
  }
  __device__ int64_t left() const { return pos - start; }  // bits not consumed (< 0: overflowed)
};
// a backward stream over [p, p + n): the marker bit (highest set bit of the last byte) is not data
__device__ __forceinline__ bool bits_back_init(BitsBack &b, const uint8_t *p, uint32_t n) {
  if (n == 0) return false;
  const uint8_t last = p[n - 1];
  if (!last) return false;
  const uint64_t a = uint64_t(p) & 7;
  b.w = reinterpret_cast<const uint64_t *>(p - a);
  b.start = int64_t(a) * 8;
  b.pos = b.start + int64_t(n - 1) * 8 + hibit(last);
  return true;
}
// forward little-endian bits (FSE table descriptions)
struct BitsFwd {
  const uint8_t *p;
  uint32_t n;    // bytes available
  uint64_t bit;  // bits consumed
  __device__ bool read(int k, uint32_t &v) {
    if (bit + uint64_t(k) > uint64_t(n) * 8) return false;
    v = 0;
    for (int i = 0; i < k; i++) {
      const uint64_t b = bit + uint64_t(i);
      v |= uint32_t((p[b >> 3] >> (b & 7)) & 1u) << i;
    }
    bit += uint64_t(k);
    return true;
  }
  __device__ uint32_t bytes_used() const { return uint32_t((bit + 7) >> 3); }
};

// ---- FSE ---------------------------------------------------------------------------------
struct Fse {  // decoding table (in LDS)
  uint8_t sym[512];
  uint8_t nb[512];
  uint16_t base[512];
  int al;  // accuracy log
};
// table from normalized counts (RFC 8878 4.1.1: symbol spreading, then states)
__device__ bool fse_build(Fse &t, const int16_t *norm, int nsym, int al, uint16_t *scratch) {
  const uint32_t size = 1u << al;
  if (al > 9 || nsym > 256) return false;
  uint32_t high = size;
  for (int s = 0; s < nsym; s++)
    if (norm[s] == -1) {
      t.sym[--high] = uint8_t(s);
      scratch[s] = 1;
    }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  uint32_t pos = 0;
  for (int s = 0; s < nsym; s++) {
    if (norm[s] <= 0) continue;
    scratch[s] = uint16_t(norm[s]);
    for (int i = 0; i < norm[s]; i++) {
      t.sym[pos] = uint8_t(s);
      do pos = (pos + step) & mask;
      while (pos >= high);
    }
  }
  if (pos != 0) return false;
  for (uint32_t i = 0; i < size; i++) {
    const uint32_t s = t.sym[i];
    const uint32_t next = scratch[s]++;
    t.nb[i] = uint8_t(al - hibit(next));
    t.base[i] = uint16_t((next << t.nb[i]) - size);
  }
  t.al = al;
  return true;
}
// FSE_Table_Description (RFC 8878 4.1.1) from a forward stream, then the table
__device__ bool fse_read(Fse &t, BitsFwd &in, int max_al, int max_sym, int16_t *norm, uint16_t *scratch) {
  uint32_t v;
  if (!in.read(4, v)) return false;
  const int al = 5 + int(v);
  if (al > max_al) return false;
  int32_t remaining = 1 << al;
  int s = 0;
  while (remaining > 0 && s <= max_sym) {
    const int bits = hibit(uint32_t(remaining + 1)) + 1;
    uint32_t val;
    if (!in.read(bits, val)) return false;
    const uint32_t lower = (1u << (bits - 1)) - 1;
    const uint32_t thr = (1u << bits) - 1 - uint32_t(remaining + 1);
    if ((val & lower) < thr) {
      in.bit -= 1;  // the short code: give the top bit back
      val &= lower;
    } else if (val > lower) {
      val -= thr;
    }
    const int16_t p = int16_t(int32_t(val) - 1);
    remaining -= p < 0 ? -p : p;
    norm[s++] = p;
    if (p == 0) {
      uint32_t rep;
      if (!in.read(2, rep)) return false;
      for (;;) {
        for (uint32_t i = 0; i < rep && s <= max_sym; i++) norm[s++] = 0;
        if (rep != 3) break;
        if (!in.read(2, rep)) return false;
      }
    }
  }
  if (remaining != 0) return false;
  in.bit = (in.bit + 7) & ~7ull;  // align to the next byte
  return fse_build(t, norm, s, al, scratch);
}
__device__ __forceinline__ void fse_rle(Fse &t, uint8_t sym) {
  t.al = 0;
  t.sym[0] = sym;
  t.nb[0] = 0;
  t.base[0] = 0;
}
__device__ __forceinline__ uint32_t fse_init(const Fse &t, BitsBack &b) { return b.read(t.al); }
__device__ __forceinline__ uint32_t fse_update(const Fse &t, uint32_t st, BitsBack &b) {
  return t.base[st] + b.read(t.nb[st]);
}

// ---- Huffman -----------------------------------------------------------------------------
struct Huf {
  uint8_t sym[2048];
  uint8_t nb[2048];
  int maxb;  // 0: no table yet
};
__device__ bool huf_from_weights(Huf &h, const uint8_t *w, int n) {
  // weights of the n transmitted symbols; the last symbol's weight is implied
  uint32_t sum = 0;
  for (int i = 0; i < n; i++) {
    if (w[i] > 12) return false;
    if (w[i]) sum += 1u << (w[i] - 1);
  }
  if (!sum) return false;
  const int maxb = hibit(sum) + 1;
  if (maxb > 11) return false;
  const uint32_t left = (1u << maxb) - sum;
  if (left & (left - 1)) return false;
  const int lastw = hibit(left) + 1;
  // bits per symbol: maxb + 1 - weight
  uint32_t count[13] = {0};
  for (int i = 0; i <= n; i++) {
    const int wt = i < n ? w[i] : lastw;
    if (wt) count[maxb + 1 - wt]++;
  }
  uint32_t idx[13];  // next table index per code length: longest codes first
  idx[maxb] = 0;
  for (int b = maxb; b >= 1; b--) idx[b - 1] = idx[b] + count[b] * (1u << (maxb - b));
  if (idx[0] != (1u << maxb)) return false;
  for (int i = 0; i <= n; i++) {
    const int wt = i < n ? w[i] : lastw;
    if (!wt) continue;
    const int b = maxb + 1 - wt;
    const uint32_t len = 1u << (maxb - b);
    for (uint32_t u = 0; u < len; u++) {
      h.sym[idx[b] + u] = uint8_t(i);
      h.nb[idx[b] + u] = uint8_t(b);
    }
    idx[b] += len;
  }
  h.maxb = maxb;
  return true;
}
// Huffman_Tree_Description (RFC 8878 4.2.1): returns the bytes it took, 0 on error
__device__ uint32_t huf_read(Huf &h, const uint8_t *p, uint32_t n, Fse &wt, int16_t *norm, uint16_t *scratch,
                             uint8_t *wbuf) {
  if (n < 1) return 0;
  const uint32_t hb = p[0];
  int nw = 0;
  if (hb >= 128) {  // direct 4-bit weights
    nw = int(hb) - 127;
    const uint32_t bytes = uint32_t(nw + 1) / 2;
    if (1 + bytes > n) return 0;
    for (int i = 0; i < nw; i++) wbuf[i] = (i & 1) ? (p[1 + i / 2] & 15) : (p[1 + i / 2] >> 4);
    if (!huf_from_weights(h, wbuf, nw)) return 0;
    return 1 + bytes;
  }
  // FSE-compressed weights: two interleaved states over one table (max accuracy 6)
  const uint32_t cs = hb;
  if (cs == 0 || 1 + cs > n) return 0;
  BitsFwd f{p + 1, cs, 0};
  if (!fse_read(wt, f, 6, 255, norm, scratch)) return 0;
  const uint32_t used = f.bytes_used();
  if (used >= cs) return 0;
  BitsBack b;
  if (!bits_back_init(b, p + 1 + used, cs - used)) return 0;
  uint32_t s1 = fse_init(wt, b), s2 = fse_init(wt, b);
  for (;;) {
    if (nw >= 255) return 0;
    wbuf[nw++] = wt.sym[s1];
    s1 = fse_update(wt, s1, b);
    if (b.left() < 0) {
      if (nw >= 255) return 0;
      wbuf[nw++] = wt.sym[s2];
      break;
    }
    if (nw >= 255) return 0;
    wbuf[nw++] = wt.sym[s2];
    s2 = fse_update(wt, s2, b);
    if (b.left() < 0) {
      if (nw >= 255) return 0;
      wbuf[nw++] = wt.sym[s1];
      break;
    }
  }
  if (!huf_from_weights(h, wbuf, nw)) return 0;
  return 1 + cs;
}
// one Huffman stream: exactly `count` symbols, every bit consumed
__device__ bool huf_stream(const Huf &h, const uint8_t *p, uint32_t n, uint8_t *out, uint32_t count) {
  BitsBack b;
  if (!bits_back_init(b, p, n)) return false;
  const uint32_t mask = (1u << h.maxb) - 1;
  uint32_t st = b.read(h.maxb);
  for (uint32_t i = 0; i < count; i++) {
    out[i] = h.sym[st];
    const int nb = h.nb[st];
    st = ((st << nb) | b.read(nb)) & mask;
  }
  return b.left() == -int64_t(h.maxb);
}

// ---- XXH64 (the frame checksum) --------------------------------------------------------------
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= uint64_t(p[i]) << (8 * i);
  return v;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ uint64_t xxh64(const uint8_t *p, uint64_t n) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                 P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  uint64_t h, i = 0;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= n; i += 32) {
      v1 = rotl64(v1 + ld64(p + i) * P2, 31) * P1;
      v2 = rotl64(v2 + ld64(p + i + 8) * P2, 31) * P1;
      v3 = rotl64(v3 + ld64(p + i + 16) * P2, 31) * P1;
      v4 = rotl64(v4 + ld64(p + i + 24) * P2, 31) * P1;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) {
      h ^= rotl64(v * P2, 31) * P1;
      h = h * P1 + P4;
    }
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) {
    h ^= rotl64(ld64(p + i) * P2, 31) * P1;
    h = rotl64(h, 27) * P1 + P4;
  }
  if (i + 4 <= n) {
    const uint64_t w = uint64_t(p[i]) | uint64_t(p[i + 1]) << 8 | uint64_t(p[i + 2]) << 16 | uint64_t(p[i + 3]) << 24;
    h ^= w * P1;
    h = rotl64(h, 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; i++) {
    h ^= uint64_t(p[i]) * P5;
    h = rotl64(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// ---- frames ---------------------------------------------------------------------------------
struct Work {  // one page's decoder state (LDS)
  uint8_t lit[kMaxBlock + 64];
  Fse ll, of, ml, wt;
  Huf huf;
  int16_t norm[256];
  uint16_t scratch[256];
  uint8_t wbuf[256];
};

// frame header: returns header bytes (0 on error); content size (or ~0 when absent),
// single segment, checksum flag
__device__ uint32_t frame_header(const uint8_t *p, uint32_t n, uint64_t &fcs, bool &csum, int &status) {
  if (n < 5) return 0;
  const uint32_t fhd = p[4];
  const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did_flag = fhd & 3;
  csum = (fhd >> 2) & 1;
  if (fhd & 8) return 0;  // reserved bit
  uint32_t o = 5;
  if (!single) o += 1;  // Window_Descriptor
  const uint32_t did_bytes = did_flag == 3 ? 4 : did_flag;
  uint64_t did = 0;
  for (uint32_t i = 0; i < did_bytes; i++) did |= uint64_t(o + i < n ? p[o + i] : 0) << (8 * i);
  o += did_bytes;
  if (did) {
    status = TSG_E_UNSUPPORTED;  // dictionaries
    return 0;
  }
  const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : (1u << fcs_flag);
  if (o + fcs_bytes > n) return 0;
  fcs = ~0ull;
  if (fcs_bytes) {
    fcs = 0;
    for (uint32_t i = 0; i < fcs_bytes; i++) fcs |= uint64_t(p[o + i]) << (8 * i);
    if (fcs_bytes == 2) fcs += 256;
  }
  return o + fcs_bytes;
}

// Upper bound (or exact size) of the decoded bytes of a zstd payload; 0 status = ok
__device__ int zstd_size(const uint8_t *p, uint32_t n, uint64_t &out) {
  out = 0;
  uint32_t s = 0;
  while (s < n) {
    if (n - s < 4) return TSG_E_CORRUPT;
    const uint32_t magic = uint32_t(p[s]) | uint32_t(p[s + 1]) << 8 | uint32_t(p[s + 2]) << 16 | uint32_t(p[s + 3]) << 24;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (n - s < 8) return TSG_E_CORRUPT;
      const uint32_t sz = uint32_t(p[s + 4]) | uint32_t(p[s + 5]) << 8 | uint32_t(p[s + 6]) << 16 | uint32_t(p[s + 7]) << 24;
      if (sz > n - s - 8) return TSG_E_CORRUPT;
      s += 8 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) return TSG_E_CORRUPT;
    uint64_t fcs;
    bool csum;
    int st = TSG_OK;
    const uint32_t h = frame_header(p + s, n - s, fcs, csum, st);
    if (!h) return st != TSG_OK ? st : TSG_E_CORRUPT;
    s += h;
    uint64_t bound = 0;
    for (;;) {
      if (n - s < 3) return TSG_E_CORRUPT;
      const uint32_t bh = uint32_t(p[s]) | uint32_t(p[s + 1]) << 8 | uint32_t(p[s + 2]) << 16;
      s += 3;
      const uint32_t type = (bh >> 1) & 3, size = bh >> 3;
      if (type == 3) return TSG_E_CORRUPT;
      const uint32_t csize = type == 1 ? 1 : size;
      if (csize > n - s) return TSG_E_CORRUPT;
      bound += type == 2 ? kMaxBlock : size;
      s += csize;
      if (bh & 1) break;
    }
    if (csum) {
      if (n - s < 4) return TSG_E_CORRUPT;
      s += 4;
    }
    out += fcs != ~0ull ? fcs : bound;
    if (out >= (1ull << 31)) return TSG_E_UNSUPPORTED;
  }
  return TSG_OK;
}

// Sequences: decode and execute (RFC 8878 3.1.1.3.2, 3.1.1.4)
__device__ int seq_table(Fse &t, int mode, const uint8_t *p, uint32_t n, uint32_t &used, const int16_t *def,
                         int defn, int defal, int max_al, int max_sym, Work &W, bool &have) {
  used = 0;
  if (mode == 0) {  // predefined
    for (int i = 0; i < defn; i++) W.norm[i] = def[i];
    if (!fse_build(t, W.norm, defn, defal, W.scratch)) return TSG_E_CORRUPT;
  } else if (mode == 1) {  // RLE
    if (n < 1 || p[0] > max_sym) return TSG_E_CORRUPT;
    fse_rle(t, p[0]);
    used = 1;
  } else if (mode == 2) {
    BitsFwd f{p, n, 0};
    if (!fse_read(t, f, max_al, max_sym, W.norm, W.scratch)) return TSG_E_CORRUPT;
    used = f.bytes_used();
  } else {  // repeat: the previous block's table of this frame
    if (!have) return TSG_E_CORRUPT;
  }
  have = true;
  return TSG_OK;
}

// One frame's blocks into out[0..cap); *written = content bytes. One lane.
struct FrameState {
  uint32_t rep[3];
  bool have_ll, have_of, have_ml;
};

__device__ int block_compressed(const uint8_t *p, uint32_t n, uint8_t *out, uint64_t &pos, uint64_t cap,
                                uint64_t frame_start, Work &W, FrameState &F) {
  // ---- literals section
  if (n < 1) return TSG_E_CORRUPT;
  const uint32_t b0 = p[0], ltype = b0 & 3, sf = (b0 >> 2) & 3;
  uint32_t regen = 0, csize = 0, hdr = 0, nstreams = 1;
  if (ltype <= 1) {
    if (sf == 0 || sf == 2) {
      regen = b0 >> 3;
      hdr = 1;
    } else if (sf == 1) {
      if (n < 2) return TSG_E_CORRUPT;
      regen = (b0 >> 4) + (uint32_t(p[1]) << 4);
      hdr = 2;
    } else {
      if (n < 3) return TSG_E_CORRUPT;
      regen = (b0 >> 4) + (uint32_t(p[1]) << 4) + (uint32_t(p[2]) << 12);
      hdr = 3;
    }
  } else {
    const uint32_t nb = sf <= 1 ? 3 : sf + 2;  // header bytes: 3, 3, 4, 5
    if (n < nb) return TSG_E_CORRUPT;
    uint64_t h = 0;
    for (uint32_t i = 0; i < nb; i++) h |= uint64_t(p[i]) << (8 * i);
    const int bits = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
    regen = uint32_t((h >> 4) & ((1ull << bits) - 1));
    csize = uint32_t((h >> (4 + bits)) & ((1ull << bits) - 1));
    nstreams = sf == 0 ? 1 : 4;
    hdr = nb;
  }
  if (regen > kMaxBlock) return TSG_E_CORRUPT;
  uint32_t o = hdr;
  if (ltype == 0) {
    if (regen > n - o) return TSG_E_CORRUPT;
    for (uint32_t i = 0; i < regen; i++) W.lit[i] = p[o + i];
    o += regen;
  } else if (ltype == 1) {
    if (n - o < 1) return TSG_E_CORRUPT;
    for (uint32_t i = 0; i < regen; i++) W.lit[i] = p[o];
    o += 1;
  } else {
    if (csize > n - o) return TSG_E_CORRUPT;
    uint32_t t = 0;
    if (ltype == 2) {
      t = huf_read(W.huf, p + o, csize, W.wt, W.norm, W.scratch, W.wbuf);
      if (!t) return TSG_E_CORRUPT;
    } else if (!W.huf.maxb) {
      return TSG_E_CORRUPT;  // treeless without a previous table
    }
    const uint8_t *sp = p + o + t;
    const uint32_t sl = csize - t;
    if (nstreams == 1) {
      if (!huf_stream(W.huf, sp, sl, W.lit, regen)) return TSG_E_CORRUPT;
    } else {
      if (sl < 6) return TSG_E_CORRUPT;
      const uint32_t l1 = uint32_t(sp[0]) | uint32_t(sp[1]) << 8, l2 = uint32_t(sp[2]) | uint32_t(sp[3]) << 8,
                     l3 = uint32_t(sp[4]) | uint32_t(sp[5]) << 8;
      if (uint64_t(l1) + l2 + l3 > sl - 6) return TSG_E_CORRUPT;
      const uint32_t l4 = sl - 6 - l1 - l2 - l3;
      const uint32_t seg = (regen + 3) / 4;
      if (regen < 3 * seg) return TSG_E_CORRUPT;
      const uint32_t last = regen - 3 * seg;
      const uint8_t *s1 = sp + 6, *s2 = s1 + l1, *s3 = s2 + l2, *s4 = s3 + l3;
      if (!huf_stream(W.huf, s1, l1, W.lit, seg) || !huf_stream(W.huf, s2, l2, W.lit + seg, seg) ||
          !huf_stream(W.huf, s3, l3, W.lit + 2 * seg, seg) || !huf_stream(W.huf, s4, l4, W.lit + 3 * seg, last))
        return TSG_E_CORRUPT;
    }
    o += csize;
  }
  // ---- sequences section
  if (o >= n) return TSG_E_CORRUPT;
  uint32_t nseq = p[o];
  if (nseq == 0) {
    o += 1;
  } else if (nseq < 128) {
    o += 1;
  } else if (nseq < 255) {
    if (n - o < 2) return TSG_E_CORRUPT;
    nseq = ((nseq - 128) << 8) + p[o + 1];
    o += 2;
  } else {
    if (n - o < 3) return TSG_E_CORRUPT;
    nseq = uint32_t(p[o + 1]) + (uint32_t(p[o + 2]) << 8) + 0x7F00;
    o += 3;
  }
  uint32_t lit_pos = 0;
  if (nseq) {
    if (n - o < 1) return TSG_E_CORRUPT;
    const uint32_t modes = p[o++];
    if (modes & 3) return TSG_E_CORRUPT;
    uint32_t used;
    int st = seq_table(W.ll, int(modes >> 6), p + o, n - o, used, kLLDef, 36, 6, 9, kLLMax, W, F.have_ll);
    if (st) return st;
    o += used;
    st = seq_table(W.of, int((modes >> 4) & 3), p + o, n - o, used, kOFDef, 29, 5, 8, kOFMax, W, F.have_of);
    if (st) return st;
    o += used;
    st = seq_table(W.ml, int((modes >> 2) & 3), p + o, n - o, used, kMLDef, 53, 6, 9, kMLMax, W, F.have_ml);
    if (st) return st;
    o += used;
    BitsBack b;
    if (o >= n || !bits_back_init(b, p + o, n - o)) return TSG_E_CORRUPT;
    uint32_t sll = fse_init(W.ll, b), sof = fse_init(W.of, b), sml = fse_init(W.ml, b);
    for (uint32_t i = 0; i < nseq; i++) {
      const uint32_t ofc = W.of.sym[sof], mlc = W.ml.sym[sml], llc = W.ll.sym[sll];
      if (ofc > 31 || mlc > kMLMax || llc > kLLMax) return TSG_E_CORRUPT;
      uint32_t ofv = (1u << ofc) + b.read(int(ofc));  // offset bits first, then match, then literal
      const uint32_t ml = kMLBase[mlc] + b.read(kMLBits[mlc]);
      const uint32_t ll = kLLBase[llc] + b.read(kLLBits[llc]);
      uint32_t off;
      if (ofv > 3) {
        off = ofv - 3;
        F.rep[2] = F.rep[1];
        F.rep[1] = F.rep[0];
        F.rep[0] = off;
      } else {
        uint32_t idx = ofv - 1 + (ll == 0 ? 1u : 0u);
        if (idx == 0) {
          off = F.rep[0];
        } else {
          off = idx < 3 ? F.rep[idx] : F.rep[0] - 1;
          if (idx > 1) F.rep[2] = F.rep[1];
          F.rep[1] = F.rep[0];
          F.rep[0] = off;
        }
      }
      if (i + 1 < nseq) {  // states: literal length, match length, offset
        sll = fse_update(W.ll, sll, b);
        sml = fse_update(W.ml, sml, b);
        sof = fse_update(W.of, sof, b);
      }
      // execute: literals, then the match
      if (ll > regen - lit_pos || uint64_t(ll) + ml > cap - pos) return TSG_E_CORRUPT;
      for (uint32_t k = 0; k < ll; k++) out[pos + k] = W.lit[lit_pos + k];
      lit_pos += ll;
      pos += ll;
      if (off == 0 || off > pos - frame_start) return TSG_E_CORRUPT;
      for (uint32_t k = 0; k < ml; k++) out[pos + k] = out[pos + k - off];
      pos += ml;
    }
    if (b.left() != 0) return TSG_E_CORRUPT;
  }
  const uint32_t rest = regen - lit_pos;
  if (rest > cap - pos) return TSG_E_CORRUPT;
  for (uint32_t k = 0; k < rest; k++) out[pos + k] = W.lit[lit_pos + k];
  pos += rest;
  return TSG_OK;
}

// the whole payload (DecodeAll): frames back to back into out[0..cap); *len = bytes written
__device__ int zstd_decode(const uint8_t *p, uint32_t n, uint8_t *out, uint64_t cap, uint64_t &len, Work &W) {
  uint64_t pos = 0;
  uint32_t s = 0;
  W.huf.maxb = 0;
  while (s < n) {
    if (n - s < 4) return TSG_E_CORRUPT;
    const uint32_t magic = uint32_t(p[s]) | uint32_t(p[s + 1]) << 8 | uint32_t(p[s + 2]) << 16 | uint32_t(p[s + 3]) << 24;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
      const uint32_t sz = uint32_t(p[s + 4]) | uint32_t(p[s + 5]) << 8 | uint32_t(p[s + 6]) << 16 | uint32_t(p[s + 7]) << 24;
      s += 8 + sz;
      continue;
    }
    uint64_t fcs;
    bool csum;
    int st = TSG_OK;
    const uint32_t h = frame_header(p + s, n - s, fcs, csum, st);
    if (!h) return st != TSG_OK ? st : TSG_E_CORRUPT;
    s += h;
    const uint64_t fstart = pos;
    FrameState F{{1, 4, 8}, false, false, false};
    W.huf.maxb = 0;
    for (;;) {
      if (n - s < 3) return TSG_E_CORRUPT;
      const uint32_t bh = uint32_t(p[s]) | uint32_t(p[s + 1]) << 8 | uint32_t(p[s + 2]) << 16;
      s += 3;
      const uint32_t type = (bh >> 1) & 3, size = bh >> 3;
      if (type == 0) {  // raw
        if (size > n - s || size > cap - pos) return TSG_E_CORRUPT;
        for (uint32_t k = 0; k < size; k++) out[pos + k] = p[s + k];
        pos += size;
        s += size;
      } else if (type == 1) {  // RLE
        if (n - s < 1 || size > cap - pos) return TSG_E_CORRUPT;
        for (uint32_t k = 0; k < size; k++) out[pos + k] = p[s];
        pos += size;
        s += 1;
      } else if (type == 2) {
        if (size > n - s || size > kMaxBlock) return TSG_E_CORRUPT;
        const int r = block_compressed(p + s, size, out, pos, cap, fstart, W, F);
        if (r) return r;
        s += size;
      } else {
        return TSG_E_CORRUPT;
      }
      if (bh & 1) break;
    }
    if (fcs != ~0ull && pos - fstart != fcs) return TSG_E_CORRUPT;
    if (csum) {
      if (n - s < 4) return TSG_E_CORRUPT;
      const uint32_t want = uint32_t(p[s]) | uint32_t(p[s + 1]) << 8 | uint32_t(p[s + 2]) << 16 | uint32_t(p[s + 3]) << 24;
      if (uint32_t(xxh64(out + fstart, pos - fstart)) != want) return TSG_E_CORRUPT;
      s += 4;
    }
  }
  len = pos;
  return TSG_OK;
}

}  // namespace zdev
}  // namespace tsg
