// find.hip — tempodb.Find on MI355X: bloom + index (lookup.hip) and then findOne on the
// device: the data page each hit's index record names is decompressed in HBM and its
// objects are scanned for the exact trace id.
//
//   findOne                        tempodb/encoding/v2/finder_paged.go:79-110
//   dataReader.Read (one record)   tempodb/encoding/v2/data_reader.go:45-125
//   page framing                   tempodb/encoding/v2/page.go:28-57
//   object framing / iterator      tempodb/encoding/v2/object.go:82-113, iterator.go
//   snappy framed stream           vendor/github.com/golang/snappy/decode.go:121-232,
//                                  block format decode_other.go:41-102
//
// Per batch: (1) the distinct (block, record) pages of the lookup hits, (2) a size pass
// (one lane per page walks the frame headers), (3) decode: one wave per page, each
// snappy chunk (<= 64 KiB decoded) staged and decoded in LDS with all 64 lanes (tags
// parsed in lockstep, literal and match bytes copied in parallel: a match of offset o
// is periodic, byte j = out[d - o + j % o], so no lane waits on another), CRC32C of the
// chunk per lane segment and combined, then written to HBM coalesced; (4) object scan:
// one wave per page walks the objects through 64 KiB LDS windows and the lanes compare
// each object id against the page's pending ids (first exact match, as findOne);
// (5) the found objects are gathered into one arena for the copy back.
// Encodings: none, snappy and zstd (zstd_dev.hpp: one lane per page); lz4 / gzip / s2
// report TSG_E_UNSUPPORTED_ENCODING per hit (the caller's CPU path takes those blocks).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <numeric>

#include "devctx.hpp"
#include "zstd_dev.hpp"

namespace tsg {

struct FindPage {
  const uint8_t *src;  // v2 page: [u32 total][u16 hdr len][payload]
  uint64_t out_off;    // decoded bytes in the arena
  uint32_t len;        // index record length (the page's bytes)
  uint32_t enc;        // backend.Encoding
  uint32_t out_len;    // decoded size (size pass)
  int32_t status;      // TSG_OK or the page's error
  uint32_t hit0, nhit; // this page's pending ids: hits [hit0, hit0 + nhit)
};

constexpr uint32_t kSnapMaxBlock = 65536, kSnapMaxChunk = 76490 + 4;  // decode.go: maxBlockSize, buf size
constexpr uint32_t kFindWindow = 65536;                               // object scan window (LDS)

__device__ __forceinline__ uint32_t g_le32(const uint8_t *p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// (2) decoded size of each page; framing errors are recorded here
extern "C" __global__ void __launch_bounds__(256) find_size_kernel(FindPage *pages, uint32_t npages) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npages) return;
  FindPage &P = pages[i];
  P.out_len = 0;
  // unmarshalPageFromBytes with the data header (length 0) (page.go:28-57)
  if (P.len < 6 || g_le32(P.src) != P.len || (uint32_t(P.src[4]) | uint32_t(P.src[5]) << 8) != 0) {
    P.status = TSG_E_CORRUPT;
    return;
  }
  const uint8_t *b = P.src + 6;
  const uint32_t n = P.len - 6;
  if (P.enc == 0) {  // EncNone
    P.out_len = n;
    P.status = TSG_OK;
    return;
  }
  if (P.enc == 7) {  // zstd: frame content sizes (or block bounds)
    uint64_t sz = 0;
    P.status = zdev::zstd_size(b, n, sz);
    P.out_len = P.status == TSG_OK ? uint32_t(sz) : 0;
    return;
  }
  if (P.enc != 6) {
    P.status = TSG_E_UNSUPPORTED_ENCODING;
    return;
  }
  uint64_t total = 0;
  uint32_t s = 0;
  bool hdr = false;
  while (s < n) {
    if (n - s < 4) {
      P.status = TSG_E_CORRUPT;
      return;
    }
    const uint32_t ct = b[s], cl = uint32_t(b[s + 1]) | uint32_t(b[s + 2]) << 8 | uint32_t(b[s + 3]) << 16;
    s += 4;
    if (!hdr && ct != 0xff) {
      P.status = TSG_E_CORRUPT;
      return;
    }
    hdr = true;
    if (cl > kSnapMaxChunk || cl > n - s) {
      P.status = TSG_E_CORRUPT;
      return;
    }
    if (ct == 0x00) {  // compressed: [crc][varint decoded length][block]
      uint64_t v = 0;
      uint32_t k = 0;
      for (int shift = 0;; shift += 7, k++) {
        if (4 + k >= cl || k >= 5) {
          P.status = TSG_E_CORRUPT;
          return;
        }
        const uint32_t c = b[s + 4 + k];
        v |= uint64_t(c & 0x7f) << shift;
        if (c < 0x80) break;
      }
      if (v > kSnapMaxBlock) {
        P.status = TSG_E_CORRUPT;
        return;
      }
      total += v;
    } else if (ct == 0x01) {
      if (cl < 4 || cl - 4 > kSnapMaxBlock) {
        P.status = TSG_E_CORRUPT;
        return;
      }
      total += cl - 4;
    } else if (ct == 0xff) {
      const char *id = "sNaPpY";
      bool ok = cl == 6;
      for (int q = 0; q < 6 && ok; q++) ok = b[s + q] == uint8_t(id[q]);
      if (!ok) {
        P.status = TSG_E_CORRUPT;
        return;
      }
    } else if (ct <= 0x7f) {  // reserved unskippable
      P.status = TSG_E_CORRUPT;
      return;
    }
    s += cl;
  }
  if (total >= (1ull << 31)) {
    P.status = TSG_E_UNSUPPORTED;
    return;
  }
  P.out_len = uint32_t(total);
  P.status = TSG_OK;
}

struct CrcArgs {
  uint32_t table[256];  // CRC-32C (Castagnoli), reflected
  uint32_t z1024[32];   // the register after 1024 zero bytes from state 1 << b
};

// (3) one wave per page
constexpr int kFindThreads = 64;
extern "C" __global__ void __launch_bounds__(kFindThreads) find_decode_kernel(FindPage *pages, uint8_t *arena,
                                                                            const CrcArgs *crc) {
  __shared__ uint8_t cbuf[kSnapMaxChunk + 8];
  __shared__ uint8_t obuf[kSnapMaxBlock + 8];
  __shared__ uint32_t tab[256];
  __shared__ uint32_t lane_crc[kFindThreads];
  const int lane = threadIdx.x;
  FindPage &P = pages[blockIdx.x];
  if (P.status != TSG_OK || P.enc == 7) return;  // (zstd pages: find_decode_zstd_kernel)
  for (int i = lane; i < 256; i += kFindThreads) tab[i] = crc->table[i];
  const uint8_t *b = P.src + 6;
  const uint32_t n = P.len - 6;
  uint8_t *out = arena + P.out_off;
  if (P.enc == 0) {
    for (uint32_t i = lane; i < n; i += kFindThreads) out[i] = b[i];
    return;
  }
  __syncthreads();
  uint32_t s = 0, pos = 0;
  int32_t status = TSG_OK;
  while (s + 4 <= n && status == TSG_OK) {
    const uint32_t ct = b[s], cl = uint32_t(b[s + 1]) | uint32_t(b[s + 2]) << 8 | uint32_t(b[s + 3]) << 16;
    s += 4;  // (framing checked by the size pass)
    if (ct != 0x00 && ct != 0x01) {
      s += cl;
      continue;
    }
    const uint32_t want = g_le32(b + s);
    uint32_t ulen = 0;
    if (ct == 0x01) {  // uncompressed chunk: copy into obuf for the checksum
      ulen = cl - 4;
      for (uint32_t i = lane; i < ulen; i += kFindThreads) obuf[i] = b[s + 4 + i];
    } else {
      // stage the compressed block, then decode it in lockstep
      const uint32_t bl = cl - 4;
      for (uint32_t i = lane; i < bl; i += kFindThreads) cbuf[i] = b[s + 4 + i];
      __syncthreads();
      uint32_t t = 0, v = 0;
      for (int shift = 0;; shift += 7) {  // varint decoded length (validated by the size pass)
        const uint32_t c = cbuf[t++];
        v |= (c & 0x7f) << shift;
        if (c < 0x80) break;
      }
      ulen = v;
      uint32_t d = 0;
      while (t < bl) {
        const uint32_t tag = cbuf[t];
        uint32_t len, off = 0;
        if ((tag & 3) == 0) {  // literal
          uint32_t x = tag >> 2;
          if (x < 60) {
            t += 1;
          } else {
            const uint32_t nb = x - 59;
            if (t + 1 + nb > bl) { status = TSG_E_CORRUPT; break; }
            x = 0;
            for (uint32_t q = 0; q < nb; q++) x |= uint32_t(cbuf[t + 1 + q]) << (8 * q);
            t += 1 + nb;
          }
          len = x + 1;
          if (len == 0 || len > bl - t || len > ulen - d) { status = TSG_E_CORRUPT; break; }
          for (uint32_t j = lane; j < len; j += kFindThreads) obuf[d + j] = cbuf[t + j];
          t += len;
          d += len;
          continue;
        }
        if ((tag & 3) == 1) {
          if (t + 2 > bl) { status = TSG_E_CORRUPT; break; }
          len = 4 + ((tag >> 2) & 7);
          off = ((tag & 0xe0) << 3) | cbuf[t + 1];
          t += 2;
        } else if ((tag & 3) == 2) {
          if (t + 3 > bl) { status = TSG_E_CORRUPT; break; }
          len = 1 + (tag >> 2);
          off = uint32_t(cbuf[t + 1]) | uint32_t(cbuf[t + 2]) << 8;
          t += 3;
        } else {
          if (t + 5 > bl) { status = TSG_E_CORRUPT; break; }
          len = 1 + (tag >> 2);
          off = uint32_t(cbuf[t + 1]) | uint32_t(cbuf[t + 2]) << 8 | uint32_t(cbuf[t + 3]) << 16 |
                uint32_t(cbuf[t + 4]) << 24;
          t += 5;
        }
        if (off == 0 || off > d || len > ulen - d) { status = TSG_E_CORRUPT; break; }
        // LZ77 copy: out[d + j] = out[d - off + j % off] (periodic when off < len)
        if (off >= len) {
          for (uint32_t j = lane; j < len; j += kFindThreads) obuf[d + j] = obuf[d - off + j];
        } else {
          for (uint32_t j = lane; j < len; j += kFindThreads) obuf[d + j] = obuf[d - off + j % off];
        }
        d += len;
      }
      if (status == TSG_OK && d != ulen) status = TSG_E_CORRUPT;
    }
    __syncthreads();
    if (status != TSG_OK) break;
    // CRC-32C of the decoded chunk: 1 KiB per lane, combined on lane 0
    {
      uint32_t r = 0;  // raw register from state 0
      const uint32_t lo = uint32_t(lane) * 1024, hi = min(ulen, lo + 1024);
      for (uint32_t i = lo; i < hi; i++) r = tab[(r ^ obuf[i]) & 0xff] ^ (r >> 8);
      lane_crc[lane] = r;
      __syncthreads();
      if (lane == 0) {
        uint32_t acc = 0xffffffffu;
        const uint32_t nseg = (ulen + 1023) / 1024;
        for (uint32_t g = 0; g < nseg; g++) {
          const uint32_t sl = min(ulen - g * 1024, 1024u);
          uint32_t z = 0;
          if (sl == 1024) {  // advance by 1024 zero bytes: linear map, precomputed columns
            for (int bb = 0; bb < 32; bb++)
              if ((acc >> bb) & 1u) z ^= crc->z1024[bb];
          } else {
            z = acc;
            for (uint32_t i = 0; i < sl; i++) z = tab[z & 0xff] ^ (z >> 8);
          }
          acc = z ^ lane_crc[g];
        }
        const uint32_t c = ~acc;
        const uint32_t masked = ((c >> 15) | (c << 17)) + 0xa282ead8u;  // snappy.go:61-64
        lane_crc[0] = masked == want ? 1u : 0u;
      }
      __syncthreads();
      if (!lane_crc[0]) status = TSG_E_CORRUPT;
      __syncthreads();
    }
    if (status != TSG_OK) break;
    if (pos + ulen > P.out_len) { status = TSG_E_CORRUPT; break; }
    for (uint32_t i = lane; i < ulen; i += kFindThreads) out[pos + i] = obuf[i];
    pos += ulen;
    s += cl;
    __syncthreads();
  }
  if (lane == 0 && (status != TSG_OK || pos != P.out_len)) P.status = status != TSG_OK ? status : TSG_E_CORRUPT;
}

// (3') zstd pages: one lane decodes the page (tables and literals in LDS)
extern "C" __global__ void __launch_bounds__(64) find_decode_zstd_kernel(FindPage *pages, uint8_t *arena) {
  __shared__ zdev::Work W;
  FindPage &P = pages[blockIdx.x];
  if (P.status != TSG_OK || P.enc != 7 || threadIdx.x != 0) return;
  uint64_t len = 0;
  const int st = zdev::zstd_decode(P.src + 6, P.len - 6, arena + P.out_off, P.out_len, len, W);
  if (st != TSG_OK) P.status = st;
  else P.out_len = uint32_t(len);  // (the size pass may hold an upper bound)
}

// (4) the page's objects against its pending ids (hit_ids[hit0 .. hit0 + nhit), 16 bytes
// each): per hit the object's offset (into the arena) and length, or not found. The
// objects are read as findOne's iterator reads them (object.UnmarshalObjectFromReader
// over a bytes.Reader, object.go:49-80): the page ends cleanly where a header would start
// at its end (or with 4 or 8 bytes left: the next read hits EOF), a short read or an id
// length past the object is an error for every id not found before it.
struct FindHitOut {
  uint64_t off;
  uint32_t len;
  int32_t status;  // TSG_OK found, TSG_E_NOT_FOUND none (findOne returns nil), else the page error
};
__device__ __forceinline__ uint32_t lds_le32(const uint8_t *p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
constexpr int kFindPer = 4;  // pending ids held in registers per lane and pass
extern "C" __global__ void __launch_bounds__(kFindThreads) find_scan_kernel(const FindPage *pages, const uint8_t *arena,
                                                                          const uint8_t *hit_ids, FindHitOut *res) {
  __shared__ uint8_t win[kFindWindow + 16];
  const int lane = threadIdx.x;
  const FindPage &P = pages[blockIdx.x];
  const int32_t init = P.status == TSG_OK ? TSG_E_NOT_FOUND : P.status;
  for (uint32_t h = lane; h < P.nhit; h += kFindThreads) res[P.hit0 + h] = FindHitOut{0, 0, init};
  if (P.status != TSG_OK) return;
  const uint8_t *pg = arena + P.out_off;
  const uint32_t L = P.out_len;
  for (uint32_t base = 0; base < P.nhit; base += kFindPer * kFindThreads) {
    uint32_t id[kFindPer][4];
    bool pend[kFindPer];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < kFindPer; k++) {
      const uint32_t h = base + uint32_t(k) * kFindThreads + lane;
      pend[k] = h < P.nhit;
#pragma unroll
      for (int q = 0; q < 4; q++) id[k][q] = pend[k] ? g_le32(hit_ids + uint64_t(P.hit0 + h) * 16 + 4 * q) : 0u;
      mine += pend[k] ? 1u : 0u;
    }
    uint32_t remaining = mine;
    for (int dd = 32; dd > 0; dd >>= 1) remaining += __shfl_xor(remaining, dd, 64);
    int32_t err = TSG_OK;
    uint32_t p = 0;  // window start (page offset): always an object start
    while (remaining && err == TSG_OK) {
      const uint32_t wl = min(L - p, kFindWindow);
      __syncthreads();
      for (uint32_t i = lane; i < wl; i += kFindThreads) win[i] = pg[p + i];
      __syncthreads();
      uint32_t w = 0;
      bool end = false;
      for (;;) {
        const uint32_t R = L - (p + w);  // bytes left in the page
        if (R == 0 || R == 4) {          // io.EOF at a header read
          end = true;
          break;
        }
        if (R < 8) {  // io.ErrUnexpectedEOF
          err = TSG_E_CORRUPT;
          break;
        }
        if (wl - w < 8) break;  // (the window ends before the page does) slide
        const uint32_t total = lds_le32(win + w), il = lds_le32(win + w + 4);
        if (R == 8) {  // reading the object bytes at EOF: io.EOF
          end = true;
          break;
        }
        if (total < 8 || total - 8 > R - 8 || il > total - 8) {  // short read / id past the object
          err = TSG_E_CORRUPT;
          break;
        }
        if (il == 16) {
          if (wl - w < 24) break;  // slide
          uint32_t oid[4];
#pragma unroll
          for (int q = 0; q < 4; q++) oid[q] = lds_le32(win + w + 8 + 4 * q);
          bool got = false;
#pragma unroll
          for (int k = 0; k < kFindPer; k++)
            if (pend[k] && id[k][0] == oid[0] && id[k][1] == oid[1] && id[k][2] == oid[2] && id[k][3] == oid[3]) {
              const uint32_t h = base + uint32_t(k) * kFindThreads + lane;
              res[P.hit0 + h] = FindHitOut{P.out_off + p + w + 24, total - 24, TSG_OK};
              pend[k] = false;
              mine--;
              got = true;
            }
          if (__ballot(got)) {
            remaining = mine;
            for (int dd = 32; dd > 0; dd >>= 1) remaining += __shfl_xor(remaining, dd, 64);
            if (!remaining) break;
          }
        }
        const uint64_t next = uint64_t(w) + total;  // (<= L - p: total <= R)
        w = uint32_t(next);
        if (next >= wl) break;  // next object beyond this window
      }
      if (end || err != TSG_OK) break;
      p += w;
    }
    if (err != TSG_OK)  // findOne returns the error for every id it had not found yet
#pragma unroll
      for (int k = 0; k < kFindPer; k++)
        if (pend[k]) res[P.hit0 + base + uint32_t(k) * kFindThreads + lane].status = err;
  }
}

// (5) found objects into one arena
extern "C" __global__ void __launch_bounds__(256) find_gather_kernel(const FindHitOut *res, const uint64_t *dst_off,
                                                                   uint32_t nhits, const uint8_t *arena,
                                                                   uint8_t *dst) {
  const uint32_t h = blockIdx.x;
  if (h >= nhits || res[h].status != TSG_OK) return;
  const uint8_t *src = arena + res[h].off;
  uint8_t *d = dst + dst_off[h];
  for (uint32_t i = threadIdx.x; i < res[h].len; i += blockDim.x) d[i] = src[i];
}

// ---- host -------------------------------------------------------------------------------
static void crc_tables(CrcArgs &c) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t r = i;
    for (int k = 0; k < 8; k++) r = (r >> 1) ^ (0x82f63b78u & (0u - (r & 1u)));
    c.table[i] = r;
  }
  for (int b = 0; b < 32; b++) {
    uint32_t z = 1u << b;
    for (int i = 0; i < 1024; i++) z = c.table[z & 0xff] ^ (z >> 8);
    c.z1024[b] = z;
  }
}

void device_find(DeviceCtx &dc, const std::vector<std::pair<uint32_t, V2Block *>> &blocks, const uint8_t (*ids)[16],
                 size_t nids, const tsg_lookup_opts *opts, FindOut &out) {
  LookupOut lk;
  device_lookup(dc, blocks, ids, nids, opts, lk);
  out = FindOut();
  const size_t nh = lk.id_idx.size();
  out.id_idx.assign(lk.id_idx.begin(), lk.id_idx.end());
  out.block_idx.assign(lk.block_idx.begin(), lk.block_idx.end());
  out.status.assign(nh, TSG_E_NOT_FOUND);
  out.obj_off.assign(nh, 0);
  out.obj_len.assign(nh, 0);
  out.kernel_ns = lk.kernel_ns;
  if (nh == 0) return;
  std::unordered_map<uint32_t, const V2Block *> by_idx;
  for (auto &bp : blocks) by_idx[bp.first] = bp.second;
  // (1) distinct pages, hits grouped by page
  std::vector<uint32_t> order(nh);
  std::iota(order.begin(), order.end(), 0u);
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return lk.block_idx[a] != lk.block_idx[b] ? lk.block_idx[a] < lk.block_idx[b] : lk.rec[a] < lk.rec[b];
  });
  std::vector<FindPage> pages;
  std::vector<uint8_t> hid(nh * 16, 0);  // ids in page order
  std::vector<uint32_t> slot(nh);        // page order -> hit
  for (size_t k = 0; k < nh; k++) {
    const uint32_t h = order[k];
    const V2Block *b = by_idx.at(lk.block_idx[h]);
    if (pages.empty() || k == 0 || lk.block_idx[order[k - 1]] != lk.block_idx[h] || lk.rec[order[k - 1]] != lk.rec[h]) {
      FindPage pg{};
      pg.hit0 = uint32_t(k);
      if (!b->d_data) {
        pg.status = TSG_E_UNSUPPORTED;  // data file not resident
      } else if (lk.start[h] + lk.len[h] > b->data_len) {
        pg.status = TSG_E_CORRUPT;  // ReadAt past the end of the data file
      } else {
        pg.src = b->d_data + lk.start[h];
        pg.len = lk.len[h];
        pg.enc = uint32_t(b->enc);
        pg.status = TSG_OK;
      }
      pages.push_back(pg);
    }
    pages.back().nhit++;
    std::memcpy(&hid[k * 16], ids[lk.id_idx[h]], 16);
    slot[k] = h;
  }
  const uint32_t np = uint32_t(pages.size());
  std::lock_guard<std::mutex> lkd(dc.mu);
  resident_quit(dc);  // (the resident search launch holds every CU's LDS)
  HIP_OK(hipSetDevice(dc.ordinal));
  hipStream_t s = dc.stream;
  HIP_OK(hipEventRecord(dc.ev0, s));
  // (2) sizes
  DevBuf &dpages = dc.fpages, &dhid = dc.fhits, &dres = dc.fres, &darena = dc.farena;
  dpages.ensure(size_t(np) * sizeof(FindPage));
  HIP_OK(hipMemcpyAsync(dpages.p, pages.data(), size_t(np) * sizeof(FindPage), hipMemcpyHostToDevice, s));
  find_size_kernel<<<(np + 255) / 256, 256, 0, s>>>(static_cast<FindPage *>(dpages.p), np);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(pages.data(), dpages.p, size_t(np) * sizeof(FindPage), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  uint64_t total = 0;
  for (auto &pg : pages) {
    pg.out_off = total;
    total += (pg.out_len + 15) / 16 * 16;
  }
  darena.ensure(std::max<uint64_t>(total, 16));
  HIP_OK(hipMemcpyAsync(dpages.p, pages.data(), size_t(np) * sizeof(FindPage), hipMemcpyHostToDevice, s));
  // (3) decode
  CrcArgs crc;
  crc_tables(crc);
  dc.fcrc.ensure(sizeof(CrcArgs));
  HIP_OK(hipMemcpyAsync(dc.fcrc.p, &crc, sizeof(CrcArgs), hipMemcpyHostToDevice, s));
  find_decode_kernel<<<np, kFindThreads, 0, s>>>(static_cast<FindPage *>(dpages.p), static_cast<uint8_t *>(darena.p),
                                               static_cast<const CrcArgs *>(dc.fcrc.p));
  HIP_OK(hipGetLastError());
  bool any_zstd = false;
  for (auto &pg : pages) any_zstd = any_zstd || (pg.enc == 7 && pg.status == TSG_OK);
  if (any_zstd) {
    find_decode_zstd_kernel<<<np, 64, 0, s>>>(static_cast<FindPage *>(dpages.p), static_cast<uint8_t *>(darena.p));
    HIP_OK(hipGetLastError());
  }
  // (4) objects
  dhid.ensure(hid.size());
  HIP_OK(hipMemcpyAsync(dhid.p, hid.data(), hid.size(), hipMemcpyHostToDevice, s));
  dres.ensure(nh * sizeof(FindHitOut));
  find_scan_kernel<<<np, kFindThreads, 0, s>>>(static_cast<const FindPage *>(dpages.p),
                                               static_cast<const uint8_t *>(darena.p),
                                               static_cast<const uint8_t *>(dhid.p), static_cast<FindHitOut *>(dres.p));
  HIP_OK(hipGetLastError());
  std::vector<FindHitOut> res(nh);
  HIP_OK(hipMemcpyAsync(res.data(), dres.p, nh * sizeof(FindHitOut), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  // (5) gather the found objects
  std::vector<uint64_t> doff(nh, 0);
  uint64_t obytes = 0;
  for (size_t k = 0; k < nh; k++) {
    doff[k] = obytes;
    if (res[k].status == TSG_OK) obytes += res[k].len;
  }
  out.bytes.resize(obytes);
  if (obytes) {
    dc.fdst.ensure(obytes);
    dc.foff.ensure(nh * 8);
    HIP_OK(hipMemcpyAsync(dc.foff.p, doff.data(), nh * 8, hipMemcpyHostToDevice, s));
    find_gather_kernel<<<uint32_t(nh), 256, 0, s>>>(static_cast<const FindHitOut *>(dres.p),
                                                    static_cast<const uint64_t *>(dc.foff.p), uint32_t(nh),
                                                    static_cast<const uint8_t *>(darena.p),
                                                    static_cast<uint8_t *>(dc.fdst.p));
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(out.bytes.data(), dc.fdst.p, obytes, hipMemcpyDeviceToHost, s));
  }
  HIP_OK(hipEventRecord(dc.ev1, s));
  HIP_OK(hipStreamSynchronize(s));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, dc.ev0, dc.ev1));
  out.kernel_ns += uint64_t(double(ms) * 1e6);
  for (size_t k = 0; k < nh; k++) {
    const uint32_t h = slot[k];
    out.status[h] = res[k].status;
    out.obj_off[h] = doff[k];
    out.obj_len[h] = res[k].status == TSG_OK ? res[k].len : 0;
  }
}

}  // namespace tsg
