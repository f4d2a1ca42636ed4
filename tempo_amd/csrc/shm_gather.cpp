// shm_gather.cpp — the frontend merge for ranks on one node through shared memory (VERDICT r5
// "What's missing" 2). A query over blocks sharded across the node's GPU ranks ends in rank 0
// merging every rank's ordered match list (modules/frontend/searchsharding.go:88-124, shouldQuit
// + the response merge). Ranks of one node share the host: each writes its packed response
// (tsg_result_pack's wire) into its own slot of a shared mapping and publishes the query's
// sequence number; rank 0 waits for every rank's number and merges the slots in place
// (tsg_wire_merge over pointers into the mapping: nothing is copied). Over a gloo group the same
// gather took three TCP collectives, 472 us per query for ~500 records per rank
// (profiles/r05_share2).
//
// Layout: a 4 KiB header — per rank a 64-byte line {put_seq u32 futex word, pad} and one line
// {done_seq u32 futex word} rank 0 advances after each merge — then per rank two slots (double
// buffered by seq & 1) of [u64 length | bytes]. A rank puts query s into slot s & 1 once
// done_seq >= s - 2 (rank 0 has merged the query that used it last); rank 0 merges query s once
// every put_seq >= s. Waits: a bounded spin, then a futex on the shared word (shared, not
// private: the ranks are processes), bounded by a timeout (TSG_E_DEVICE, "no response").
#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "tsg.h"

namespace tsg {
void set_last_error(const std::string &m);
}

struct tsg_shm {
  int fd = -1;
  uint8_t *base = nullptr;
  size_t bytes = 0;
  uint32_t world = 0, rank = 0;
  uint64_t slot_bytes = 0;
  std::string path;
  bool owner = false;
};

namespace {
constexpr size_t kHdr = 4096, kLine = 64;

std::atomic<uint32_t> *put_word(tsg_shm *s, uint32_t r) {
  return reinterpret_cast<std::atomic<uint32_t> *>(s->base + size_t(r) * kLine);
}
std::atomic<uint32_t> *done_word(tsg_shm *s) {
  return reinterpret_cast<std::atomic<uint32_t> *>(s->base + kHdr - kLine);
}
uint8_t *slot(tsg_shm *s, uint32_t r, uint32_t seq) {
  return s->base + kHdr + (size_t(r) * 2 + (seq & 1u)) * (s->slot_bytes + 8);
}
void futex_wait(std::atomic<uint32_t> *w, uint32_t v, int64_t ns) {
  timespec ts{time_t(ns / 1000000000), long(ns % 1000000000)};
  syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAIT, v, &ts, nullptr, 0);
}
void futex_wake(std::atomic<uint32_t> *w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}
// until (int32)(word - target) >= 0 (sequence numbers wrap): spin ~20 us, then park
bool wait_ge(std::atomic<uint32_t> *w, uint32_t target, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; it++) {
    const uint32_t v = w->load(std::memory_order_acquire);
    if (int32_t(v - target) >= 0) return true;
    if (it < 4000) {
      __builtin_ia32_pause();
      continue;
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return false;
    futex_wait(w, v, 1000000);  // (1 ms: a missed wake costs at most that)
  }
}
template <class F>
int guard_shm(F &&f) {
  try {
    f();
    return TSG_OK;
  } catch (const tsg::Error &e) {
    tsg::set_last_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    tsg::set_last_error(e.what());
    return TSG_E_INVALID;
  }
}
}  // namespace

extern "C" {

int tsg_shm_open(const char *name, uint32_t world, uint32_t rank, uint64_t slot_bytes, int reset, tsg_shm **out) {
  if (!name || !out || !world || rank >= world || world > kHdr / kLine - 1 || !slot_bytes) return TSG_E_INVALID;
  return guard_shm([&] {
    auto *s = new tsg_shm();
    s->world = world;
    s->rank = rank;
    s->slot_bytes = (slot_bytes + 7) / 8 * 8;
    s->bytes = kHdr + size_t(world) * 2 * (s->slot_bytes + 8);
    s->path = std::string("/dev/shm/") + name;
    s->fd = open(s->path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (s->fd < 0) {
      delete s;
      tsg::fail(TSG_E_IO, "tsg_shm_open: cannot open /dev/shm/" + std::string(name));
    }
    struct stat st;
    if (reset && ftruncate(s->fd, 0) != 0) {  // (a file left by an earlier run: every word back to 0)
      close(s->fd);
      delete s;
      tsg::fail(TSG_E_IO, "tsg_shm_open: cannot reset the mapping");
    }
    if (fstat(s->fd, &st) != 0 || (size_t(st.st_size) < s->bytes && ftruncate(s->fd, off_t(s->bytes)) != 0)) {
      close(s->fd);
      delete s;
      tsg::fail(TSG_E_IO, "tsg_shm_open: cannot size the mapping");
    }
    void *m = mmap(nullptr, s->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, s->fd, 0);
    if (m == MAP_FAILED) {
      close(s->fd);
      delete s;
      tsg::fail(TSG_E_IO, "tsg_shm_open: mmap failed");
    }
    s->base = static_cast<uint8_t *>(m);
    s->owner = rank == 0;
    *out = s;
  });
}

void tsg_shm_close(tsg_shm *s) {
  if (!s) return;
  if (s->base) munmap(s->base, s->bytes);
  if (s->fd >= 0) close(s->fd);
  if (s->owner) unlink(s->path.c_str());  // (the others hold their mappings: the file goes with the last)
  delete s;
}

int tsg_shm_put(tsg_shm *s, uint32_t seq, const uint8_t *wire, size_t len, double timeout_s) {
  if (!s || (len && !wire) || !seq) return TSG_E_INVALID;
  return guard_shm([&] {
    if (len > s->slot_bytes) tsg::fail(TSG_E_INVALID, "tsg_shm_put: response larger than the slot");
    if (seq > 2 && !wait_ge(done_word(s), seq - 2, timeout_s))
      tsg::fail(TSG_E_DEVICE, "tsg_shm_put: rank 0 did not merge the query that last used this slot");
    uint8_t *p = slot(s, s->rank, seq);
    const uint64_t l = len;
    std::memcpy(p, &l, 8);
    if (len) std::memcpy(p + 8, wire, len);
    put_word(s, s->rank)->store(seq, std::memory_order_release);
    futex_wake(put_word(s, s->rank));
  });
}

int tsg_shm_merge(tsg_shm *s, uint32_t seq, uint64_t limit, uint64_t total_blocks, uint8_t *out, size_t cap,
                  size_t *out_len, double timeout_s) {
  if (!s || !out_len || s->rank != 0 || !seq) return TSG_E_INVALID;
  return guard_shm([&] {
    std::vector<const uint8_t *> wires(s->world);
    std::vector<size_t> lens(s->world);
    for (uint32_t r = 0; r < s->world; r++) {
      if (!wait_ge(put_word(s, r), seq, timeout_s))
        tsg::fail(TSG_E_DEVICE, "tsg_shm_merge: no response from rank " + std::to_string(r));
      const uint8_t *p = slot(s, r, seq);
      uint64_t l = 0;
      std::memcpy(&l, p, 8);
      if (l > s->slot_bytes) tsg::fail(TSG_E_CORRUPT, "tsg_shm_merge: slot length out of range");
      wires[r] = p + 8;
      lens[r] = size_t(l);
    }
    const int rc = tsg_wire_merge(wires.data(), lens.data(), s->world, limit, total_blocks, out, cap, out_len);
    // (a size query, cap 0, keeps the slots: the caller merges again with a buffer)
    if (rc == TSG_OK && cap) {
      done_word(s)->store(seq, std::memory_order_release);
      futex_wake(done_word(s));
    }
    if (rc) tsg::fail(rc, tsg_last_error());
  });
}

}  // extern "C"
