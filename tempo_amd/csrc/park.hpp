// park.hpp — host-side waiting that never outstays a short spin: every waiter of libtsg (and
// of the shim-pattern driver) spins for a bounded few microseconds, then parks on a futex.
//
// Why ("What's weak" 1): a search's leader thread does the real work — the launch,
// the poll of the workgroup counts, the result assembly — while the other callers of a
// coalesced batch wait. Waiters that spin without a bound, on a host with fewer free CPUs than
// spinning threads, keep the leader (or a caller that must copy out its records) off a CPU
// until the scheduler's next tick: the shim's limit-20 query took 10 ms, 20 ms, 50 ms in
// whole ticks. A parked thread costs the CPU nothing; the wake-up (FUTEX_WAKE) costs the
// waker ~1 µs and the woken thread its scheduling latency.
#pragma once
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdint>

namespace tsg {

// returns false when the wait ended by its timeout
inline bool futex_wait_u32(std::atomic<uint32_t> *a, uint32_t expected, int64_t timeout_ns = -1) {
  static_assert(sizeof(std::atomic<uint32_t>) == 4, "futex word");
  struct timespec ts, *tp = nullptr;
  if (timeout_ns >= 0) {
    ts.tv_sec = time_t(timeout_ns / 1000000000);
    ts.tv_nsec = long(timeout_ns % 1000000000);
    tp = &ts;
  }
  return !(syscall(SYS_futex, reinterpret_cast<uint32_t *>(a), FUTEX_WAIT_PRIVATE, expected, tp, nullptr, 0) == -1 &&
           errno == ETIMEDOUT);
}
inline void futex_wake_u32(std::atomic<uint32_t> *a, int n = INT_MAX) {
  syscall(SYS_futex, reinterpret_cast<uint32_t *>(a), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
}

// Bounded spin: `ready()` polled with pause for at most `spin_ns`, yielding the CPU every 64
// polls (a runnable thread queued on this CPU — e.g. the leader — gets it back at once).
template <class Ready>
inline bool spin_for(uint64_t spin_ns, Ready &&ready) {
  if (ready()) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t n = 1;; n++) {
    __builtin_ia32_pause();
    if (ready()) return true;
    if ((n & 63u) == 0) {
      if (uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                       .count()) >= spin_ns)
        return false;
      sched_yield();
    }
  }
}

// A mutex for short critical sections: a bounded spin, then the futex (0 free, 1 held,
// 2 held with parked waiters; the classic three-state futex lock).
struct ParkLock {
  std::atomic<uint32_t> s{0};
  void lock() {
    uint32_t c = 0;
    if (s.compare_exchange_strong(c, 1, std::memory_order_acquire)) return;
    for (int i = 0; i < 256; i++) {
      __builtin_ia32_pause();
      c = 0;
      if (s.load(std::memory_order_relaxed) == 0 && s.compare_exchange_strong(c, 1, std::memory_order_acquire)) return;
    }
    if (c != 2) c = s.exchange(2, std::memory_order_acquire);
    while (c != 0) {
      futex_wait_u32(&s, 2);
      c = s.exchange(2, std::memory_order_acquire);
    }
  }
  void unlock() {
    if (s.exchange(0, std::memory_order_release) == 2) futex_wake_u32(&s, 1);
  }
};

// An epoch word many threads wait on for "something changed": waiters read the epoch, test
// their condition, and park while the epoch is unchanged; a notifier bumps it and wakes every
// parked waiter with one system call (none when nobody is parked).
struct EpochPark {
  std::atomic<uint32_t> epoch{0};
  std::atomic<int> sleepers{0};
  uint32_t read() const { return epoch.load(std::memory_order_acquire); }
  // parks until the epoch moves past `seen` (or timeout_ns passes: a safety net, never the
  // hand-off itself); false when it ended by the timeout
  bool wait(uint32_t seen, int64_t timeout_ns) {
    sleepers.fetch_add(1, std::memory_order_seq_cst);
    bool woke = true;
    if (epoch.load(std::memory_order_seq_cst) == seen) woke = futex_wait_u32(&epoch, seen, timeout_ns);
    sleepers.fetch_sub(1, std::memory_order_relaxed);
    return woke;
  }
  void notify() {
    epoch.fetch_add(1, std::memory_order_seq_cst);
    if (sleepers.load(std::memory_order_seq_cst) > 0) futex_wake_u32(&epoch);
  }
};

}  // namespace tsg
