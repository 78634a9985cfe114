// enq_pool.hpp -- per-device host enqueue threads for mde_group (group.cpp run_all).
//
// A device-resident group call launches work on every device (a pipelined build per device, a
// diff, an extract, ...); each launch costs the host several microseconds (argument setup, the HIP
// runtime's launch path), so one thread launching for 8 GPUs spends 8x that per step against a
// device step of ~0.2 ms (C4 at N = 8). EnqPool::run hands share i to thread i (share 0 to the
// caller) and returns when every share has run: the host cost per call is one device's, not G
// devices'. After a job a worker spins on its job word for kSpin only while calls come back to
// back (the gap before its previous job was under kSpin: a run of pipelined group calls keeps it
// hot), else for kSpinCold -- a process calling now and then does not burn G-1 cores for 200 us
// after every call -- then sleeps on a condition variable.
//
// Host-only (no HIP): tests/cpp/enq_pool_test.cpp drives it under ThreadSanitizer.
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace mde {

class EnqPool {
 public:
  static constexpr auto kSpin = std::chrono::microseconds(200);
  static constexpr auto kSpinCold = std::chrono::microseconds(5);

  // `shares` = the number of shares per call (the group's devices); threads for shares 1.. start
  // here and stop in the destructor.
  explicit EnqPool(uint32_t shares) : w_(shares) {
    for (uint32_t i = 1; i < shares; i++) w_[i].reset(new Worker());
    for (uint32_t i = 1; i < shares; i++) w_[i]->th = std::thread(&EnqPool::loop, this, i);
  }
  ~EnqPool() {
    for (auto& w : w_) {
      if (!w) continue;
      {
        std::lock_guard<std::mutex> lk(w->m);
        w->quit.store(true);
      }
      w->cv.notify_one();
      if (w->th.joinable()) w->th.join();
    }
  }
  EnqPool(const EnqPool&) = delete;
  EnqPool& operator=(const EnqPool&) = delete;

  // fn(i) for every share i, share 0 on the calling thread; returns the lowest failing share's
  // code (fn's non-zero return) with *failed = that share, or 0. One call at a time per pool.
  int run(const std::function<int(uint32_t)>& fn, uint32_t* failed) {
    std::lock_guard<std::mutex> lk(run_mu_);
    const uint32_t n = (uint32_t)w_.size();
    job_ = &fn;
    const uint64_t seq = ++seq_;
    for (uint32_t i = 1; i < n; i++) {
      Worker& w = *w_[i];
      w.posted.store(seq);
      if (w.sleeping.load()) {
        { std::lock_guard<std::mutex> wl(w.m); }
        w.cv.notify_one();
      }
    }
    int rc = fn(0);
    *failed = 0;
    for (uint32_t i = 1; i < n; i++) {
      Worker& w = *w_[i];
      for (uint32_t spin = 1; w.finished.load() != seq; spin++) {
        if (spin < 4096)
          _mm_pause();
        else
          std::this_thread::yield();
      }
      if (!rc && w.rc) {
        rc = w.rc;
        *failed = i;
      }
    }
    job_ = nullptr;
    return rc;
  }

 private:
  struct Worker {
    std::thread th;
    std::atomic<uint64_t> posted{0}, finished{0};
    std::atomic<bool> sleeping{false}, quit{false};
    std::mutex m;
    std::condition_variable cv;
    int rc = 0;  // written by the worker before `finished`, read by run() after it
  };

  // Lost wake-ups: the worker sets `sleeping` and re-checks `posted` under its mutex; run() stores
  // `posted` before it loads `sleeping` (both sequentially consistent), so either the worker sees
  // the new job word or run() sees it sleeping and notifies under the same mutex.
  void loop(uint32_t i) {
    Worker& w = *w_[i];
    uint64_t last = 0;
    bool hot = false;  // the previous job came within kSpin of the one before it
    for (;;) {
      uint64_t p = w.posted.load();
      auto t0 = std::chrono::steady_clock::now();
      const auto budget = hot ? std::chrono::duration_cast<std::chrono::steady_clock::duration>(kSpin)
                              : std::chrono::duration_cast<std::chrono::steady_clock::duration>(kSpinCold);
      bool slept = false;
      for (uint32_t spin = 1; p == last && !w.quit.load(); spin++) {
        _mm_pause();
        if ((spin & 63) == 0 && std::chrono::steady_clock::now() - t0 > budget) {
          slept = true;
          std::unique_lock<std::mutex> lk(w.m);
          w.sleeping.store(true);
          w.cv.wait(lk, [&] { return w.posted.load() != last || w.quit.load(); });
          w.sleeping.store(false);
          t0 = std::chrono::steady_clock::now();
        }
        p = w.posted.load();
      }
      if (p == last) return;  // quit
      hot = !slept && std::chrono::steady_clock::now() - t0 <= kSpin;
      w.rc = (*job_)(i);
      last = p;
      w.finished.store(p);
    }
  }

  std::vector<std::unique_ptr<Worker>> w_;
  const std::function<int(uint32_t)>* job_ = nullptr;
  uint64_t seq_ = 0;
  std::mutex run_mu_;
};

}  // namespace mde
