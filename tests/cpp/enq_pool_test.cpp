// CPU stress test of mde_group's enqueue threads (mydatastore_amd/csrc/enq_pool.hpp), meant to run
// under ThreadSanitizer (tests/test_enq_pool.py builds it with -fsanitize=thread):
//   * every call runs every share exactly once, share 0 on the caller, the others each on its
//     own worker thread, and run() returns only after all of them;
//   * the lowest failing share's code is returned with its index;
//   * idle gaps longer than the workers' spin put them to sleep and the next call wakes them (no
//     lost wake-up: a lost one hangs, which the pytest timeout turns into a failure);
//   * pools are created and destroyed repeatedly, with workers asleep or spinning.
// Prints "ok <calls>" and exits 0, or names the first mismatch and exits 1.
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../mydatastore_amd/csrc/enq_pool.hpp"

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 4000;
  uint64_t total = 0;
  for (uint32_t shares : {2u, 3u, 8u}) {
    for (int rep = 0; rep < 2; rep++) {
      mde::EnqPool pool(shares);
      std::vector<uint64_t> seen(shares, 0);       // plain: each share writes only its own slot
      std::vector<std::thread::id> who(shares);
      std::atomic<uint32_t> ran{0};
      for (int c = 1; c <= calls; c++) {
        const uint64_t tag = (uint64_t)c;
        const uint32_t fail_a = (c % 7 == 0) ? (uint32_t)(c % shares) : UINT32_MAX;
        const uint32_t fail_b = (c % 11 == 0) ? (uint32_t)((c / 11) % shares) : UINT32_MAX;
        ran.store(0);
        uint32_t failed = 99;
        const int rc = pool.run(
            [&](uint32_t i) {
              seen[i] = tag;
              who[i] = std::this_thread::get_id();
              ran.fetch_add(1);
              if (i == fail_a) return -3;
              if (i == fail_b) return -7;
              return 0;
            },
            &failed);
        if (ran.load() != shares) {
          fprintf(stderr, "shares %u call %d: %u of %u shares ran\n", shares, c, ran.load(), shares);
          return 1;
        }
        for (uint32_t i = 0; i < shares; i++) {
          if (seen[i] != tag) {
            fprintf(stderr, "shares %u call %d: share %u saw call %llu\n", shares, c, i, (unsigned long long)seen[i]);
            return 1;
          }
        }
        if (who[0] != std::this_thread::get_id()) {
          fprintf(stderr, "share 0 did not run on the caller\n");
          return 1;
        }
        for (uint32_t i = 1; i < shares; i++)
          for (uint32_t j = 0; j < i; j++)
            if (who[i] == who[j]) {
              fprintf(stderr, "shares %u and %u ran on one thread\n", j, i);
              return 1;
            }
        uint32_t want_i = UINT32_MAX;
        int want_rc = 0;
        for (uint32_t i = 0; i < shares; i++) {
          const int r = i == fail_a ? -3 : (i == fail_b ? -7 : 0);
          if (r) {
            want_i = i;
            want_rc = r;
            break;
          }
        }
        if (rc != want_rc || (want_rc && failed != want_i)) {
          fprintf(stderr, "shares %u call %d: rc %d failed %u, want %d at %u\n", shares, c, rc, failed, want_rc,
                  want_i);
          return 1;
        }
        if (c % 500 == 0)  // longer than the spin: the workers go to sleep, the next call wakes them
          std::this_thread::sleep_for(mde::EnqPool::kSpin * 3);
        total++;
      }
      if (rep == 1) std::this_thread::sleep_for(mde::EnqPool::kSpin * 3);  // destroy with sleepers
    }
  }
  printf("ok %llu\n", (unsigned long long)total);
  return 0;
}
