// server.cpp -- the resident build service (mde_server, include/mde.h): one-partition builds
// without a kernel launch per call.
//
// The reference builds ONE partition per VerifyEpoch (main/manager.go:1036 ->
// RawPartitionMerkleTree, main/merkle_tree.go:86-116): a few KB of 8-byte timestamps
// (main/manager.go:816) at partition_buckets = 1000 (config/default-config.yaml:10), on up to
// partition_concurrency = 10 workers. Through mde_build or the batcher (batch.cpp) every call pays
// a launch, a copy command each way and a completion event -- ~20 us of round trip around a few us
// of digest work. Here a persistent launch (digest.hip server_kernel) keeps one workgroup per
// request slot resident on the device; the slots live in coherent pinned host memory:
//   * a caller takes a free slot, packs its records into the slot's pinned in region (values, the
//     rebased seg_rec, value_off unless the records have one length), writes the request
//     descriptor and then the slot's sequence word (release);
//   * the slot's workgroup, polling that word over PCIe, copies the inputs into device memory in
//     one round trip, runs the one-launch small build (small_build_body: bucket sums in LDS, then
//     the split-schedule SHA-256 tree, or no tree for a digest-only build) with its outputs stored
//     straight into the slot's pinned out region, and publishes `done` (system-scope release);
//   * the caller spins on `done` and copies its outputs out.
// Lifetime: the launch ends by itself after `lifetime` (MDE_SERVER_LIFETIME_MS, default 100 ms),
// so an idle process holds no GPU work; the next request relaunches it. Each workgroup, when its
// lifetime is over, sets its slot's `closed` word, fences and reads the slot once more; a caller
// that posts and then reads `closed` set waits for the launch to end and relaunches (a request
// is served either by the closing workgroup's last read or by the next launch, never lost).
// The launch runs on a CU-masked stream: such a stream gets a hardware queue of its own, so no
// other stream of the process queues behind the persistent kernel (destroyed with the service, its
// context destroyed first: see mde_server_create).
// Requests the resident workgroups do not take (more partitions than one workgroup holds, inputs
// or outputs beyond a slot, B beyond the launch's LDS) run as mde_build on the service's own
// context. Each caller gets exactly what mde_build returns for its inputs (tests/cpp/server_test.c
// against mde_build and the C oracle under concurrent callers).
#include "../../include/mde.h"
#include "device_scope.hpp"
#include "mde_internal.hpp"

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace {

void put_msg(char* buf, uint64_t cap, const char* msg) {
  if (!buf || !cap) return;
  const uint64_t n = std::min<uint64_t>(std::strlen(msg), cap - 1);
  std::memcpy(buf, msg, n);
  buf[n] = 0;
}

int failf(char* buf, uint64_t cap, int code, const char* fmt, ...) {
  char m[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(m, sizeof m, fmt, ap);
  va_end(ap);
  put_msg(buf, cap, m);
  return code;
}

uint64_t a16(uint64_t x) { return (x + 15) & ~15ull; }

constexpr uint32_t kDefaultSlots = 16;
constexpr uint32_t kMaxSlots = 256;
constexpr uint64_t kDefaultInCap = 256ull << 10;
constexpr uint64_t kDefaultLifetimeMs = 100;
constexpr double kWaitTimeoutS = 30.0;
constexpr double kSpinS = 10e-6;  // pure spinning before a waiting caller starts yielding
constexpr uint32_t kMaxPeers = 16;  // decision steps with more peers run on the service's context

// MDE_SERVER_CUMASK=2: CU-masked streams kept for the process (see mde_server_create), per device: a service takes one
// no live service holds (two services on one stream would queue each launch behind the other's
// lifetime) and hands it back when its launch has ended.
constexpr int kKeptDevices = 64;
std::mutex g_kept_m;
std::vector<hipStream_t> g_kept_free[kKeptDevices];

// A caller waiting for a request slot (take_slot / give_slot).
struct SlotWaiter {
  std::condition_variable cv;
  uint32_t slot = UINT32_MAX;
};

}  // namespace

struct mde_server {
  int device = 0;
  uint32_t n_slots = kDefaultSlots;
  uint32_t max_buckets = 1024;
  uint64_t in_cap = kDefaultInCap, out_cap = 0;
  size_t lds = 0;
  uint64_t lifetime_ticks = 0;  // s_memrealtime ticks (wall_khz per ms)
  uint32_t wall_khz = 0;
  bool stage = true;  // MDE_SERVER_STAGE=0: the build reads its inputs in place over PCIe (A/B)
  uint8_t* pin = nullptr;      // [n_slots ServerSlot][n_slots x in_cap][n_slots x out_cap], coherent
  uint8_t* pin_dev = nullptr;  // its device address
  uint8_t* dev_in = nullptr;   // [n_slots x in_cap] device staging
  uint8_t* vscr = nullptr;     // [n_slots x vscr_cap] decision-step scratch (peer digests, nodes, diffs, ...)
  uint64_t vscr_cap = 0;
  hipStream_t stream = nullptr;
  bool keep_stream = false;  // a process-lifetime stream (MDE_SERVER_CUMASK=2, the round-4 pool)
  hipEvent_t exit_ev = nullptr;
  bool running = false;
  std::mutex launch_m;
  std::mutex m;
  std::vector<uint32_t> free_slots;
  std::deque<SlotWaiter*> slot_waiters;  // callers waiting for a slot, first come first served
  std::vector<uint64_t> seq;  // per slot, owned by the caller holding the slot
  std::atomic<uint64_t> n_req{0}, n_launch{0}, n_ctx{0};
  // MDE_SERVER_DEBUG totals, printed by mde_server_destroy: time waiting for a slot and for `done`
  std::atomic<uint64_t> ns_slot{0}, ns_done{0};
  // a launch failed, a request timed out or mde_server_disable: every later call runs on the
  // service's context (a slot whose request failed is never reused -- its workgroup may still write it)
  std::atomic<bool> broken{false};
  std::string broken_msg;
  mde_ctx* ctx = nullptr;  // requests the resident workgroups do not take
  std::mutex ctx_m;

  mde::ServerSlot* slot(uint32_t i) { return reinterpret_cast<mde::ServerSlot*>(pin) + i; }
  uint64_t in_off(uint32_t i) const { return (uint64_t)n_slots * sizeof(mde::ServerSlot) + (uint64_t)i * in_cap; }
  uint64_t out_off(uint32_t i) const {
    return (uint64_t)n_slots * sizeof(mde::ServerSlot) + (uint64_t)n_slots * in_cap + (uint64_t)i * out_cap;
  }
};

namespace {

// Output layout of one request in a slot's out region.
struct OutLayout {
  uint64_t dig, size, items, root, nodes, total;
};
OutLayout out_layout(uint32_t P, uint32_t B, bool tree, bool nodes) {
  OutLayout o{};
  const uint64_t S = (uint64_t)P * B;
  o.dig = 0;
  o.size = a16(S * 8);
  o.items = o.size + a16(S * 4);
  o.root = o.items + a16((uint64_t)P * 4);
  o.nodes = o.root + (tree ? a16((uint64_t)P * 32) : 0);
  o.total = o.nodes + (nodes ? a16((uint64_t)P * mde::tree_internal(B) * 32) : 0);
  return o;
}

// Device scratch of one decision step (mde_api.cpp verify_async, P = 1): peer digests, sizes,
// bucket counts, valid flags, nodes, roots, diff ids, statuses; the local tree's nodes and root
// (built in the launch only when a peer of another shape needs them); the partition's valid flag
// (read back by the encoder); the decoder's spill area for nested unknown groups.
struct VerifyScratch {
  uint64_t off[13];
};
VerifyScratch verify_scratch(uint32_t B, uint32_t R, uint64_t peer_bytes) {
  const uint32_t cap = mde_verify_peer_capacity(B);
  const uint64_t T = R, NI = mde::tree_internal(cap), idcap = mde_diff_capacity(B, cap), NL = mde::tree_internal(B);
  const uint64_t part[12] = {T * cap * 8, T * cap * 4, T * 4, T, T * NI * 32, T * 32, T * idcap * 4, T * 4,
                             NL * 32, 32, 1, mde::wire_deep_entries(T, peer_bytes) * 4};
  VerifyScratch v{};
  for (int i = 0; i < 12; i++) v.off[i + 1] = v.off[i] + ((part[i] + 255) & ~255ull);
  return v;
}

// The checks mde_build makes on host records (layout A), with the caller's message buffer.
int validate(const mde_records* r, const mde_tree_out* o, char* err, uint64_t cap) {
  if (r->layout != MDE_LAYOUT_SORTED) return failf(err, cap, MDE_E_INVAL, "mde_server_build takes layout A records");
  if (!r->seg_rec || !r->n_buckets || !r->n_partitions)
    return failf(err, cap, MDE_E_INVAL, "seg_rec, n_buckets and n_partitions are required");
  if (!o->root && o->nodes) return failf(err, cap, MDE_E_INVAL, "out/nodes needs out/root");
  if ((uint64_t)r->n_partitions * r->n_buckets > 0xffffffffull)
    return failf(err, cap, MDE_E_INVAL, "n_partitions * n_buckets exceeds 2^32");
  if (r->value_stride == 0 && !r->value_off && r->n_records)
    return failf(err, cap, MDE_E_INVAL, "variable-length values need value_off");
  if (!r->values && r->values_bytes) return failf(err, cap, MDE_E_INVAL, "values is NULL");
  if (r->value_stride && (uint64_t)r->value_stride * r->n_records > r->values_bytes)
    return failf(err, cap, MDE_E_INVAL, "n_records * value_stride exceeds values_bytes");
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  for (uint64_t s = 0; s < S; s++)
    if (r->seg_rec[s] > r->seg_rec[s + 1])
      return failf(err, cap, MDE_E_INVAL, "seg_rec not nondecreasing at %llu", (unsigned long long)s);
  if (r->seg_rec[S] > r->n_records)
    return failf(err, cap, MDE_E_INVAL, "seg_rec[%llu] exceeds n_records", (unsigned long long)S);
  if (!r->value_stride && r->n_records) {
    for (uint64_t i = 0; i < r->n_records; i++)
      if (r->value_off[i] > r->value_off[i + 1])
        return failf(err, cap, MDE_E_INVAL, "value_off not nondecreasing at %llu", (unsigned long long)i);
    if (r->value_off[r->n_records] > r->values_bytes)
      return failf(err, cap, MDE_E_INVAL, "value_off[n_records] exceeds values_bytes");
  }
  return MDE_OK;
}

// Make sure a launch is serving (or relaunch after the previous one ended its lifetime).
int ensure_running(mde_server* s, std::string* msg) {
  std::lock_guard<std::mutex> lk(s->launch_m);
  if (s->running) {
    hipError_t e = hipEventQuery(s->exit_ev);
    if (e == hipErrorNotReady) {
      bool closing = false;
      for (uint32_t i = 0; i < s->n_slots && !closing; i++)
        closing = __atomic_load_n(&s->slot(i)->closed, __ATOMIC_ACQUIRE) != 0;
      if (!closing) return MDE_OK;
      // its workgroups share one lifetime: the rest close within about one request
      e = hipEventSynchronize(s->exit_ev);
    }
    if (e != hipSuccess) {
      *msg = std::string("resident build launch failed: ") + hipGetErrorString(e);
      return MDE_E_DEVICE;
    }
    s->running = false;
  }
  for (uint32_t i = 0; i < s->n_slots; i++) __atomic_store_n(&s->slot(i)->closed, 0u, __ATOMIC_RELAXED);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  DeviceScope ds(s->device);
  hipError_t e = mde::launch_server(reinterpret_cast<mde::ServerSlot*>(s->pin_dev), s->n_slots, s->lifetime_ticks,
                                    s->lds, s->stream);
  if (e == hipSuccess) e = hipEventRecord(s->exit_ev, s->stream);
  if (e != hipSuccess) {
    for (uint32_t i = 0; i < s->n_slots; i++) __atomic_store_n(&s->slot(i)->closed, 1u, __ATOMIC_RELAXED);
    *msg = std::string("resident build launch: ") + hipGetErrorString(e);
    return MDE_E_DEVICE;
  }
  s->running = true;
  s->n_launch.fetch_add(1, std::memory_order_relaxed);
  return MDE_OK;
}

// Post request `q` on slot i and wait for its `done`.
int post_and_wait(mde_server* s, uint32_t i, std::string* msg) {
  const auto tw = std::chrono::steady_clock::now();
  struct WaitTime {
    mde_server* s;
    std::chrono::steady_clock::time_point t;
    ~WaitTime() {
      s->ns_done.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - t).count(), std::memory_order_relaxed);
    }
  } wait_time{s, tw};
  mde::ServerSlot* sl = s->slot(i);
  const uint64_t q = ++s->seq[i];
  __atomic_store_n(&sl->req, q, __ATOMIC_RELEASE);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);  // req before closed (the workgroup: closed before req)
  if (__atomic_load_n(&sl->closed, __ATOMIC_ACQUIRE)) {
    const int rc = ensure_running(s, msg);
    if (rc) return rc;
  }
  const auto t0 = std::chrono::steady_clock::now();
  bool yielding = false;
  for (uint64_t spin = 1;; spin++) {
    if (__atomic_load_n(&sl->done, __ATOMIC_ACQUIRE) == q) return MDE_OK;
    // spin through a short call's round trip, then give the core away between checks: with more
    // callers than cores (100 goroutines on a 16-core share) spinning slot holders would starve
    // the callers that pack requests or build host trees
    if (yielding)
      std::this_thread::yield();
    else
      _mm_pause();
    if ((spin & 15) == 0 && !yielding)
      yielding = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kSpinS;
    if ((spin & 63) == 0) {
      if (__atomic_load_n(&sl->closed, __ATOMIC_ACQUIRE)) {
        // the workgroup closed: served by its last read, or by the next launch
        const int rc = ensure_running(s, msg);
        if (rc) return rc;
        continue;
      }
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (dt > kWaitTimeoutS) {
        const hipError_t e = hipEventQuery(s->exit_ev);
        *msg = std::string("resident build request timed out (launch: ") + hipGetErrorString(e) + ")";
        return MDE_E_DEVICE;
      }
      if ((spin & 4095) == 0) {
        const hipError_t e = hipEventQuery(s->exit_ev);
        if (e != hipSuccess && e != hipErrorNotReady) {
          *msg = std::string("resident build launch failed: ") + hipGetErrorString(e);
          return MDE_E_DEVICE;
        }
      }
    }
  }
}

// Once the service is out of service no request is posted again: the workgroup of an idle slot is
// told to exit (kServerStop), so the launch gives its CUs back as its slots go idle instead of
// polling until its lifetime ends. Called under s->m for a slot no caller holds.
void stop_idle_slot(mde_server* s, uint32_t i) {
  __atomic_store_n(&s->slot(i)->req, mde::kServerStop, __ATOMIC_RELEASE);
}

// A free slot, or UINT32_MAX once the service is broken. Callers finding none queue in FIFO order
// and sleep on a condition variable of their own; give_slot hands a returned slot straight to the
// first of them (one wakeup per handoff: a shared condition variable woke callers that found the
// slot already re-taken -- 25-56 k futile wakeups per 80-110 k calls at 100 callers, most of the
// process's CPU time spent in the kernel, profiles/r04/r04cw_callers_wait.txt).
uint32_t take_slot(mde_server* s) {
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(s->m);
  uint32_t i = UINT32_MAX;
  if (!s->broken.load() && !s->free_slots.empty()) {
    i = s->free_slots.back();
    s->free_slots.pop_back();
  } else if (!s->broken.load()) {
    SlotWaiter w;
    s->slot_waiters.push_back(&w);
    w.cv.wait(lk, [&] { return w.slot != UINT32_MAX || s->broken.load(); });
    if (s->broken.load()) {  // give back a slot handed over meanwhile, leave the queue
      if (w.slot != UINT32_MAX) {
        stop_idle_slot(s, w.slot);
        s->free_slots.push_back(w.slot);
      }
      auto it = std::find(s->slot_waiters.begin(), s->slot_waiters.end(), &w);
      if (it != s->slot_waiters.end()) s->slot_waiters.erase(it);
    } else {
      i = w.slot;
    }
  }
  lk.unlock();
  s->ns_slot.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                           std::chrono::steady_clock::now() - t0).count(), std::memory_order_relaxed);
  return i;
}

void mark_broken(mde_server* s, const std::string& msg) {
  std::lock_guard<std::mutex> lk(s->m);
  if (!s->broken.load()) s->broken_msg = msg;
  s->broken.store(true);
  for (SlotWaiter* w : s->slot_waiters) w->cv.notify_one();  // under the lock: w lives on its caller's stack
}

void give_slot(mde_server* s, uint32_t i) {
  std::lock_guard<std::mutex> lk(s->m);
  if (s->broken.load()) {  // out of service: no waiter is served by the launch any more
    stop_idle_slot(s, i);
    s->free_slots.push_back(i);
  } else if (!s->slot_waiters.empty()) {
    SlotWaiter* w = s->slot_waiters.front();
    s->slot_waiters.pop_front();
    w->slot = i;
    w->cv.notify_one();  // under the lock (see mark_broken)
  } else {
    s->free_slots.push_back(i);
  }
}

}  // namespace

extern "C" {

int mde_server_create(int device, uint32_t n_slots, uint32_t max_buckets, mde_server** out) {
  if (!out) return MDE_E_INVAL;
  *out = nullptr;
  if (n_slots > kMaxSlots || max_buckets > mde::kTreeLdsMaxBuckets) return MDE_E_INVAL;
  {  // the device checks mde_create makes, before any allocation (its context is created later)
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      (void)hipGetLastError();
      return MDE_E_DEVICE;
    }
    if (device < 0 || device >= n) return MDE_E_INVAL;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return MDE_E_DEVICE;
  }
  mde_server* s = new (std::nothrow) mde_server();
  if (!s) return MDE_E_NOMEM;
  s->device = device;
  if (n_slots) s->n_slots = n_slots;
  if (max_buckets) s->max_buckets = max_buckets;
  uint64_t life_ms = kDefaultLifetimeMs;
  if (const char* e = std::getenv("MDE_SERVER_LIFETIME_MS")) {
    const long long ms = std::atoll(e);
    if (ms >= 1) life_ms = (uint64_t)ms;
  }
  // s_memrealtime ticks at the device's wall-clock rate (kHz)
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) {
    (void)hipGetLastError();
    khz = 100000;
  }
  s->wall_khz = (uint32_t)khz;
  s->lifetime_ticks = life_ms * (uint64_t)khz;
  if (const char* e = std::getenv("MDE_SERVER_STAGE")) s->stage = std::atoi(e) != 0;
  auto bail = [&](int code) {
    mde_server_destroy(s);
    return code;
  };
  DeviceScope ds(device);
  s->lds = mde::server_lds_bytes(s->max_buckets);
  uint32_t G, words, duo;
  if (!s->lds || !mde::server_plan(1, s->max_buckets, s->lds, &G, &words, &duo)) return bail(MDE_E_INVAL);
  // outputs of a build with nodes, or of a decision step with its object and kMaxPeers statuses
  s->out_cap = a16(std::max<uint64_t>(out_layout(1, s->max_buckets, true, true).total,
                                      64 + a16((uint64_t)s->max_buckets * 4) + a16(kMaxPeers * 4) +
                                          a16(mde_epoch_tree_object_max_bytes(s->max_buckets))));
  const uint64_t bytes = (uint64_t)s->n_slots * (sizeof(mde::ServerSlot) + s->in_cap + s->out_cap);
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    (void)hipGetLastError();
    return bail(MDE_E_NOMEM);
  }
  s->pin = static_cast<uint8_t*>(p);
  std::memset(s->pin, 0, bytes);
  void* pd = nullptr;
  if (hipHostGetDevicePointer(&pd, s->pin, 0) != hipSuccess) return bail(MDE_E_DEVICE);
  s->pin_dev = static_cast<uint8_t*>(pd);
  void* di = nullptr;
  if (hipMalloc(&di, (uint64_t)s->n_slots * s->in_cap) != hipSuccess) {
    (void)hipGetLastError();
    return bail(MDE_E_NOMEM);
  }
  s->dev_in = static_cast<uint8_t*>(di);
  s->vscr_cap = verify_scratch(s->max_buckets, kMaxPeers, s->in_cap).off[12];
  void* vs = nullptr;
  if (hipMalloc(&vs, (uint64_t)s->n_slots * s->vscr_cap) != hipSuccess) {
    (void)hipGetLastError();
    return bail(MDE_E_NOMEM);
  }
  s->vscr = static_cast<uint8_t*>(vs);
  // a CU-masked stream gets a hardware queue of its own (all CUs enabled): nothing else of this
  // process queues behind the persistent launch
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
  std::vector<uint32_t> mask((size_t)std::max(1, (cus + 31) / 32), 0u);
  for (int c = 0; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
  // The launch's stream: a CU-masked stream (all CUs) gets a hardware queue of its own, so no other
  // stream of the process queues behind the persistent kernel. By default (MDE_SERVER_CUMASK=2) it
  // is never destroyed: it goes back to a per-device pool and a later service on the device reuses
  // it (never two live ones). Destroying a CU-masked stream is what hung: hipStreamDestroy of a
  // stream created BEFORE the masked stream and destroyed AFTER it, with work of that stream run
  // while the persistent launch was live (profiles/r04/r04n_service_streams.txt,
  // profiles/r05/r05g_teardown_bisect.txt; the runtime-side wait was not identified -- DESIGN.md
  // section 7). The service's own context is created after the stream and destroyed before it
  // either way, but a caller's context created before the service and destroyed after it (the Go
  // shim's batchers, two services destroyed in creation order) would recreate the pattern if the
  // masked stream were destroyed, so the pool stays the default. MDE_SERVER_CUMASK=1: destroy it
  // with the service (callers then create every other context of the device after the service,
  // or destroy it before the service -- include/mde.h); 0: a plain non-blocking stream.
  const char* cm = std::getenv("MDE_SERVER_CUMASK");
  const int cmode = cm ? std::atoi(cm) : 2;
  s->keep_stream = cmode == 2 && device >= 0 && device < kKeptDevices;
  hipError_t se = hipSuccess;
  if (cmode == 0) {
    se = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  } else if (s->keep_stream) {
    std::lock_guard<std::mutex> lk(g_kept_m);
    std::vector<hipStream_t>& pool = g_kept_free[device];
    if (!pool.empty()) {
      s->stream = pool.back();
      pool.pop_back();
    } else {
      se = hipExtStreamCreateWithCUMask(&s->stream, (uint32_t)mask.size(), mask.data());
    }
  } else {
    se = hipExtStreamCreateWithCUMask(&s->stream, (uint32_t)mask.size(), mask.data());
  }
  if (se != hipSuccess || !s->stream) {
    (void)hipGetLastError();
    s->stream = nullptr;
    return bail(MDE_E_DEVICE);
  }
  if (hipEventCreateWithFlags(&s->exit_ev, hipEventDisableTiming) != hipSuccess) {
    s->exit_ev = nullptr;
    return bail(MDE_E_DEVICE);
  }
  // The service's own context (requests the resident workgroups do not take), created AFTER the
  // launch stream: a stream created before a CU-masked stream and destroyed after it hung in
  // hipStreamDestroy (ROCm 7.2); created after it, either order completes (DESIGN.md section 7,
  // profiles/r05/r05g_teardown_bisect.txt). mde_server_destroy also destroys it first.
  if (int rc = mde_create(device, &s->ctx)) return bail(rc);
  s->seq.assign(s->n_slots, 0);
  for (uint32_t i = 0; i < s->n_slots; i++) {
    s->free_slots.push_back(s->n_slots - 1 - i);
    s->slot(i)->closed = 1;  // no launch yet
  }
  std::string msg;
  if (ensure_running(s, &msg)) return bail(MDE_E_DEVICE);
  *out = s;
  return MDE_OK;
}

// Teardown contract: the launch stream is a CU-masked stream, and with the
// default MDE_SERVER_CUMASK=2 it is parked in the device's pool here, never destroyed -- the only
// teardown order known to hang is hipStreamDestroy of a masked stream while a stream created before
// it (used during the persistent launch) is destroyed after it. With MDE_SERVER_CUMASK=1 the
// caller must keep that order out: create services before, and destroy them after, every other
// context / stream of the device.
void mde_server_destroy(mde_server* s) {
  if (!s) return;
  DeviceScope ds(s->device);
  if (s->pin) {
    for (uint32_t i = 0; i < s->n_slots; i++) __atomic_store_n(&s->slot(i)->req, mde::kServerStop, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  const bool dbg = std::getenv("MDE_SERVER_DEBUG") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  // bounded wait for the launch to end (it reads the stop word within microseconds, and ends at
  // its lifetime in any case); a launch that does not end keeps its buffers (never freed under it)
  bool ended = true;
  if (s->running && s->exit_ev) {
    bool told = false;
    for (;;) {
      const hipError_t e = hipEventQuery(s->exit_ev);
      if (e != hipErrorNotReady) {
        if (dbg) std::fprintf(stderr, "mde_server_destroy: launch ended after %.6f s (%s)\n", since(), hipGetErrorString(e));
        break;
      }
      const double dt = since();
      if (dt > 1.0 && !told) {
        told = true;
        std::fprintf(stderr, "mde_server_destroy: launch still running after 1 s; slots (req done closed):");
        for (uint32_t i = 0; i < s->n_slots; i++)
          std::fprintf(stderr, " [%llx %llu %u]", (unsigned long long)__atomic_load_n(&s->slot(i)->req, __ATOMIC_ACQUIRE),
                       (unsigned long long)__atomic_load_n(&s->slot(i)->done, __ATOMIC_ACQUIRE),
                       __atomic_load_n(&s->slot(i)->closed, __ATOMIC_ACQUIRE));
        std::fprintf(stderr, "\n");
      }
      if (dt > 10.0) {
        std::fprintf(stderr, "mde_server_destroy: launch did not end within 10 s; its buffers are kept\n");
        ended = false;
        break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  if (ended) {
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (dbg) std::fprintf(stderr, "mde_server_destroy: stream synchronized %.6f s\n", since());
    // the service's context before its launch stream (see mde_server_create)
    if (s->ctx) {
      mde_destroy(s->ctx);
      s->ctx = nullptr;
      if (dbg) std::fprintf(stderr, "mde_server_destroy: context destroyed %.6f s\n", since());
    }
    if (s->exit_ev) (void)hipEventDestroy(s->exit_ev);
    if (dbg) std::fprintf(stderr, "mde_server_destroy: destroying the launch stream %.6f s\n", since());
    if (s->stream && !s->keep_stream) (void)hipStreamDestroy(s->stream);
    if (s->stream && s->keep_stream) {
      std::lock_guard<std::mutex> lk(g_kept_m);
      g_kept_free[s->device].push_back(s->stream);
    }
    if (s->dev_in) (void)hipFree(s->dev_in);
    if (s->vscr) (void)hipFree(s->vscr);
    if (s->pin) (void)hipHostFree(s->pin);
    if (dbg) std::fprintf(stderr, "mde_server_destroy: freed %.6f s\n", since());
  }
  if (s->ctx) mde_destroy(s->ctx);
  if (dbg)
    std::fprintf(stderr,
                 "mde_server_destroy: done %.6f s; requests %llu, waiting for a slot %.3f s, for done %.3f s\n",
                 since(), (unsigned long long)s->n_req.load(), 1e-9 * (double)s->ns_slot.load(),
                 1e-9 * (double)s->ns_done.load());
  delete s;
}

int mde_server_stats(mde_server* s, uint64_t* requests, uint64_t* launches, uint64_t* on_context) {
  if (!s) return MDE_E_INVAL;
  if (requests) *requests = s->n_req.load();
  if (launches) *launches = s->n_launch.load();
  if (on_context) *on_context = s->n_ctx.load();
  return MDE_OK;
}

uint32_t mde_server_slots(const mde_server* s) { return s ? s->n_slots : 0u; }

}  // extern "C"

namespace {

// A build through the service; top_nodes > 0: the tree stops at the first level of at most
// top_nodes nodes (mde_server_build_levels).
int server_build(mde_server* s, const mde_records* rec, const mde_tree_out* out_in, uint32_t top_nodes, char* err,
                 uint64_t err_cap) {
  put_msg(err, err_cap, "");
  if (!s || !rec || !out_in) return failf(err, err_cap, MDE_E_INVAL, "null server, records or out");
  mde_tree_out levels_out;
  uint8_t root_sink[32];
  if (top_nodes) {  // levels: nodes required, root not written (a scratch root keeps the tree phase)
    if (!out_in->nodes) return failf(err, err_cap, MDE_E_INVAL, "mde_server_build_levels needs out->nodes");
    levels_out = *out_in;
    levels_out.root = root_sink;
  }
  const mde_tree_out* out = top_nodes ? &levels_out : out_in;
  int rc = validate(rec, out, err, err_cap);
  if (rc) return rc;
  const uint32_t P = rec->n_partitions, B = rec->n_buckets;
  const uint64_t S = (uint64_t)P * B;
  const uint64_t r0 = rec->seg_rec[0], r1 = rec->seg_rec[S], n = r1 - r0;
  // records of one length (given, or detected from value_off): no offsets to send
  uint64_t stride = rec->value_stride;
  if (!stride && n) {
    const uint64_t d0 = rec->value_off[r0 + 1] - rec->value_off[r0];
    bool uniform = d0 > 0;
    for (uint64_t k = r0 + 1; k < r1 && uniform; k++) uniform = rec->value_off[k + 1] - rec->value_off[k] == d0;
    if (uniform && d0 <= 0xffffffffull) stride = d0;
  }
  const uint64_t b0 = rec->value_stride ? r0 * rec->value_stride : (n ? rec->value_off[r0] : 0);
  const uint64_t b1 = rec->value_stride ? r1 * rec->value_stride : (n ? rec->value_off[r1] : 0);
  const uint64_t V = b1 - b0;
  const uint64_t o_seg = a16(std::max<uint64_t>(V, 16));
  const uint64_t o_off = o_seg + a16((S + 1) * 8);
  const uint64_t in_bytes = o_off + (stride ? 0 : a16((n + 1) * 8));
  const bool tree = out->root != nullptr, nodes = out->nodes != nullptr;
  const OutLayout ol = out_layout(P, B, tree, nodes);
  uint32_t G = 0, words = 0, duo = 0;
  const bool fits = B <= s->max_buckets && in_bytes <= s->in_cap && ol.total <= s->out_cap &&
                    mde::server_plan(P, B, s->lds, &G, &words, &duo);
  s->n_req.fetch_add(1, std::memory_order_relaxed);
  // the service's context: the ordinary synchronous build (a levels call gets every level) -- for
  // requests the resident workgroups do not take, and for every request once the resident launch
  // is out of service (a failed launch, a timed-out request, mde_server_disable)
  auto on_context = [&](const char* why) {
    s->n_ctx.fetch_add(1, std::memory_order_relaxed);
    std::vector<uint8_t> roots;
    mde_tree_out o = *out;
    if (top_nodes) {
      roots.resize((uint64_t)P * 32);
      o.root = roots.data();
    }
    std::lock_guard<std::mutex> lk(s->ctx_m);
    const int r = mde_build(s->ctx, rec, &o);
    if (r) failf(err, err_cap, r, "%s%s", why, mde_last_error(s->ctx));
    return r;
  };
  if (!fits) return on_context("");
  const uint32_t i = take_slot(s);
  if (i == UINT32_MAX) return on_context("resident build service unusable, on its context: ");
  uint8_t* in_h = s->pin + s->in_off(i);
  const uint64_t in_d_pin = reinterpret_cast<uint64_t>(s->pin_dev + s->in_off(i));
  uint8_t* out_h = s->pin + s->out_off(i);
  uint8_t* out_d = s->pin_dev + s->out_off(i);
  // pack: values, seg_rec rebased to the first record, value_off rebased (variable lengths only)
  if (V) std::memcpy(in_h, rec->values + b0, V);
  std::memset(in_h + V, 0, o_seg - V);
  uint64_t* seg = reinterpret_cast<uint64_t*>(in_h + o_seg);
  for (uint64_t k = 0; k <= S; k++) seg[k] = rec->seg_rec[k] - r0;
  if (!stride) {
    uint64_t* off = reinterpret_cast<uint64_t*>(in_h + o_off);
    for (uint64_t k = 0; k <= n; k++) off[k] = rec->value_off[r0 + k] - b0;
  }
  const uint64_t in_base = s->stage ? reinterpret_cast<uint64_t>(s->dev_in + (uint64_t)i * s->in_cap) : in_d_pin;
  mde::ServerReq q{};
  q.d.base = reinterpret_cast<const uint8_t*>(in_base);
  q.d.shift = 0;
  q.d.stride = (uint32_t)stride;
  q.d.value_off = stride ? nullptr : reinterpret_cast<const uint64_t*>(in_base + o_off);
  q.d.seg_rec = reinterpret_cast<const uint64_t*>(in_base + o_seg);
  q.d.S = (uint32_t)S;
  q.d.n_records = n;
  q.d.end = V;
  q.t.P = P;
  q.t.B = B;
  q.t.seg_rec = q.d.seg_rec;
  q.t.digest_out = reinterpret_cast<uint64_t*>(out_d + ol.dig);
  q.t.size_out = reinterpret_cast<int32_t*>(out_d + ol.size);
  q.t.items_out = reinterpret_cast<int32_t*>(out_d + ol.items);
  q.t.root_out = tree ? out_d + ol.root : nullptr;
  q.t.nodes_out = nodes ? out_d + ol.nodes : nullptr;
  q.t.n_int = mde::tree_internal(B);
  q.t.top_nodes = top_nodes;
  q.kind = 0;
  q.G = G;
  q.words = words;
  q.duo = duo;
  q.stage = s->stage ? 1u : 0u;
  q.src = reinterpret_cast<const uint8_t*>(in_d_pin);
  q.dev_in = s->dev_in + (uint64_t)i * s->in_cap;
  q.stage_bytes = a16(in_bytes);
  std::memcpy(&s->slot(i)->r, &q, sizeof q);
  std::string msg;
  rc = post_and_wait(s, i, &msg);
  if (rc == MDE_OK) {
    if (out->digest) std::memcpy(out->digest, out_h + ol.dig, S * 8);
    if (out->size) std::memcpy(out->size, out_h + ol.size, S * 4);
    if (out->items) std::memcpy(out->items, out_h + ol.items, (uint64_t)P * 4);
    if (tree && !top_nodes) std::memcpy(out->root, out_h + ol.root, (uint64_t)P * 32);
    if (nodes) {
      const uint64_t per = top_nodes ? mde_tree_prefix_nodes(B, top_nodes) : q.t.n_int;
      for (uint32_t p = 0; p < P; p++)
        std::memcpy(out->nodes + (uint64_t)p * q.t.n_int * 32, out_h + ol.nodes + (uint64_t)p * q.t.n_int * 32, per * 32);
    }
    give_slot(s, i);
  } else {
    // the slot's workgroup may still write it: it stays out of the free list; this call and every
    // later one run on the service's context
    mark_broken(s, msg);
    rc = on_context((msg + "; on the service's context: ").c_str());
  }
  return rc;
}

}  // namespace

extern "C" {

int mde_server_build(mde_server* s, const mde_records* rec, const mde_tree_out* out, char* err, uint64_t err_cap) {
  return server_build(s, rec, out, 0, err, err_cap);
}

int mde_server_build_levels(mde_server* s, const mde_records* rec, const mde_tree_out* out, uint32_t top_nodes,
                            char* err, uint64_t err_cap) {
  return server_build(s, rec, out, top_nodes ? top_nodes : 1u, err, err_cap);
}

int mde_server_verify(mde_server* s, uint32_t n_buckets, int32_t partition, int64_t epoch, const uint64_t* digest,
                      const int32_t* size, uint32_t n_peers, const uint8_t* peer_bytes, const uint64_t* peer_off,
                      uint32_t replica_count, uint8_t* valid, int32_t* valid_count, int32_t* diff_ids,
                      int32_t* diff_count, int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                      uint32_t* object_len, char* err, uint64_t err_cap) {
  put_msg(err, err_cap, "");
  if (!s) return failf(err, err_cap, MDE_E_INVAL, "null server");
  const uint32_t B = n_buckets, R = n_peers;
  // mde_batch_verify's checks
  if (!B || !mde_verify_peer_capacity(B) || B > 65536u) return failf(err, err_cap, MDE_E_INVAL, "bad n_buckets %u", B);
  if (!digest || !valid || !valid_count || !diff_ids || !diff_count)
    return failf(err, err_cap, MDE_E_INVAL, "bad verify arguments");
  if (R && !peer_off) return failf(err, err_cap, MDE_E_INVAL, "peer_off is NULL");
  if (object_out && (!size || !object_len))
    return failf(err, err_cap, MDE_E_INVAL, "object_out needs size and object_len");
  if (object_out && object_stride < mde_epoch_tree_object_max_bytes(B))
    return failf(err, err_cap, MDE_E_CAPACITY, "object_stride too small");
  for (uint32_t r = 0; r < R; r++)
    if (peer_off[r] > peer_off[r + 1]) return failf(err, err_cap, MDE_E_INVAL, "peer_off not nondecreasing");
  const uint64_t nbytes = R ? peer_off[R] - peer_off[0] : 0;
  if (nbytes && !peer_bytes) return failf(err, err_cap, MDE_E_INVAL, "peer_bytes is NULL");
  // the slot's in region: digests, sizes, partition, peer offsets (rebased), peer bytes
  const uint64_t i_dig = 0, i_size = a16((uint64_t)B * 8), i_part = i_size + a16((uint64_t)B * 4),
                 i_off = i_part + 16, i_peer = i_off + a16(((uint64_t)R + 1) * 8);
  const uint64_t in_bytes = i_peer + a16(nbytes + 1);
  // out region: valid, valid_count, diff_count, object_len, then diff ids, statuses, the object
  const uint64_t o_ids = 64, o_st = o_ids + a16((uint64_t)B * 4), o_obj = o_st + a16((uint64_t)R * 4);
  const uint64_t ostride = object_out ? mde_epoch_tree_object_max_bytes(B) : 0;
  const uint64_t out_bytes = o_obj + a16(ostride);
  const uint32_t cap = mde_verify_peer_capacity(B);
  const VerifyScratch vs = verify_scratch(B, R, nbytes);
  s->n_req.fetch_add(1, std::memory_order_relaxed);
  // the service's context (see server_build)
  auto on_context = [&](const char* why) {
    s->n_ctx.fetch_add(1, std::memory_order_relaxed);
    std::lock_guard<std::mutex> lk(s->ctx_m);
    const int r = mde_verify_epochs(s->ctx, 1, B, &partition, epoch, digest, size, nullptr, R, peer_bytes, peer_off,
                                    replica_count, valid, valid_count, diff_ids, diff_count, peer_status, object_out,
                                    object_stride, object_len);
    if (r) failf(err, err_cap, r, "%s%s", why, mde_last_error(s->ctx));
    return r;
  };
  if (B > s->max_buckets || R > kMaxPeers || !mde::verify_fused_fits(R, cap) || in_bytes > s->in_cap ||
      out_bytes > s->out_cap || vs.off[12] > s->vscr_cap)
    return on_context("");
  const uint32_t i = take_slot(s);
  if (i == UINT32_MAX) return on_context("resident build service unusable, on its context: ");
  uint8_t* in_h = s->pin + s->in_off(i);
  const uint8_t* in_pin_d = s->pin_dev + s->in_off(i);
  uint8_t* out_h = s->pin + s->out_off(i);
  uint8_t* out_d = s->pin_dev + s->out_off(i);
  std::memcpy(in_h + i_dig, digest, (uint64_t)B * 8);
  if (size) std::memcpy(in_h + i_size, size, (uint64_t)B * 4);
  std::memcpy(in_h + i_part, &partition, 4);
  uint64_t* off = reinterpret_cast<uint64_t*>(in_h + i_off);
  for (uint32_t r = 0; r <= R; r++) off[r] = R ? peer_off[r] - peer_off[0] : 0;
  if (nbytes) std::memcpy(in_h + i_peer, peer_bytes + peer_off[0], nbytes);
  const uint8_t* in = s->stage ? s->dev_in + (uint64_t)i * s->in_cap : in_pin_d;
  uint8_t* sc = s->vscr + (uint64_t)i * s->vscr_cap;
  auto at = [&](int k) { return static_cast<void*>(sc + vs.off[k]); };
  const uint64_t T = R, NI = mde::tree_internal(cap), idcap = mde_diff_capacity(B, cap);
  const uint64_t* d_dig = reinterpret_cast<const uint64_t*>(in + i_dig);
  uint64_t* pd = static_cast<uint64_t*>(at(0));
  int32_t* nbk = static_cast<int32_t*>(at(2));
  uint8_t* pvalid = static_cast<uint8_t*>(at(3));
  uint8_t* pnodes = static_cast<uint8_t*>(at(4));
  int32_t* pids = static_cast<int32_t*>(at(6));
  int32_t* pst = static_cast<int32_t*>(at(7));
  uint8_t* lnodes = static_cast<uint8_t*>(at(8));
  uint8_t* vdev = static_cast<uint8_t*>(at(10));
  mde::ServerReq q{};
  q.kind = 1;
  q.v.dec = mde::WireDecodeLaunch{(uint32_t)T, in + i_peer, reinterpret_cast<const uint64_t*>(in + i_off), cap,
                                  nullptr, nullptr, nullptr, pd, static_cast<int32_t*>(at(1)), pvalid, nullptr, nbk};
  q.v.dec.deep = static_cast<uint32_t*>(at(11));
  q.v.dec.deep_cap = (vs.off[12] - vs.off[11]) / 4;
  q.v.tree.B = cap;
  q.v.tree.digest_in = pd;
  q.v.tree.root_out = static_cast<uint8_t*>(at(5));
  q.v.tree.nodes_out = pnodes;
  q.v.tree.n_int = NI;
  q.v.diff = mde::DiffLaunch{(uint32_t)T, B, cap, d_dig, lnodes, pd, pnodes, pids, idcap, pst, R, nbk};
  q.v.fold = mde::VerifyLaunch{1, R, B, pst, pids, idcap, pvalid, replica_count, vdev,
                               reinterpret_cast<int32_t*>(out_d + 4), reinterpret_cast<int32_t*>(out_d + o_ids),
                               reinterpret_cast<int32_t*>(out_d + 8), out_d, reinterpret_cast<int32_t*>(out_d + o_st)};
  if (object_out)
    q.v.enc = mde::WireEncodeLaunch{1, B, reinterpret_cast<const int32_t*>(in + i_part), epoch, epoch + 1, d_dig,
                                    reinterpret_cast<const int32_t*>(in + i_size), vdev, nullptr, out_d + o_obj, ostride,
                                    reinterpret_cast<uint32_t*>(out_d + 12)};
  q.v.local.P = 1;
  q.v.local.B = B;
  q.v.local.digest_in = d_dig;
  q.v.local.root_out = static_cast<uint8_t*>(at(9));
  q.v.local.nodes_out = lnodes;
  q.v.local.n_int = mde::tree_internal(B);
  uint32_t vst = 0;
  (void)mde::verify_fused_lds(cap, &q.v_G, &q.v_words, &vst);
  q.v_stage = vst;
  q.v_deep = B > 64 ? 1u : 0u;
  q.stage = s->stage ? 1u : 0u;
  q.src = in_pin_d;
  q.dev_in = s->dev_in + (uint64_t)i * s->in_cap;
  q.stage_bytes = a16(in_bytes);
  std::memcpy(&s->slot(i)->r, &q, sizeof q);
  std::string msg;
  int rc = post_and_wait(s, i, &msg);
  if (rc == MDE_OK) {
    *valid = out_h[0];
    std::memcpy(valid_count, out_h + 4, 4);
    std::memcpy(diff_count, out_h + 8, 4);
    int32_t dc = 0;
    std::memcpy(&dc, out_h + 8, 4);
    if (dc > 0) std::memcpy(diff_ids, out_h + o_ids, (uint64_t)std::min<uint32_t>((uint32_t)dc, B) * 4);
    if (peer_status && R) std::memcpy(peer_status, out_h + o_st, (uint64_t)R * 4);
    if (object_out) {
      uint32_t len = 0;
      std::memcpy(&len, out_h + 12, 4);
      *object_len = len;
      std::memcpy(object_out, out_h + o_obj, std::min<uint64_t>(len, ostride));
    }
    give_slot(s, i);
  } else {  // the slot stays out of the free list; on the service's context (see server_build)
    mark_broken(s, msg);
    rc = on_context((msg + "; on the service's context: ").c_str());
  }
  return rc;
}

int mde_server_usable(mde_server* s) { return s && !s->broken.load() ? 1 : 0; }

int mde_server_disable(mde_server* s, const char* why) {
  if (!s) return MDE_E_INVAL;
  mark_broken(s, why && *why ? why : "disabled by the caller");
  // the idle slots' workgroups exit now; a slot serving a call exits when its caller gives it back
  std::lock_guard<std::mutex> lk(s->m);
  for (uint32_t i : s->free_slots) stop_idle_slot(s, i);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  return MDE_OK;
}

}  // extern "C"
