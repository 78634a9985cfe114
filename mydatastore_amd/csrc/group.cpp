// group.cpp -- device groups: one process driving the G GPUs of a node (include/mde.h mde_group_*).
//
// The reference spreads partitions over nodes with consistent hashing (hashring/hashring.go:126-154);
// a Go node is one process. Inside one MI355X node the engine spreads them over the node's GPUs:
// partition p lives on device p % G. Each device builds its own partitions --
// no data-path collective -- and the one exchange step, the per-partition roots, is ONE RCCL
// all-gather of fixed-size root slabs over xGMI, on communicators created once (ncclCommInitAll)
// with the group. RCCL is bound at run time (dlopen of librccl.so.1: torch's own copy carries the
// same SONAME, so a torch process shares one RCCL, and libmde has no link-time RCCL dependency).
// A group that lists a device more than once (several contexts on one GPU: the multi-device logic
// rehearsed on a one-GPU box) gathers with device copies instead -- the same bytes land in the same
// places -- and says so (mde_group_gather_kind).
//
// Written against the public C ABI plus HIP, like batch.cpp.
#include "../../include/mde.h"
#include "device_scope.hpp"
#include "enq_pool.hpp"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace {

// RCCL entry points, resolved once.
struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string why;  // empty when usable
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      x.why = std::string("librccl not loadable: ") + (e ? e : "?");
      return x;
    }
    x.init_all = reinterpret_cast<decltype(x.init_all)>(dlsym(h, "ncclCommInitAll"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(h, "ncclAllGather"));
    x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(h, "ncclGroupStart"));
    x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(h, "ncclGroupEnd"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    if (!x.init_all || !x.destroy || !x.all_gather || !x.group_start || !x.group_end || !x.error_string)
      x.why = "librccl lacks a required entry point";
    return x;
  }();
  return r;
}

struct Buf {
  void* p = nullptr;
  uint64_t cap = 0;
};

}  // namespace

struct mde_group {
  std::vector<int> dev;
  std::vector<mde_ctx*> ctx;
  std::vector<ncclComm_t> comm;   // one per device (empty: copy gather)
  std::vector<hipEvent_t> ready;  // each device's send buffer is ready (recorded on its context stream)
  std::vector<hipEvent_t> copied; // copy gather in stream order: device i's copies are done
  // overlapped gathers (mde_group_gather_overlapped_async): one side stream per device, and a ring
  // of kRing "gather done" events per device; ticket t uses ring slot t % kRing
  enum { kRing = 8 };
  std::vector<hipStream_t> side;
  std::vector<hipEvent_t> done;  // [slot * G + i]
  uint64_t next_ticket = 1;
  std::string gather_kind;
  std::mutex mu;  // held by the host-pointer builds for the whole call; guards err
  std::string err;
  // mde_multi_build staging, per device: values, value_off, seg_rec / part_rec, bucket_tag,
  // digest, size, items, root slab, nodes, gathered roots
  // mde_multi_build_streamed's two-slot ring per device: values, index arrays, value_off or tags
  enum { kVals, kVoff, kSeg, kTag, kDig, kSize, kItems, kRoot, kNodes, kRecv,
         kRingV0, kRingV1, kRingI0, kRingI1, kRingA0, kRingA1, kBufs };
  std::vector<std::vector<Buf>> stage;
  // and its copy stream + events per device (created on first use): [4 i + {loaded 0, loaded 1,
  // done 0, done 1}]
  std::vector<hipStream_t> copy;
  std::vector<hipEvent_t> ring_ev;
  // Per-device enqueue threads (run_all, enq_pool.hpp): devices 1..G-1 each have one; the calling
  // thread enqueues device 0's share. Started on the first device-resident call of a group of
  // G > 1 (MDE_GROUP_THREADS=0: the calling thread enqueues every device's share in turn).
  bool threaded = true;
  std::unique_ptr<mde::EnqPool> pool;
  std::mutex pool_mu;  // guards the pool's creation
};

namespace {

// Error messages go to `msg` (g->err, or a per-thread string while shards build concurrently).
int fail(std::string& msg, int code, const char* fmt, ...) {
  char m[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(m, sizeof m, fmt, ap);
  va_end(ap);
  msg = m;
  return code;
}

int grow(mde_group* g, uint32_t i, int which, uint64_t bytes, std::string& msg) {
  Buf& b = g->stage[i][which];
  if (b.p && b.cap >= bytes) return MDE_OK;
  (void)hipSetDevice(g->dev[i]);
  if (b.p) {
    (void)hipStreamSynchronize(static_cast<hipStream_t>(mde_get_stream(g->ctx[i])));
    (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
  }
  const uint64_t cap = std::max<uint64_t>(bytes + bytes / 8, 256);
  if (hipMalloc(&b.p, cap) != hipSuccess) {
    b.p = nullptr;
    return fail(msg, MDE_E_NOMEM, "device %d: staging allocation of %llu bytes failed", g->dev[i], (unsigned long long)cap);
  }
  b.cap = cap;
  return MDE_OK;
}

uint64_t parts_on(uint32_t P, uint32_t G, uint32_t i) { return i < P ? (uint64_t)(P - i + G - 1) / G : 0; }

// The one exchange step: device i contributes `bytes` from send[i]; recv[i] receives G slabs of
// `bytes`, slab r = device r's. Enqueued on every device's context stream.
int gather(mde_group* g, const void* const* send, void* const* recv, uint64_t bytes, std::string& msg) {
  const uint32_t G = (uint32_t)g->ctx.size();
  if (!g->comm.empty()) {
    const Rccl& r = rccl();
    ncclResult_t e = r.group_start();
    for (uint32_t i = 0; i < G && e == ncclSuccess; i++) {
      (void)hipSetDevice(g->dev[i]);
      e = r.all_gather(send[i], recv[i], bytes, ncclUint8, g->comm[i], static_cast<hipStream_t>(mde_get_stream(g->ctx[i])));
    }
    const ncclResult_t e2 = r.group_end();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(msg, MDE_E_DEVICE, "ncclAllGather: %s", r.error_string(e));
    return MDE_OK;
  }
  for (uint32_t i = 0; i < G; i++) {
    (void)hipSetDevice(g->dev[i]);
    if (hipEventRecord(g->ready[i], static_cast<hipStream_t>(mde_get_stream(g->ctx[i]))) != hipSuccess)
      return fail(msg, MDE_E_DEVICE, "hipEventRecord failed");
  }
  for (uint32_t i = 0; i < G; i++) {
    (void)hipSetDevice(g->dev[i]);
    hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[i]));
    for (uint32_t r = 0; r < G; r++) {
      if (hipStreamWaitEvent(st, g->ready[r], 0) != hipSuccess ||
          hipMemcpyAsync(static_cast<uint8_t*>(recv[i]) + (uint64_t)r * bytes, send[r], bytes, hipMemcpyDefault, st) !=
              hipSuccess)
        return fail(msg, MDE_E_DEVICE, "device copy gather failed");
    }
    if (hipEventRecord(g->copied[i], st) != hipSuccess) return fail(msg, MDE_E_DEVICE, "hipEventRecord failed");
  }
  // The collective's stream-order contract: work enqueued on stream r after the gather may rewrite
  // send[r] -- so stream r waits until every device's copies (which read send[r]) are done.
  for (uint32_t r = 0; r < G; r++) {
    (void)hipSetDevice(g->dev[r]);
    hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[r]));
    for (uint32_t i = 0; i < G; i++)
      if (i != r && hipStreamWaitEvent(st, g->copied[i], 0) != hipSuccess)
        return fail(msg, MDE_E_DEVICE, "hipStreamWaitEvent failed");
  }
  return MDE_OK;
}

// The exchange step off the build streams: device i's side stream waits for the send slabs'
// producers (the work already enqueued on the context streams: its own for RCCL, whose kernel on
// device i reads only send[i]; every device's for the copies, which read every send[r]), gathers,
// and records the ticket's ring event. The context streams go on with the next build at once.
int gather_overlapped(mde_group* g, const void* const* send, void* const* recv, uint64_t bytes, uint64_t* ticket,
                      std::string& msg) {
  const uint32_t G = (uint32_t)g->ctx.size();
  const uint64_t t = g->next_ticket++;
  const uint64_t slot = t % mde_group::kRing;
  for (uint32_t i = 0; i < G; i++) {
    (void)hipSetDevice(g->dev[i]);
    if (hipEventRecord(g->ready[i], static_cast<hipStream_t>(mde_get_stream(g->ctx[i]))) != hipSuccess)
      return fail(msg, MDE_E_DEVICE, "hipEventRecord failed");
  }
  if (!g->comm.empty()) {
    for (uint32_t i = 0; i < G; i++) {
      (void)hipSetDevice(g->dev[i]);
      if (hipStreamWaitEvent(g->side[i], g->ready[i], 0) != hipSuccess)
        return fail(msg, MDE_E_DEVICE, "hipStreamWaitEvent failed");
    }
    const Rccl& r = rccl();
    ncclResult_t e = r.group_start();
    for (uint32_t i = 0; i < G && e == ncclSuccess; i++) {
      (void)hipSetDevice(g->dev[i]);
      e = r.all_gather(send[i], recv[i], bytes, ncclUint8, g->comm[i], g->side[i]);
    }
    const ncclResult_t e2 = r.group_end();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) return fail(msg, MDE_E_DEVICE, "ncclAllGather: %s", r.error_string(e));
  } else {
    for (uint32_t i = 0; i < G; i++) {
      (void)hipSetDevice(g->dev[i]);
      for (uint32_t r = 0; r < G; r++) {
        if (hipStreamWaitEvent(g->side[i], g->ready[r], 0) != hipSuccess ||
            hipMemcpyAsync(static_cast<uint8_t*>(recv[i]) + (uint64_t)r * bytes, send[r], bytes, hipMemcpyDefault,
                           g->side[i]) != hipSuccess)
          return fail(msg, MDE_E_DEVICE, "device copy gather failed");
      }
    }
  }
  for (uint32_t i = 0; i < G; i++) {
    (void)hipSetDevice(g->dev[i]);
    if (hipEventRecord(g->done[slot * G + i], g->side[i]) != hipSuccess)
      return fail(msg, MDE_E_DEVICE, "hipEventRecord failed");
  }
  if (ticket) *ticket = t;
  return MDE_OK;
}

// Every context stream waits for gather `t`: RCCL -- device r's own side stream (its collective
// completes only after it has sent send[r] and received recv[r]); copies -- every side stream (each
// reads send[r]). A ticket whose ring slot a later gather re-recorded waits for that later gather:
// later in every side stream's order, so the wait is longer, never wrong.
int gather_wait(mde_group* g, uint64_t t, std::string& msg) {
  const uint32_t G = (uint32_t)g->ctx.size();
  if (!t || t >= g->next_ticket) return fail(msg, MDE_E_INVAL, "unknown gather ticket %llu", (unsigned long long)t);
  const uint64_t slot = t % mde_group::kRing;
  for (uint32_t r = 0; r < G; r++) {
    (void)hipSetDevice(g->dev[r]);
    hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[r]));
    for (uint32_t i = 0; i < G; i++) {
      if (!g->comm.empty() && i != r) continue;
      if (hipStreamWaitEvent(st, g->done[slot * G + i], 0) != hipSuccess)
        return fail(msg, MDE_E_DEVICE, "hipStreamWaitEvent failed");
    }
  }
  return MDE_OK;
}

// Host-side validation of a host-pointer build (the checks mde_build makes), before slicing.
int check(const mde_records* r, const mde_tree_out* o, std::string& msg) {
  if (!r || !o) return fail(msg, MDE_E_INVAL, "records or out is NULL");
  if (!r->n_buckets) return fail(msg, MDE_E_INVAL, "n_buckets must be >= 1");
  if (r->layout > MDE_LAYOUT_TAGGED) return fail(msg, MDE_E_INVAL, "unknown layout %u", r->layout);
  if ((uint64_t)r->n_partitions * r->n_buckets > 0xffffffffull)
    return fail(msg, MDE_E_INVAL, "n_partitions * n_buckets exceeds 2^32");
  if (!o->root && o->nodes) return fail(msg, MDE_E_INVAL, "out/nodes needs out/root");
  if (!r->values && r->values_bytes) return fail(msg, MDE_E_INVAL, "values is NULL");
  if (r->value_stride && (uint64_t)r->value_stride * r->n_records > r->values_bytes)
    return fail(msg, MDE_E_INVAL, "n_records * value_stride exceeds values_bytes");
  const uint32_t P = r->n_partitions, B = r->n_buckets;
  if (r->layout == MDE_LAYOUT_TAGGED) {
    if (!r->part_rec || (!r->bucket_tag && r->n_records)) return fail(msg, MDE_E_INVAL, "layout B needs part_rec and bucket_tag");
    if (!r->value_stride) return fail(msg, MDE_E_INVAL, "layout B needs fixed-length values");
    if (B > 65536) return fail(msg, MDE_E_INVAL, "layout B supports n_buckets <= 65536");
    for (uint32_t p = 0; p < P; p++)
      if (r->part_rec[p] > r->part_rec[p + 1]) return fail(msg, MDE_E_INVAL, "part_rec not nondecreasing");
    if (r->part_rec[P] > r->n_records) return fail(msg, MDE_E_INVAL, "part_rec exceeds n_records");
    for (uint64_t k = r->part_rec[0]; k < r->part_rec[P]; k++)
      if (r->bucket_tag[k] >= B) return fail(msg, MDE_E_INVAL, "bucket_tag[%llu] out of range", (unsigned long long)k);
    return MDE_OK;
  }
  if (!r->seg_rec) return fail(msg, MDE_E_INVAL, "seg_rec is NULL");
  if (!r->value_stride && !r->value_off && r->n_records) return fail(msg, MDE_E_INVAL, "variable-length values need value_off");
  const uint64_t S = (uint64_t)P * B;
  for (uint64_t s = 0; s < S; s++)
    if (r->seg_rec[s] > r->seg_rec[s + 1]) return fail(msg, MDE_E_INVAL, "seg_rec not nondecreasing at %llu", (unsigned long long)s);
  if (r->seg_rec[S] > r->n_records) return fail(msg, MDE_E_INVAL, "seg_rec[%llu] exceeds n_records", (unsigned long long)S);
  if (!r->value_stride && r->n_records) {
    for (uint64_t k = 0; k < r->n_records; k++)
      if (r->value_off[k] > r->value_off[k + 1]) return fail(msg, MDE_E_INVAL, "value_off not nondecreasing");
    if (r->value_off[r->n_records] > r->values_bytes) return fail(msg, MDE_E_INVAL, "value_off exceeds values_bytes");
  }
  return MDE_OK;
}

int ctx_err(mde_group* g, uint32_t i, int rc, std::string& msg) {
  char m[512];
  mde_last_error_copy(g->ctx[i], m, sizeof m);
  return fail(msg, rc, "member %u (device %d): %s", i, g->dev[i], m);
}

// fn(i) for every device i (fn returns an MDE code); the lowest failing device's code, or MDE_OK.
// Device i's share runs on its enqueue thread (enq_pool.hpp), device 0's on the caller.
int run_all(mde_group* g, const std::function<int(uint32_t)>& fn, uint32_t* failed) {
  const uint32_t G = (uint32_t)g->ctx.size();
  if (!g->threaded || G == 1) {
    for (uint32_t i = 0; i < G; i++) {
      const int rc = fn(i);
      if (rc) {
        *failed = i;
        return rc;
      }
    }
    return MDE_OK;
  }
  {
    std::lock_guard<std::mutex> lk(g->pool_mu);
    if (!g->pool) g->pool.reset(new mde::EnqPool(G));
  }
  return g->pool->run(fn, failed);
}

// A device-resident group call: fn(i) enqueues device i's share on its context (run_all: one host
// thread per device); a failure reports the lowest failing device's context message.
int group_call(mde_group* g, const std::function<int(uint32_t)>& fn) {
  uint32_t failed = 0;
  const int rc = run_all(g, fn, &failed);
  if (!rc) return MDE_OK;
  std::lock_guard<std::mutex> lk(g->mu);
  return ctx_err(g, failed, rc, g->err);
}

void stop_workers(mde_group* g) { g->pool.reset(); }

#define GHIP(expr)                                                                                   \
  do {                                                                                               \
    const hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(msg, MDE_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

// Waits for the given streams when it goes out of scope: a host-pointer entry point that returns
// early (an error) must not leave copies in flight from host vectors about to be freed.
struct StreamDrain {
  hipStream_t a, b;
  ~StreamDrain() {
    if (a) (void)hipStreamSynchronize(a);
    if (b) (void)hipStreamSynchronize(b);
  }
};

// Shard i of a host-pointer build: its partitions' records copied to device i (one copy per
// partition range: partition p's records are contiguous in the host arena), rebased, and the
// build enqueued on the device's context stream.
int upload_and_build(mde_group* g, uint32_t i, const mde_records* r, bool tree, bool want_nodes, uint64_t slab_parts,
                     std::string& msg) {
  const uint32_t G = (uint32_t)g->ctx.size(), P = r->n_partitions, B = r->n_buckets;
  const uint64_t Pi = parts_on(P, G, i);
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  const uint64_t NI = mde_tree_internal_nodes(B);
  auto pos = [&](uint64_t k) { return r->value_stride ? k * r->value_stride : r->value_off[k]; };
  auto first_rec = [&](uint64_t p) { return tagged ? r->part_rec[p] : r->seg_rec[p * B]; };
  uint64_t recs = 0, bytes = 0;
  for (uint64_t p = i; p < P; p += G) {
    recs += first_rec(p + 1) - first_rec(p);
    bytes += pos(first_rec(p + 1)) - pos(first_rec(p));
  }
  const uint64_t nseg = tagged ? Pi + 1 : Pi * B + 1;
  int rc;
  if ((rc = grow(g, i, mde_group::kVals, bytes + 16, msg)) || (rc = grow(g, i, mde_group::kSeg, nseg * 8, msg)) ||
      (!r->value_stride && (rc = grow(g, i, mde_group::kVoff, (recs + 1) * 8, msg))) ||
      (tagged && (rc = grow(g, i, mde_group::kTag, recs * 2 + 2, msg))) ||
      (rc = grow(g, i, mde_group::kDig, Pi * B * 8, msg)) || (rc = grow(g, i, mde_group::kSize, Pi * B * 4, msg)) ||
      (rc = grow(g, i, mde_group::kItems, Pi * 4, msg)) || (rc = grow(g, i, mde_group::kRoot, slab_parts * 32, msg)) ||
      (want_nodes && (rc = grow(g, i, mde_group::kNodes, Pi * NI * 32, msg))) ||
      (rc = grow(g, i, mde_group::kRecv, G * slab_parts * 32, msg)))
    return rc;
  auto dptr = [&](int k) { return static_cast<uint8_t*>(g->stage[i][k].p); };
  // host-side rebased index arrays
  std::vector<uint64_t> seg(nseg), voff(r->value_stride ? 0 : recs + 1);
  uint64_t rb = 0, bb = 0, k = 0;
  hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[i]));
  StreamDrain drain{st, nullptr};  // an early return waits for the copies from seg / voff
  GHIP(hipSetDevice(g->dev[i]));
  for (uint64_t p = i; p < P; p += G, k++) {
    const uint64_t r0 = first_rec(p), r1 = first_rec(p + 1), b0 = pos(r0), b1 = pos(r1);
    if (tagged) {
      seg[k] = rb;
    } else {
      for (uint32_t b = 0; b < B; b++) seg[k * B + b] = r->seg_rec[p * B + b] - r0 + rb;
    }
    if (!r->value_stride)
      for (uint64_t j = r0; j < r1; j++) voff[rb + j - r0] = r->value_off[j] - b0 + bb;
    if (b1 > b0) GHIP(hipMemcpyAsync(dptr(mde_group::kVals) + bb, r->values + b0, b1 - b0, hipMemcpyHostToDevice, st));
    if (tagged && r1 > r0)
      GHIP(hipMemcpyAsync(dptr(mde_group::kTag) + rb * 2, r->bucket_tag + r0, (r1 - r0) * 2, hipMemcpyHostToDevice, st));
    rb += r1 - r0;
    bb += b1 - b0;
  }
  seg[nseg - 1] = rb;
  if (!r->value_stride) voff[recs] = bb;
  GHIP(hipMemcpyAsync(dptr(mde_group::kSeg), seg.data(), nseg * 8, hipMemcpyHostToDevice, st));
  if (!r->value_stride) GHIP(hipMemcpyAsync(dptr(mde_group::kVoff), voff.data(), (recs + 1) * 8, hipMemcpyHostToDevice, st));
  // the root slab is fixed-size: rows past this shard's partitions stay zero
  if (tree) GHIP(hipMemsetAsync(dptr(mde_group::kRoot), 0, slab_parts * 32, st));
  mde_records dr{};
  dr.values = dptr(mde_group::kVals);
  dr.values_bytes = bb;
  dr.value_stride = r->value_stride;
  dr.layout = r->layout;
  dr.value_off = r->value_stride ? nullptr : reinterpret_cast<const uint64_t*>(dptr(mde_group::kVoff));
  dr.n_records = rb;
  dr.n_partitions = (uint32_t)Pi;
  dr.n_buckets = B;
  if (tagged) {
    dr.part_rec = reinterpret_cast<const uint64_t*>(dptr(mde_group::kSeg));
    dr.bucket_tag = reinterpret_cast<const uint16_t*>(dptr(mde_group::kTag));
  } else {
    dr.seg_rec = reinterpret_cast<const uint64_t*>(dptr(mde_group::kSeg));
  }
  mde_tree_out dout{reinterpret_cast<uint64_t*>(dptr(mde_group::kDig)), reinterpret_cast<int32_t*>(dptr(mde_group::kSize)),
                    reinterpret_cast<int32_t*>(dptr(mde_group::kItems)), tree ? dptr(mde_group::kRoot) : nullptr,
                    want_nodes ? dptr(mde_group::kNodes) : nullptr};
  // the host copies above must complete before the host vectors go out of scope
  GHIP(hipStreamSynchronize(st));
  rc = mde_build_async(g->ctx[i], &dr, &dout);
  return rc ? ctx_err(g, i, rc, msg) : MDE_OK;
}

// mde_multi_build_streamed's member i: its partitions i, i + G, ... streamed in chunks through a
// two-slot device ring (see there). Host index arrays are kept until the member is done (the
// copies from them are asynchronous).
int stream_member(mde_group* g, uint32_t i, const mde_records* r, const mde_tree_out* o, uint64_t chunk_bytes,
                  std::string& msg) {
  const uint32_t G = (uint32_t)g->ctx.size(), P = r->n_partitions, B = r->n_buckets;
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  const uint64_t NI = mde_tree_internal_nodes(B), Pi = parts_on(P, G, i);
  const bool nodes = o->nodes != nullptr;
  auto pos = [&](uint64_t k) { return r->value_stride ? k * r->value_stride : r->value_off[k]; };
  auto first_rec = [&](uint64_t p) { return tagged ? r->part_rec[p] : r->seg_rec[p * B]; };
  auto part = [&](uint64_t k) { return (uint64_t)i + k * G; };  // list entry k -> partition
  // chunks of list entries, ~chunk_bytes each (at least one partition)
  std::vector<uint64_t> cuts{0};
  uint64_t max_bytes = 0, max_recs = 0, max_parts = 0;
  for (uint64_t k = 0; k < Pi;) {
    uint64_t q = k, bytes = 0, recs = 0;
    do {
      const uint64_t p = part(q);
      bytes += pos(first_rec(p + 1)) - pos(first_rec(p));
      recs += first_rec(p + 1) - first_rec(p);
      q++;
    } while (q < Pi && bytes + pos(first_rec(part(q) + 1)) - pos(first_rec(part(q))) <= chunk_bytes);
    cuts.push_back(q);
    max_bytes = std::max(max_bytes, bytes);
    max_recs = std::max(max_recs, recs);
    max_parts = std::max(max_parts, q - k);
    k = q;
  }
  const uint64_t seg_per = tagged ? 1 : B;
  GHIP(hipSetDevice(g->dev[i]));
  hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[i]));
  // ring: 2 x (values, index, value_off or tags) and the member's outputs in list order, in the
  // group's grow-only staging; the copy stream and its events persist with the group
  const uint64_t aux_bytes = tagged ? max_recs * 2 + 16 : (r->value_stride ? 0 : (max_recs + 1) * 8);
  int rc;
  for (int s = 0; s < 2; s++)
    if ((rc = grow(g, i, mde_group::kRingV0 + s, max_bytes + 16, msg)) ||
        (rc = grow(g, i, mde_group::kRingI0 + s, (max_parts * seg_per + 1) * 8, msg)) ||
        (aux_bytes && (rc = grow(g, i, mde_group::kRingA0 + s, aux_bytes, msg))))
      return rc;
  if ((rc = grow(g, i, mde_group::kDig, Pi * B * 8, msg)) || (rc = grow(g, i, mde_group::kSize, Pi * B * 4, msg)) ||
      (rc = grow(g, i, mde_group::kItems, Pi * 4, msg)) || (rc = grow(g, i, mde_group::kRoot, Pi * 32, msg)) ||
      (nodes && (rc = grow(g, i, mde_group::kNodes, Pi * NI * 32, msg))))
    return rc;
  auto sp = [&](int k) { return g->stage[i][k].p; };
  void* vals[2] = {sp(mde_group::kRingV0), sp(mde_group::kRingV1)};
  void* idx[2] = {sp(mde_group::kRingI0), sp(mde_group::kRingI1)};
  void* aux[2] = {sp(mde_group::kRingA0), sp(mde_group::kRingA1)};
  GHIP(hipSetDevice(g->dev[i]));
  if (!g->copy[i]) {
    GHIP(hipStreamCreateWithFlags(&g->copy[i], hipStreamNonBlocking));
    for (int k = 0; k < 4; k++) GHIP(hipEventCreateWithFlags(&g->ring_ev[4 * i + k], hipEventDisableTiming));
  }
  hipStream_t cs = g->copy[i];
  hipEvent_t* loaded = &g->ring_ev[4 * i];
  hipEvent_t* done = &g->ring_ev[4 * i + 2];
  for (int s = 0; s < 2; s++) GHIP(hipEventRecord(done[s], st));
  std::vector<std::vector<uint64_t>> host_idx(cuts.size()), host_voff(cuts.size());
  // every return, an error one included, waits for the copies and builds issued from here: they
  // read host_idx / host_voff and the caller's arena
  StreamDrain drain{cs, st};
  for (size_t c = 0; c + 1 < cuts.size(); c++) {
    const int s = (int)(c & 1);
    const uint64_t k0 = cuts[c], k1 = cuts[c + 1];
    std::vector<uint64_t>& hi = host_idx[c];
    std::vector<uint64_t>& hv = host_voff[c];
    hi.resize((k1 - k0) * seg_per + 1);
    uint64_t rb = 0, bb = 0;
    GHIP(hipStreamWaitEvent(cs, done[s], 0));  // the build two chunks back released this slot
    for (uint64_t k = k0; k < k1; k++) {
      const uint64_t p = part(k), r0 = first_rec(p), r1 = first_rec(p + 1), b0 = pos(r0), b1 = pos(r1);
      if (tagged) {
        hi[k - k0] = rb;
      } else {
        for (uint32_t b = 0; b < B; b++) hi[(k - k0) * B + b] = r->seg_rec[p * B + b] - r0 + rb;
      }
      if (!r->value_stride && !tagged)
        for (uint64_t j = r0; j < r1; j++) hv.push_back(r->value_off[j] - b0 + bb);
      if (b1 > b0)
        GHIP(hipMemcpyAsync(static_cast<uint8_t*>(vals[s]) + bb, r->values + b0, b1 - b0, hipMemcpyHostToDevice, cs));
      if (tagged && r1 > r0)
        GHIP(hipMemcpyAsync(static_cast<uint8_t*>(aux[s]) + rb * 2, r->bucket_tag + r0, (r1 - r0) * 2,
                            hipMemcpyHostToDevice, cs));
      rb += r1 - r0;
      bb += b1 - b0;
    }
    hi.back() = rb;
    GHIP(hipMemcpyAsync(idx[s], hi.data(), hi.size() * 8, hipMemcpyHostToDevice, cs));
    if (!r->value_stride && !tagged) {
      hv.push_back(bb);
      GHIP(hipMemcpyAsync(aux[s], hv.data(), hv.size() * 8, hipMemcpyHostToDevice, cs));
    }
    GHIP(hipEventRecord(loaded[s], cs));
    GHIP(hipStreamWaitEvent(st, loaded[s], 0));
    mde_records dr{};
    dr.values = static_cast<const uint8_t*>(vals[s]);
    dr.values_bytes = bb;
    dr.value_stride = r->value_stride;
    dr.layout = r->layout;
    dr.value_off = (r->value_stride || tagged) ? nullptr : static_cast<const uint64_t*>(aux[s]);
    dr.n_records = rb;
    dr.n_partitions = (uint32_t)(k1 - k0);
    dr.n_buckets = B;
    if (tagged) {
      dr.part_rec = static_cast<const uint64_t*>(idx[s]);
      dr.bucket_tag = static_cast<const uint16_t*>(aux[s]);
    } else {
      dr.seg_rec = static_cast<const uint64_t*>(idx[s]);
    }
    mde_tree_out dout{static_cast<uint64_t*>(sp(mde_group::kDig)) + k0 * B,
                      static_cast<int32_t*>(sp(mde_group::kSize)) + k0 * B,
                      static_cast<int32_t*>(sp(mde_group::kItems)) + k0,
                      static_cast<uint8_t*>(sp(mde_group::kRoot)) + k0 * 32,
                      nodes ? static_cast<uint8_t*>(sp(mde_group::kNodes)) + k0 * NI * 32 : nullptr};
    if ((rc = mde_build_async(g->ctx[i], &dr, &dout))) return ctx_err(g, i, rc, msg);
    GHIP(hipEventRecord(done[s], st));
  }
  // the member's outputs home in list order, then to partition order
  std::vector<uint8_t> h;
  auto home = [&](const void* src, uint64_t row_bytes, uint8_t* dst) -> int {
    h.resize(Pi * row_bytes);
    GHIP(hipMemcpyAsync(h.data(), src, Pi * row_bytes, hipMemcpyDeviceToHost, st));
    GHIP(hipStreamSynchronize(st));
    for (uint64_t k = 0; k < Pi; k++) std::memcpy(dst + part(k) * row_bytes, h.data() + k * row_bytes, row_bytes);
    return MDE_OK;
  };
  if (o->digest && (rc = home(sp(mde_group::kDig), (uint64_t)B * 8, reinterpret_cast<uint8_t*>(o->digest)))) return rc;
  if (o->size && (rc = home(sp(mde_group::kSize), (uint64_t)B * 4, reinterpret_cast<uint8_t*>(o->size)))) return rc;
  if (o->items && (rc = home(sp(mde_group::kItems), 4, reinterpret_cast<uint8_t*>(o->items)))) return rc;
  if ((rc = home(sp(mde_group::kRoot), 32, o->root))) return rc;
  if (nodes && (rc = home(sp(mde_group::kNodes), NI * 32, o->nodes))) return rc;
  GHIP(hipStreamSynchronize(cs));
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_group_create(const int* devices, uint32_t n, mde_group** out) {
  if (!out) return MDE_E_INVAL;
  *out = nullptr;
  if (!devices || !n) return MDE_E_INVAL;
  DeviceScope keep(devices[0]);  // every hipSetDevice below undone on return
  mde_group* g = new (std::nothrow) mde_group();
  if (!g) return MDE_E_NOMEM;
  for (uint32_t i = 0; i < n; i++) {
    mde_ctx* c = nullptr;
    const int rc = mde_create(devices[i], &c);
    if (rc != MDE_OK) {
      mde_group_destroy(g);
      return rc;
    }
    g->ctx.push_back(c);
    g->dev.push_back(devices[i]);
  }
  g->stage.assign(n, std::vector<Buf>(mde_group::kBufs));
  if (const char* e = std::getenv("MDE_GROUP_THREADS")) g->threaded = std::atoi(e) != 0;
  std::vector<int> sorted(g->dev);
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  const char* force = std::getenv("MDE_GROUP_GATHER");  // "copy": device copies even on distinct GPUs
  const bool want_rccl = distinct && !(force && !std::strcmp(force, "copy"));
  if (want_rccl && rccl().why.empty()) {
    g->comm.assign(n, nullptr);
    const ncclResult_t e = rccl().init_all(g->comm.data(), (int)n, g->dev.data());
    if (e != ncclSuccess) {
      g->comm.clear();
      g->gather_kind = std::string("device copies (ncclCommInitAll failed: ") + rccl().error_string(e) + ")";
    } else {
      g->gather_kind = "rccl all_gather";
    }
  } else {
    g->gather_kind = !distinct ? "device copies (a device listed twice)"
                     : want_rccl ? "device copies (" + rccl().why + ")" : "device copies (MDE_GROUP_GATHER=copy)";
  }
  g->ready.assign(n, nullptr);
  g->copied.assign(n, nullptr);
  g->side.assign(n, nullptr);
  g->copy.assign(n, nullptr);
  g->ring_ev.assign(4 * (size_t)n, nullptr);
  g->done.assign((size_t)mde_group::kRing * n, nullptr);
  for (uint32_t i = 0; i < n; i++) {
    (void)hipSetDevice(g->dev[i]);
    bool ok = hipEventCreateWithFlags(&g->ready[i], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&g->copied[i], hipEventDisableTiming) == hipSuccess &&
              hipStreamCreateWithFlags(&g->side[i], hipStreamNonBlocking) == hipSuccess;
    for (uint32_t k = 0; ok && k < mde_group::kRing; k++)
      ok = hipEventCreateWithFlags(&g->done[k * n + i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
      mde_group_destroy(g);
      return MDE_E_DEVICE;
    }
  }
  *out = g;
  return MDE_OK;
}

void mde_group_destroy(mde_group* g) {
  if (!g) return;
  stop_workers(g);
  DeviceScope keep(g->dev.empty() ? 0 : g->dev[0]);
  for (mde_ctx* c : g->ctx) (void)mde_synchronize(c);
  for (size_t i = 0; i < g->side.size(); i++)
    if (g->side[i]) {
      (void)hipSetDevice(g->dev[i]);
      (void)hipStreamSynchronize(g->side[i]);
    }
  for (ncclComm_t c : g->comm)
    if (c) (void)rccl().destroy(c);
  const size_t n = g->dev.size();
  for (size_t i = 0; i < g->ready.size(); i++) {
    (void)hipSetDevice(g->dev[i]);
    if (i < g->copy.size() && g->copy[i]) {
      (void)hipStreamSynchronize(g->copy[i]);
      (void)hipStreamDestroy(g->copy[i]);
    }
    for (size_t k = 0; k < 4 && 4 * i + k < g->ring_ev.size(); k++)
      if (g->ring_ev[4 * i + k]) (void)hipEventDestroy(g->ring_ev[4 * i + k]);
    if (g->ready[i]) (void)hipEventDestroy(g->ready[i]);
    if (i < g->copied.size() && g->copied[i]) (void)hipEventDestroy(g->copied[i]);
    for (size_t k = 0; k < mde_group::kRing && k * n + i < g->done.size(); k++)
      if (g->done[k * n + i]) (void)hipEventDestroy(g->done[k * n + i]);
    if (i < g->side.size() && g->side[i]) (void)hipStreamDestroy(g->side[i]);
  }
  for (size_t i = 0; i < g->stage.size(); i++) {
    (void)hipSetDevice(g->dev[i]);
    for (Buf& b : g->stage[i])
      if (b.p) (void)hipFree(b.p);
  }
  for (mde_ctx* c : g->ctx) mde_destroy(c);
  delete g;
}

uint32_t mde_group_size(const mde_group* g) { return g ? (uint32_t)g->ctx.size() : 0u; }

mde_ctx* mde_group_ctx(mde_group* g, uint32_t i) { return g && i < g->ctx.size() ? g->ctx[i] : nullptr; }

const char* mde_group_gather_kind(const mde_group* g) { return g ? g->gather_kind.c_str() : "null group"; }

uint32_t mde_group_partitions(const mde_group* g, uint32_t n_partitions, uint32_t i) {
  return g && i < g->ctx.size() ? (uint32_t)parts_on(n_partitions, (uint32_t)g->ctx.size(), i) : 0u;
}

const char* mde_group_last_error(const mde_group* g) { return g ? g->err.c_str() : "null group"; }

uint64_t mde_group_last_error_copy(mde_group* g, char* buf, uint64_t cap) {
  std::string m = "null group";
  if (g) {
    std::lock_guard<std::mutex> lk(g->mu);
    m = g->err;
  }
  if (buf && cap) {
    const uint64_t k = std::min<uint64_t>(m.size(), cap - 1);
    std::memcpy(buf, m.data(), k);
    buf[k] = 0;
  }
  return m.size();
}

int mde_group_build_async(mde_group* g, const mde_records* shard, const mde_tree_out* shard_out) {
  if (!g || !shard || !shard_out) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  return group_call(g, [&](uint32_t i) {
    return shard[i].n_partitions ? mde_build_async(g->ctx[i], &shard[i], &shard_out[i]) : MDE_OK;
  });
}

int mde_group_build_pipelined_async(mde_group* g, const mde_records* shard, const mde_tree_out* shard_out) {
  if (!g || !shard || !shard_out) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  return group_call(g, [&](uint32_t i) {
    return shard[i].n_partitions ? mde_build_pipelined_async(g->ctx[i], &shard[i], &shard_out[i]) : MDE_OK;
  });
}

int mde_group_build_pipeline_drain_async(mde_group* g) {
  if (!g) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  return group_call(g, [&](uint32_t i) { return mde_build_pipeline_drain_async(g->ctx[i]); });
}

int mde_group_gather_async(mde_group* g, const void* const* send, void* const* recv, uint64_t bytes) {
  if (!g || !send || !recv) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  std::lock_guard<std::mutex> lk(g->mu);
  return gather(g, send, recv, bytes, g->err);
}

int mde_group_gather_overlapped_async(mde_group* g, const void* const* send, void* const* recv, uint64_t bytes,
                                      uint64_t* ticket) {
  if (!g || !send || !recv) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  std::lock_guard<std::mutex> lk(g->mu);
  return gather_overlapped(g, send, recv, bytes, ticket, g->err);
}

int mde_group_gather_wait_async(mde_group* g, uint64_t ticket) {
  if (!g) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  std::lock_guard<std::mutex> lk(g->mu);
  return gather_wait(g, ticket, g->err);
}

int mde_group_diff_async(mde_group* g, const mde_diff_args* shard) {
  if (!g || !shard) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  return group_call(g, [&](uint32_t i) {
    const mde_diff_args& a = shard[i];
    return a.n_pairs ? mde_diff_async(g->ctx[i], a.n_pairs, a.n_buckets_a, a.digest_a, a.nodes_a, a.n_buckets_b,
                                      a.digest_b, a.nodes_b, a.out_ids, a.out_stride, a.out_count)
                     : MDE_OK;
  });
}

int mde_group_extract_async(mde_group* g, const mde_records* shard, const mde_extract_args* args) {
  if (!g || !shard || !args) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  return group_call(g, [&](uint32_t i) {
    const mde_extract_args& a = args[i];
    return shard[i].n_partitions
               ? mde_extract_async(g->ctx[i], &shard[i], a.ids, a.ids_stride, a.counts, a.part_off, a.out_rec,
                                   a.rec_cap, a.out_values, a.out_value_off, a.bytes_cap, a.status)
               : MDE_OK;
  });
}

int mde_group_synchronize(mde_group* g) {
  if (!g) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  for (uint32_t i = 0; i < g->ctx.size(); i++) {
    const int rc = mde_synchronize(g->ctx[i]);
    if (rc) {
      std::lock_guard<std::mutex> lk(g->mu);
      return ctx_err(g, i, rc, g->err);
    }
  }
  for (uint32_t i = 0; i < g->side.size(); i++) {
    (void)hipSetDevice(g->dev[i]);
    const hipError_t e = hipStreamSynchronize(g->side[i]);
    if (e != hipSuccess) {
      std::lock_guard<std::mutex> lk(g->mu);
      return fail(g->err, MDE_E_DEVICE, "device %d: gather stream: %s", g->dev[i], hipGetErrorString(e));
    }
  }
  return MDE_OK;
}

int mde_multi_build(mde_group* g, const mde_records* r, const mde_tree_out* o) {
  if (!g || g->ctx.empty()) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  std::lock_guard<std::mutex> lk(g->mu);
  g->err.clear();
  std::string& msg = g->err;
  int rc = check(r, o, msg);
  if (rc) return rc;
  const uint32_t G = (uint32_t)g->ctx.size(), P = r->n_partitions, B = r->n_buckets;
  if (!P) return MDE_OK;
  const uint64_t NI = mde_tree_internal_nodes(B), slab = (P + G - 1) / G;
  const bool tree = o->root != nullptr, nodes = o->nodes != nullptr;
  // every shard's copies and build, concurrently (one host thread per device: pageable copies
  // block the calling thread)
  std::vector<int> rcs(G, MDE_OK);
  std::vector<std::string> errs(G);
  {
    std::vector<std::thread> th;
    for (uint32_t i = 0; i < G && i < P; i++)
      th.emplace_back([&, i] { rcs[i] = upload_and_build(g, i, r, tree, nodes, slab, errs[i]); });
    for (auto& t : th) t.join();
  }
  for (uint32_t i = 0; i < G; i++)
    if (rcs[i]) {
      g->err = errs[i];
      return rcs[i];
    }
  // the exchange step: every device's root slab to every device (device 0's copy comes home)
  std::vector<const void*> send(G);
  std::vector<void*> recv(G);
  for (uint32_t i = 0; i < G; i++) {
    if ((rc = grow(g, i, mde_group::kRoot, slab * 32, msg)) || (rc = grow(g, i, mde_group::kRecv, G * slab * 32, msg)))
      return rc;
    send[i] = g->stage[i][mde_group::kRoot].p;
    recv[i] = g->stage[i][mde_group::kRecv].p;
    if (i >= P) {  // a device without partitions still takes part with a zero slab
      (void)hipSetDevice(g->dev[i]);
      GHIP(hipMemsetAsync(g->stage[i][mde_group::kRoot].p, 0, slab * 32,
                          static_cast<hipStream_t>(mde_get_stream(g->ctx[i]))));
    }
  }
  if (tree && (rc = gather(g, send.data(), recv.data(), slab * 32, msg))) return rc;
  // results home, in partition order
  std::vector<uint8_t> h;
  for (uint32_t i = 0; i < G && i < P; i++) {
    const uint64_t Pi = parts_on(P, G, i);
    hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[i]));
    GHIP(hipSetDevice(g->dev[i]));
    auto home = [&](int which, uint64_t row_bytes, uint8_t* dst) -> int {
      h.resize(Pi * row_bytes);
      GHIP(hipMemcpyAsync(h.data(), g->stage[i][which].p, Pi * row_bytes, hipMemcpyDeviceToHost, st));
      GHIP(hipStreamSynchronize(st));
      for (uint64_t k = 0; k < Pi; k++) std::memcpy(dst + (i + k * G) * row_bytes, h.data() + k * row_bytes, row_bytes);
      return MDE_OK;
    };
    if (o->digest && (rc = home(mde_group::kDig, (uint64_t)B * 8, reinterpret_cast<uint8_t*>(o->digest)))) return rc;
    if (o->size && (rc = home(mde_group::kSize, (uint64_t)B * 4, reinterpret_cast<uint8_t*>(o->size)))) return rc;
    if (o->items && (rc = home(mde_group::kItems, 4, reinterpret_cast<uint8_t*>(o->items)))) return rc;
    if (nodes && (rc = home(mde_group::kNodes, NI * 32, o->nodes))) return rc;
  }
  if (tree) {  // the gathered slabs on device 0: slab r row k = partition r + k * G
    h.resize(G * slab * 32);
    hipStream_t st = static_cast<hipStream_t>(mde_get_stream(g->ctx[0]));
    GHIP(hipSetDevice(g->dev[0]));
    GHIP(hipMemcpyAsync(h.data(), g->stage[0][mde_group::kRecv].p, G * slab * 32, hipMemcpyDeviceToHost, st));
    GHIP(hipStreamSynchronize(st));
    for (uint32_t rr = 0; rr < G; rr++)
      for (uint64_t k = 0; k < slab; k++) {
        const uint64_t p = rr + k * G;
        if (p < P) std::memcpy(o->root + p * 32, h.data() + (rr * slab + k) * 32, 32);
      }
  }
  for (uint32_t i = 0; i < G; i++) {
    (void)hipSetDevice(g->dev[i]);
    GHIP(hipStreamSynchronize(static_cast<hipStream_t>(mde_get_stream(g->ctx[i]))));
  }
  return MDE_OK;
}

// Host ingest over the group (arenas larger than HBM): nothing stays resident. Partition p goes to
// member p % G, the placement of every other group entry point (mde_multi_build, the
// device-resident calls, mde_group_partitions). Member i streams its partitions i, i + G, ... in
// chunks of about chunk_bytes through a two-slot device ring on its own thread: a copy stream
// packs chunk k's partitions back to back into slot k % 2 -- one host-to-device copy per partition
// range (a partition's records are contiguous in the host arena) plus the chunk's rebased index
// arrays -- while the context stream builds chunk k - 1 from the other slot. The member's outputs
// collect on its device in list order and come home once, scattered to partition order. Same
// results as mde_multi_build.
int mde_multi_build_streamed(mde_group* g, const mde_records* r, const mde_tree_out* o, uint64_t chunk_bytes) {
  if (!g || g->ctx.empty()) return MDE_E_INVAL;
  DeviceScope keep(g->dev[0]);
  std::lock_guard<std::mutex> lk(g->mu);
  g->err.clear();
  int rc = check(r, o, g->err);
  if (rc) return rc;
  if (!o->root) return fail(g->err, MDE_E_INVAL, "out/root is NULL");
  if (!chunk_bytes) chunk_bytes = 256ull << 20;
  const uint32_t G = (uint32_t)g->ctx.size(), P = r->n_partitions;
  std::vector<int> rcs(G, MDE_OK);
  std::vector<std::string> errs(G);
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < G && i < P; i++)
    th.emplace_back([&, i] { rcs[i] = stream_member(g, i, r, o, chunk_bytes, errs[i]); });
  for (auto& t : th) t.join();
  for (uint32_t i = 0; i < G; i++)
    if (rcs[i]) {
      g->err = errs[i];
      return rcs[i];
    }
  return MDE_OK;
}

}  // extern "C"
