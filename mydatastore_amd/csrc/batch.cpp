// batch.cpp -- request coalescing for the production call shape (mde_batcher, include/mde.h).
//
// The reference builds ONE partition per call: Manager.VerifyEpoch (main/manager.go:998-1118)
// runs RawPartitionMerkleTree(p, E, E+1) and the peer decision for a single (partition, epoch) on
// any of workers_count = 100 goroutines, with up to partition_concurrency = 10 verifies in flight
// (config/default-config.yaml:7,9; main/manager.go:68,166-170,489-497). A synchronous mde_build
// per partition pays a whole device round trip -- copies, launches and the tree's dependent
// SHA-256 chain -- for a few KB of 8-byte timestamps. The batcher turns concurrent calls into one
// device build by group commit:
//   * a caller validates its request on its own thread and enqueues it;
//   * if no batch is being taken it becomes the leader: it takes every compatible queued request
//     (up to max_partitions partitions; optionally waiting up to max_wait_us for more to arrive)
//     into a free slot, passes the leader role on at once (the next leader takes the next batch
//     while this one stages), packs their records into ONE pinned arena, runs ONE H2D copy and
//     mde_build_async (or mde_verify_epochs_async with the local trees given by their digests) on
//     the slot's context, waits for the batch's event and marks its callers ready;
//   * each ready caller copies its own outputs out of the slot's pinned buffer on its own thread
//     (100 callers' nodes are ~0.7 MB of copies: spread over their threads, not the leader's), and
//     the last one frees the slot;
//   * up to mde_batcher_contexts() batches are in flight at once (one context, stream and staging
//     area per slot), so staging, copies and launches overlap the earlier batches' device work,
//     and a finished batch wakes only its own callers (one condition variable per request: no
//     thundering herd at 100 callers).
// Liveness: a leader hands the role on right after taking its batch, and the caller that frees a
// slot hands it on again, so a queued request is picked up by the next free slot even when the
// request it was handed the role to has meanwhile finished inside another batch.
// mde_batcher_destroy must not race with calls in flight (like mde_destroy).
// Each caller gets exactly what the per-call entry point returns for its own inputs (bit-exact:
// a partition's digests, sizes and tree depend only on its own records; tests/cpp/batch_test.c
// checks it against mde_build / mde_verify_epochs and the C oracle under concurrent callers).
//
// Written against the public C ABI plus HIP memory calls only, like any other client of mde.h.
#include "../../include/mde.h"
#include "device_scope.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
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
#include <vector>

namespace {

enum class Kind { Build, Verify };

struct Req {
  Kind kind = Kind::Build;
  uint32_t parts = 1;  // partitions this request adds to a batch
  uint64_t key[4] = {0, 0, 0, 0};
  // RawPartitionMerkleTree (layout A, host pointers)
  mde_records rec{};
  mde_tree_out out{};
  uint64_t r0 = 0, r1 = 0;  // records actually in buckets: [seg_rec[0], seg_rec[P*B])
  uint64_t b0 = 0, b1 = 0;  // their bytes
  // VerifyEpoch decision step (one partition)
  uint32_t B = 0, R = 0, replica_count = 0;
  int32_t partition = 0;
  int64_t epoch = 0;
  const uint64_t* digest = nullptr;
  const int32_t* size = nullptr;
  const uint8_t* peer_bytes = nullptr;
  const uint64_t* peer_off = nullptr;
  uint8_t* valid = nullptr;
  int32_t *valid_count = nullptr, *diff_ids = nullptr, *diff_count = nullptr, *peer_status = nullptr;
  uint8_t* object_out = nullptr;
  uint32_t* object_len = nullptr;
  // result
  int rc = MDE_OK;
  char* err = nullptr;
  uint64_t err_cap = 0;
  bool done = false;
  bool lead = false;   // handed the leader role for the next batch
  bool ready = false;  // its batch finished on the device: copy its own outputs out, then done
  void* slot = nullptr;  // the mde_batcher::Slot its batch ran in
  uint64_t pos = 0;      // build: its first partition in the batch; verify: its index
  std::chrono::steady_clock::time_point lead_t;  // when it was handed the role (MDE_BATCH_PROFILE)
  std::condition_variable cv;
};

void put_msg(char* buf, uint64_t cap, const char* msg) {
  if (!buf || !cap) return;
  const uint64_t n = std::min<uint64_t>(std::strlen(msg), cap - 1);
  std::memcpy(buf, msg, n);
  buf[n] = 0;
}

int fail(Req* q, int code, const char* fmt, ...) {
  char m[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(m, sizeof m, fmt, ap);
  va_end(ap);
  put_msg(q->err, q->err_cap, m);
  q->rc = code;
  return code;
}

struct Buf {
  void* p = nullptr;
  uint64_t cap = 0;
};

uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

// A batch between its launch and the last of its callers' copies: the output layout in the slot's
// pinned out buffer, which stays the batch's until every caller has copied its part out.
struct Batch {
  std::vector<Req*> v;
  bool launched = false;  // device work enqueued (else every request already failed)
  uint32_t B = 0;
  uint64_t NI = 0, stride = 0, R = 0;
  uint64_t o[9] = {0};   // output offsets in the slot's pinned out buffer
  size_t pending = 0;    // callers still copying their outputs out
};

}  // namespace

// Batches in flight at once. Each slot owns a context -- its own stream and scratch -- so the
// device runs several batches concurrently (a batch of small partitions is a few workgroups whose
// time is the tree's dependent SHA-256 chain, so batches overlap instead of queueing on one
// stream). Default 4 = GPU_MAX_HW_QUEUES, the HIP runtime's hardware queues per process;
// MDE_BATCH_SLOTS=1..8 overrides it (A/B).
constexpr int kMaxSlots = 8;
constexpr int kDefaultSlots = 4;

struct mde_batcher {
  int device = 0;
  uint32_t max_parts = 256;
  uint32_t max_wait_us = 0;
  std::mutex m;
  std::condition_variable collect;  // a collecting leader waits here for more requests
  std::deque<Req*> q;
  bool leading = false;  // a leader is taking / staging / launching a batch
  struct Slot {
    mde_ctx* ctx = nullptr;  // own stream + scratch
    Buf pin_in, pin_out, dev_in, dev_out;
    hipEvent_t done = nullptr;
    bool busy = false;
    Batch bt;
  } slots[kMaxSlots];
  int n_slots = kDefaultSlots;
  uint64_t n_batches = 0, n_requests = 0, n_partitions = 0;
  // write-once outputs stored by the kernels straight into the slot's pinned out buffer (no D2H
  // copy; above ~16 KB such a copy starts ~11 us after the kernel, profiles/r03q_call_trace.txt);
  // MDE_DIRECT_OUT=0 turns it off (A/B)
  bool direct_out = true;
  // inputs of a small batch read by the kernels straight from the slot's pinned in buffer (no H2D
  // copy command: at one small partition the copy, its gap to the kernel and its host call cost
  // more than reading ~10 KB over PCIe); MDE_DIRECT_IN=0/1 overrides (A/B)
  bool direct_in = false;
  bool blocking_sync = false;  // MDE_BATCH_BLOCKING_SYNC=1: leaders sleep on their batch's event (A/B)
  // MDE_BATCH_PROFILE=1: host-side phase times summed over batches, printed by mde_batcher_destroy
  bool profile = false;
  bool early_handoff = true;  // MDE_BATCH_EARLY=0: pass the leader role on only after the launch (A/B)
  double t_handoff = 0, t_stage = 0, t_device = 0, t_scatter = 0;
  uint64_t n_handoff = 0;
};

namespace {

int grow(Buf& x, uint64_t bytes, bool pinned, std::string* msg) {
  if (x.p && x.cap >= bytes) return MDE_OK;
  if (x.p) {
    if (pinned) (void)hipHostFree(x.p);
    else (void)hipFree(x.p);
    x.p = nullptr;
    x.cap = 0;
  }
  uint64_t cap = std::max<uint64_t>(bytes, 1 << 16);
  cap += cap / 4;  // grow-only, with headroom: batch sizes vary call to call
  const hipError_t e = pinned ? hipHostMalloc(&x.p, cap, hipHostMallocDefault) : hipMalloc(&x.p, cap);
  if (e != hipSuccess) {
    x.p = nullptr;
    *msg = std::string(pinned ? "pinned" : "device") + " staging allocation of " + std::to_string(cap) +
           " bytes failed";
    return MDE_E_NOMEM;
  }
  x.cap = cap;
  return MDE_OK;
}

// Host-side validation of one build request (the checks mde_build makes), on the caller's thread.
int check_build(Req* q) {
  const mde_records* r = &q->rec;
  if (r->layout != MDE_LAYOUT_SORTED) return fail(q, MDE_E_INVAL, "mde_batch_build takes layout A records");
  if (!r->seg_rec || !r->n_buckets || !r->n_partitions)
    return fail(q, MDE_E_INVAL, "seg_rec, n_buckets and n_partitions are required");
  if (!q->out.root && q->out.nodes) return fail(q, MDE_E_INVAL, "out/nodes needs out/root");
  if ((uint64_t)r->n_partitions * r->n_buckets > 0xffffffffull)
    return fail(q, MDE_E_INVAL, "n_partitions * n_buckets exceeds 2^32");
  if (r->value_stride == 0 && !r->value_off && r->n_records)
    return fail(q, MDE_E_INVAL, "variable-length values need value_off");
  if (!r->values && r->values_bytes) return fail(q, MDE_E_INVAL, "values is NULL");
  if (r->value_stride && (uint64_t)r->value_stride * r->n_records > r->values_bytes)
    return fail(q, MDE_E_INVAL, "n_records * value_stride exceeds values_bytes");
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  for (uint64_t s = 0; s < S; s++)
    if (r->seg_rec[s] > r->seg_rec[s + 1])
      return fail(q, MDE_E_INVAL, "seg_rec not nondecreasing at %llu", (unsigned long long)s);
  if (r->seg_rec[S] > r->n_records) return fail(q, MDE_E_INVAL, "seg_rec[%llu] exceeds n_records", (unsigned long long)S);
  if (!r->value_stride && r->n_records) {
    for (uint64_t i = 0; i < r->n_records; i++)
      if (r->value_off[i] > r->value_off[i + 1])
        return fail(q, MDE_E_INVAL, "value_off not nondecreasing at %llu", (unsigned long long)i);
    if (r->value_off[r->n_records] > r->values_bytes)
      return fail(q, MDE_E_INVAL, "value_off[n_records] exceeds values_bytes");
  }
  q->r0 = r->seg_rec[0];
  q->r1 = r->seg_rec[S];
  q->b0 = r->value_stride ? q->r0 * r->value_stride : (r->n_records ? r->value_off[q->r0] : 0);
  q->b1 = r->value_stride ? q->r1 * r->value_stride : (r->n_records ? r->value_off[q->r1] : 0);
  q->parts = r->n_partitions;
  q->key[0] = 1;
  q->key[1] = r->n_buckets;
  q->key[2] = q->out.root ? 1 : 0;  // digest-only builds (root NULL) batch apart: no tree latency
  return MDE_OK;
}

bool same_key(const Req* a, const Req* b) { return std::memcmp(a->key, b->key, sizeof a->key) == 0; }

// The leader's batch: its own request first (still queued: a leader only leads for its own
// request, so the batch it then waits for is the one its outputs come from; alone it may exceed
// max_parts), then every other compatible queued request in arrival order while the batch stays
// within max_parts (and, for builds, within 2^32 buckets in all: mde_build's limit on
// n_partitions * n_buckets, which every request already meets on its own).
std::vector<Req*> take(mde_batcher* b, Req* first) {
  std::vector<Req*> out{first};
  const uint64_t per_part = first->kind == Kind::Build ? first->rec.n_buckets : 1;
  uint64_t parts = first->parts;
  const auto self = std::find(b->q.begin(), b->q.end(), first);
  if (self != b->q.end()) b->q.erase(self);
  for (auto it = b->q.begin(); it != b->q.end();) {
    Req* x = *it;
    if (same_key(x, first) && parts + x->parts <= b->max_parts && (parts + x->parts) * per_part <= 0xffffffffull) {
      out.push_back(x);
      parts += x->parts;
      it = b->q.erase(it);
    } else {
      ++it;
    }
  }
  return out;
}

void fail_all(const std::vector<Req*>& v, int code, const std::string& msg) {
  for (Req* x : v) fail(x, code, "%s", msg.c_str());
}

#define BHIP(expr)                                                                               \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) {                                                                      \
      fail_all(v, MDE_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));              \
      return;                                                                                    \
    }                                                                                            \
  } while (0)

void ctx_error(mde_ctx* c, const std::vector<Req*>& v, int rc) {
  char m[512];
  mde_last_error_copy(c, m, sizeof m);
  fail_all(v, rc, m);
}

int grow_slot(mde_batcher::Slot* sl, uint64_t in_bytes, uint64_t d2h_bytes, uint64_t dev_out_bytes, std::string* msg,
              bool blocking) {
  int rc;
  if ((rc = grow(sl->pin_in, in_bytes, true, msg)) || (rc = grow(sl->dev_in, in_bytes, false, msg)) ||
      (rc = grow(sl->pin_out, d2h_bytes, true, msg)) || (rc = grow(sl->dev_out, dev_out_bytes, false, msg)))
    return rc;
  if (!sl->done && hipEventCreateWithFlags(&sl->done, hipEventDisableTiming | (blocking ? hipEventBlockingSync : 0u)) !=
                       hipSuccess) {
    sl->done = nullptr;
    *msg = "hipEventCreate failed";
    return MDE_E_DEVICE;
  }
  return MDE_OK;
}

// Device address of the slot's pinned out buffer (NULL: not mapped, copy instead).
uint8_t* mapped_out(mde_batcher* b, mde_batcher::Slot* sl) {
  void* p = nullptr;
  if (!b->direct_out || hipHostGetDevicePointer(&p, sl->pin_out.p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<uint8_t*>(p);
}

// Batches whose inputs are at most this many bytes may be read in place from pinned memory.
constexpr uint64_t kDirectInMax = 64ull << 10;

// Device address of the slot's pinned in buffer for a small batch (NULL: copy to the device).
const uint8_t* mapped_in(mde_batcher* b, mde_batcher::Slot* sl, uint64_t in_bytes) {
  void* p = nullptr;
  if (!b->direct_in || in_bytes > kDirectInMax || hipHostGetDevicePointer(&p, sl->pin_in.p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<const uint8_t*>(p);
}

// Stage + launch one build batch (records rebased into one arena): ONE H2D copy, mde_build_async,
// ONE D2H copy and an event, all enqueued on the batcher context's stream.
void launch_build(mde_batcher* b, mde_batcher::Slot* sl) {
  Batch* bt = &sl->bt;
  const std::vector<Req*>& v = bt->v;
  // the batcher's device before any allocation (grow_slot) or event creation: the leader is
  // whichever caller thread leads, whatever device it has current
  DeviceScope ds(b->device);  // the caller thread's device restored when the launch is enqueued
  const uint32_t B = v[0]->rec.n_buckets;
  const bool want_tree = v[0]->out.root != nullptr;  // same for the whole batch (request key)
  uint32_t stride = v[0]->rec.value_stride;
  for (Req* x : v)
    if (x->rec.value_stride != stride) stride = 0;  // mixed: variable-length offsets for all
  uint64_t P = 0, N = 0, V = 0;
  bool want_nodes = false;
  for (Req* x : v) {
    P += x->parts;
    N += x->r1 - x->r0;
    V += x->b1 - x->b0;
    want_nodes |= x->out.nodes != nullptr;
  }
  const uint64_t S = P * B, NI = mde_tree_internal_nodes(B);
  const uint64_t o_vals = 0, o_voff = align256(V + 16), o_seg = o_voff + (stride ? 0 : align256((N + 1) * 8));
  const uint64_t in_bytes = o_seg + (S + 1) * 8;
  uint64_t* o = bt->o;  // digest, size, items, root, nodes
  o[0] = 0;
  o[1] = align256(S * 8);
  o[2] = o[1] + align256(S * 4);
  o[3] = o[2] + align256(P * 4);
  o[4] = o[3] + (want_tree ? align256(P * 32) : 0);
  const uint64_t out_bytes = o[4] + (want_nodes ? P * NI * 32 : 0);
  bt->B = B;
  bt->NI = NI;
  std::string msg;
  const int rc = grow_slot(sl, in_bytes, out_bytes, out_bytes, &msg, b->blocking_sync);
  if (rc) {
    fail_all(v, rc, msg);
    return;
  }
  uint8_t* hin = static_cast<uint8_t*>(sl->pin_in.p);
  uint64_t* hvoff = reinterpret_cast<uint64_t*>(hin + o_voff);
  uint64_t* hseg = reinterpret_cast<uint64_t*>(hin + o_seg);
  uint64_t rbase = 0, bbase = 0, sbase = 0;
  for (Req* x : v) {
    const mde_records& r = x->rec;
    x->pos = sbase / B;
    if (x->b1 > x->b0) std::memcpy(hin + o_vals + bbase, r.values + x->b0, x->b1 - x->b0);
    if (!stride) {
      for (uint64_t k = x->r0; k < x->r1; k++)
        hvoff[rbase + k - x->r0] = bbase + (r.value_stride ? (k - x->r0) * r.value_stride : r.value_off[k] - x->b0);
    }
    const uint64_t Si = (uint64_t)x->parts * B;
    for (uint64_t s = 0; s < Si; s++) hseg[sbase + s] = r.seg_rec[s] - x->r0 + rbase;
    rbase += x->r1 - x->r0;
    bbase += x->b1 - x->b0;
    sbase += Si;
  }
  if (!stride) hvoff[N] = V;
  hseg[S] = N;
  hipStream_t st = static_cast<hipStream_t>(mde_get_stream(sl->ctx));
  const uint8_t* min_ = mapped_in(b, sl, in_bytes);
  const uint8_t* din = min_ ? min_ : static_cast<const uint8_t*>(sl->dev_in.p);
  // every build output is stored once by the tree pass (trees wider than the LDS levels re-read
  // their nodes: device memory and a copy for those)
  uint8_t* mapped = B <= 4096u ? mapped_out(b, sl) : nullptr;
  uint8_t* dout = mapped ? mapped : static_cast<uint8_t*>(sl->dev_out.p);
  if (!min_) BHIP(hipMemcpyAsync(sl->dev_in.p, hin, in_bytes, hipMemcpyHostToDevice, st));
  mde_records dr{};
  dr.values = din + o_vals;
  dr.values_bytes = V;
  dr.value_stride = stride;
  dr.layout = MDE_LAYOUT_SORTED;
  dr.value_off = stride ? nullptr : reinterpret_cast<const uint64_t*>(din + o_voff);
  dr.n_records = N;
  dr.n_partitions = (uint32_t)P;
  dr.n_buckets = B;
  dr.seg_rec = reinterpret_cast<const uint64_t*>(din + o_seg);
  mde_tree_out to{reinterpret_cast<uint64_t*>(dout + o[0]), reinterpret_cast<int32_t*>(dout + o[1]),
                  reinterpret_cast<int32_t*>(dout + o[2]), want_tree ? dout + o[3] : nullptr,
                  want_nodes ? dout + o[4] : nullptr};
  int brc = mde_build_async(sl->ctx, &dr, &to);
  if (brc) {
    ctx_error(sl->ctx, v, brc);
    return;
  }
  if (!mapped) BHIP(hipMemcpyAsync(sl->pin_out.p, dout, out_bytes, hipMemcpyDeviceToHost, st));
  BHIP(hipEventRecord(sl->done, st));
  bt->launched = true;
}

// One caller's part of a finished build batch, copied out on the caller's own thread.
void scatter_build(const mde_batcher::Slot* sl, Req* x) {
  const Batch& bt = sl->bt;
  const uint8_t* hout = static_cast<const uint8_t*>(sl->pin_out.p);
  const uint64_t B = bt.B, NI = bt.NI, Pi = x->parts, pbase = x->pos;
  const uint64_t* o = bt.o;
  if (x->out.digest) std::memcpy(x->out.digest, hout + o[0] + pbase * B * 8, Pi * B * 8);
  if (x->out.size) std::memcpy(x->out.size, hout + o[1] + pbase * B * 4, Pi * B * 4);
  if (x->out.items) std::memcpy(x->out.items, hout + o[2] + pbase * 4, Pi * 4);
  if (x->out.root) std::memcpy(x->out.root, hout + o[3] + pbase * 32, Pi * 32);
  if (x->out.nodes) std::memcpy(x->out.nodes, hout + o[4] + pbase * NI * 32, Pi * NI * 32);
}

int check_verify(Req* q, uint64_t object_stride) {
  if (!q->B || !mde_verify_peer_capacity(q->B) || q->B > 65536u)
    return fail(q, MDE_E_INVAL, "bad n_buckets %u", q->B);
  if (!q->digest || !q->valid || !q->valid_count || !q->diff_ids || !q->diff_count)
    return fail(q, MDE_E_INVAL, "bad verify arguments");
  if (q->R && !q->peer_off) return fail(q, MDE_E_INVAL, "peer_off is NULL");
  if (q->object_out && (!q->size || !q->object_len)) return fail(q, MDE_E_INVAL, "object_out needs size and object_len");
  if (q->object_out && object_stride < mde_epoch_tree_object_max_bytes(q->B))
    return fail(q, MDE_E_CAPACITY, "object_stride too small");
  for (uint32_t r = 0; r < q->R; r++)
    if (q->peer_off[r] > q->peer_off[r + 1]) return fail(q, MDE_E_INVAL, "peer_off not nondecreasing");
  if (q->R && q->peer_off[q->R] > q->peer_off[0] && !q->peer_bytes) return fail(q, MDE_E_INVAL, "peer_bytes is NULL");
  q->parts = 1;
  q->key[0] = 2;
  q->key[1] = q->B;
  q->key[2] = (uint64_t)q->epoch;
  q->key[3] = ((uint64_t)q->replica_count << 1) | (q->object_out ? 1u : 0u);
  return MDE_OK;
}

// Stage + launch one verify batch: mde_verify_epochs over all of them, the local trees given by
// their digests; peers padded to the batch's largest peer count with absent (empty) objects, which
// the reference skips like a failed EpochTreeObjectRequest (main/manager.go:1064-1070).
void launch_verify(mde_batcher* b, mde_batcher::Slot* sl) {
  Batch* bt = &sl->bt;
  const std::vector<Req*>& v = bt->v;
  DeviceScope ds(b->device);  // before grow_slot (see launch_build)
  const uint32_t B = v[0]->B;
  const int64_t epoch = v[0]->epoch;
  const uint32_t rcount = v[0]->replica_count;
  const bool want_obj = v[0]->object_out != nullptr;
  const uint64_t P = v.size();
  uint32_t R = 0;
  uint64_t nbytes = 0;
  for (Req* x : v) {
    R = std::max(R, x->R);
    if (x->R) nbytes += x->peer_off[x->R] - x->peer_off[0];
  }
  const uint64_t stride = want_obj ? mde_epoch_tree_object_max_bytes(B) : 0;
  const uint64_t i_dig = 0, i_size = align256(P * B * 8), i_part = i_size + align256(P * B * 4),
                 i_off = i_part + align256(P * 4), i_peer = i_off + align256((P * R + 1) * 8);
  const uint64_t in_bytes = i_peer + nbytes + 16;
  uint64_t* o = bt->o;  // valid, valid_count, ids, diff_count, status, object_len, objects
  o[0] = 0;
  o[1] = align256(P);
  o[2] = o[1] + align256(P * 4);
  o[3] = o[2] + align256(P * B * 4);
  o[4] = o[3] + align256(P * 4);
  o[5] = o[4] + align256(P * R * 4 + 4);
  o[6] = o[5] + align256(P * 4);
  o[7] = o[6] + align256(P * stride);
  const uint64_t out_bytes = o[7];
  bt->B = B;
  bt->stride = stride;
  bt->R = R;
  std::string msg;
  const int grc = grow_slot(sl, in_bytes, o[7], out_bytes, &msg, b->blocking_sync);
  if (grc) {
    fail_all(v, grc, msg);
    return;
  }
  uint8_t* hin = static_cast<uint8_t*>(sl->pin_in.p);
  uint64_t* hoff = reinterpret_cast<uint64_t*>(hin + i_off);
  int32_t* hpart = reinterpret_cast<int32_t*>(hin + i_part);
  uint64_t base = 0;
  for (uint64_t p = 0; p < P; p++) {
    Req* x = v[p];
    x->pos = p;
    std::memcpy(hin + i_dig + p * B * 8, x->digest, (uint64_t)B * 8);
    if (x->size) std::memcpy(hin + i_size + p * B * 4, x->size, (uint64_t)B * 4);
    else std::memset(hin + i_size + p * B * 4, 0, (uint64_t)B * 4);
    hpart[p] = x->partition;
    const uint64_t lo = x->R ? x->peer_off[0] : 0, hi = x->R ? x->peer_off[x->R] : 0;
    if (hi > lo) std::memcpy(hin + i_peer + base, x->peer_bytes + lo, hi - lo);
    for (uint32_t r = 0; r < R; r++) hoff[p * R + r] = base + (r < x->R ? x->peer_off[r] - lo : hi - lo);
    base += hi - lo;
  }
  hoff[P * R] = base;
  hipStream_t st = static_cast<hipStream_t>(mde_get_stream(sl->ctx));
  const uint8_t* min_ = mapped_in(b, sl, in_bytes);
  const uint8_t* din = min_ ? min_ : static_cast<const uint8_t*>(sl->dev_in.p);
  uint8_t* dout = static_cast<uint8_t*>(sl->dev_out.p);
  // every verify output is stored once by the launch: straight into pinned memory
  uint8_t* mapped = mapped_out(b, sl);
  uint8_t* wout = mapped ? mapped : dout;
  if (!min_) BHIP(hipMemcpyAsync(sl->dev_in.p, hin, in_bytes, hipMemcpyHostToDevice, st));
  const uint64_t* d_dig = reinterpret_cast<const uint64_t*>(din + i_dig);
  int rc = mde_reserve_decode_scratch(sl->ctx, P * R, nbytes);  // linear decode of any peer object
  if (rc) {
    ctx_error(sl->ctx, v, rc);
    return;
  }
  // local trees as digests only (nodes NULL): a partition builds its own tree on the device only
  // when a peer of another shape needs its inner nodes
  rc = mde_verify_epochs_async(sl->ctx, (uint32_t)P, B, reinterpret_cast<const int32_t*>(din + i_part), epoch, d_dig,
                               reinterpret_cast<const int32_t*>(din + i_size), nullptr, R, din + i_peer,
                               reinterpret_cast<const uint64_t*>(din + i_off), rcount, wout + o[0],
                               reinterpret_cast<int32_t*>(wout + o[1]), reinterpret_cast<int32_t*>(wout + o[2]),
                               reinterpret_cast<int32_t*>(wout + o[3]), reinterpret_cast<int32_t*>(wout + o[4]),
                               want_obj ? wout + o[6] : nullptr, stride,
                               want_obj ? reinterpret_cast<uint32_t*>(wout + o[5]) : nullptr);
  if (rc) {
    ctx_error(sl->ctx, v, rc);
    return;
  }
  uint8_t* hout = static_cast<uint8_t*>(sl->pin_out.p);
  if (!mapped) BHIP(hipMemcpyAsync(hout, dout, o[7], hipMemcpyDeviceToHost, st));
  BHIP(hipEventRecord(sl->done, st));
  bt->launched = true;
}

// One caller's part of a finished verify batch, copied out on the caller's own thread.
void scatter_verify(const mde_batcher::Slot* sl, Req* x) {
  const Batch& bt = sl->bt;
  const uint8_t* hout = static_cast<const uint8_t*>(sl->pin_out.p);
  const uint64_t B = bt.B, R = bt.R, stride = bt.stride, p = x->pos;
  const uint64_t* o = bt.o;
  *x->valid = hout[o[0] + p];
  std::memcpy(x->valid_count, hout + o[1] + p * 4, 4);
  int32_t dc;
  std::memcpy(&dc, hout + o[3] + p * 4, 4);
  *x->diff_count = dc;
  if (dc > 0) std::memcpy(x->diff_ids, hout + o[2] + p * B * 4, (uint64_t)dc * 4);
  if (x->peer_status && x->R) std::memcpy(x->peer_status, hout + o[4] + p * R * 4, (uint64_t)x->R * 4);
  if (x->object_out) {
    uint32_t len;
    std::memcpy(&len, hout + o[5] + p * 4, 4);
    *x->object_len = len;
    std::memcpy(x->object_out, hout + o[6] + p * stride, len);
  }
}

// Hand the leader role to the oldest waiting request when no leader is active and a staging slot
// is free (called with the lock held). That request's thread wakes alone.
void handoff(mde_batcher* b) {
  if (b->leading || b->q.empty()) return;
  for (int i = 0; i < b->n_slots; i++)
    if (!b->slots[i].busy) {
      Req* x = b->q.front();
      x->lead = true;
      if (b->profile) x->lead_t = std::chrono::steady_clock::now();
      x->cv.notify_one();
      return;
    }
}

bool free_slot(const mde_batcher* b) {
  for (int i = 0; i < b->n_slots; i++)
    if (!b->slots[i].busy) return true;
  return false;
}

// The leader's turn (lock held on entry and exit; `r` = the leader's own request, still queued):
// take a batch into a free slot, pass the leader role on (the next leader stages its batch while
// this one stages and runs), stage and launch with the lock released, wait for the batch's event,
// then mark its callers ready: each copies its own outputs out of the slot on its own thread, and
// the last one frees the slot.
void lead(mde_batcher* b, Req* r, std::unique_lock<std::mutex>& lk) {
  b->leading = true;
  if (b->max_wait_us) {  // let concurrent callers join, until the batch is full or the window ends
    const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(b->max_wait_us);
    for (;;) {
      uint64_t parts = 0;
      for (Req* x : b->q)
        if (same_key(x, r)) parts += x->parts;
      if (parts >= b->max_parts || b->collect.wait_until(lk, until) == std::cv_status::timeout) break;
    }
  }
  mde_batcher::Slot* sl = nullptr;
  for (int i = 0; i < b->n_slots && !sl; i++)
    if (!b->slots[i].busy) sl = &b->slots[i];
  sl->busy = true;
  Batch& bt = sl->bt;
  bt = Batch{};
  bt.v = take(b, r);
  uint64_t parts = 0;
  for (Req* x : bt.v) {
    parts += x->parts;
    x->slot = sl;
  }
  b->n_batches++;
  b->n_requests += bt.v.size();
  b->n_partitions += parts;
  if (b->early_handoff) {
    b->leading = false;
    handoff(b);
  }
  lk.unlock();
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = b->profile ? clk::now() : clk::time_point{};
  const Kind kind = bt.v[0]->kind;
  if (kind == Kind::Build) launch_build(b, sl);
  else launch_verify(b, sl);
  if (!b->early_handoff) {
    lk.lock();
    b->leading = false;
    handoff(b);  // the next batch stages and launches while this one runs on the device
    lk.unlock();
  }
  const clk::time_point t1 = b->profile ? clk::now() : clk::time_point{};
  clk::time_point t2 = t1;
  if (bt.launched) {
    const hipError_t e = hipEventSynchronize(sl->done);
    if (b->profile) t2 = clk::now();
    if (e != hipSuccess) {
      fail_all(bt.v, MDE_E_DEVICE, std::string("batch: ") + hipGetErrorString(e));
      bt.launched = false;
    }
  }
  lk.lock();
  if (b->profile) {
    b->t_stage += std::chrono::duration<double>(t1 - t0).count();
    b->t_device += std::chrono::duration<double>(t2 - t1).count();
  }
  bt.pending = bt.v.size();
  for (Req* x : bt.v) {
    x->ready = true;
    x->cv.notify_one();
  }
}

// A ready request copies its outputs out (lock released), then frees its batch's slot if it was
// the last one (lock held on entry and exit).
void finish(mde_batcher* b, Req* r, std::unique_lock<std::mutex>& lk) {
  r->ready = false;
  mde_batcher::Slot* sl = static_cast<mde_batcher::Slot*>(r->slot);
  const bool copy = sl->bt.launched && r->rc == MDE_OK;
  lk.unlock();
  using clk = std::chrono::steady_clock;
  const clk::time_point t0 = b->profile ? clk::now() : clk::time_point{};
  if (copy) {
    if (r->kind == Kind::Build) scatter_build(sl, r);
    else scatter_verify(sl, r);
  }
  const clk::time_point t1 = b->profile ? clk::now() : clk::time_point{};
  lk.lock();
  if (b->profile) b->t_scatter += std::chrono::duration<double>(t1 - t0).count();
  r->done = true;
  if (--sl->bt.pending == 0) {
    sl->bt.v.clear();
    sl->busy = false;
    handoff(b);
  }
}

// Enqueue, then either lead a batch or wait (on this request's own condition variable) until its
// batch is ready or it is handed the leader role.
int submit(mde_batcher* b, Req* r) {
  std::unique_lock<std::mutex> lk(b->m);
  b->q.push_back(r);
  b->collect.notify_one();
  if (!b->leading && free_slot(b)) r->lead = true;
  while (!r->done) {
    if (r->ready) {
      finish(b, r, lk);
      continue;
    }
    if (r->lead) {
      r->lead = false;
      // Lead only while this request is still queued, so the leader waits for its own batch. A
      // stale role (another leader took this request meanwhile, or is active, or no slot is free)
      // is passed on to the oldest queued request instead of being dropped.
      if (!r->slot && !b->leading && free_slot(b)) {
        if (b->profile && r->lead_t != std::chrono::steady_clock::time_point{}) {
          b->t_handoff += std::chrono::duration<double>(std::chrono::steady_clock::now() - r->lead_t).count();
          b->n_handoff++;
        }
        lead(b, r, lk);
      } else {
        handoff(b);
      }
      continue;
    }
    r->cv.wait(lk);
  }
  return r->rc;
}

}  // namespace

extern "C" {

int mde_batcher_create(int device, uint32_t max_partitions, uint32_t max_wait_us, mde_batcher** out) {
  if (!out) return MDE_E_INVAL;
  *out = nullptr;
  mde_batcher* b = new (std::nothrow) mde_batcher();
  if (!b) return MDE_E_NOMEM;
  if (const char* e = std::getenv("MDE_BATCH_SLOTS")) b->n_slots = std::min(kMaxSlots, std::max(1, std::atoi(e)));
  for (int i = 0; i < b->n_slots; i++) {
    const int rc = mde_create(device, &b->slots[i].ctx);
    if (rc != MDE_OK) {
      for (auto& x : b->slots)
        if (x.ctx) mde_destroy(x.ctx);
      delete b;
      return rc;
    }
  }
  b->device = device;
  if (const char* e = std::getenv("MDE_DIRECT_OUT")) b->direct_out = std::atoi(e) != 0;
  if (const char* e = std::getenv("MDE_DIRECT_IN")) b->direct_in = std::atoi(e) != 0;
  if (const char* e = std::getenv("MDE_BATCH_BLOCKING_SYNC")) b->blocking_sync = std::atoi(e) != 0;
  if (const char* e = std::getenv("MDE_BATCH_PROFILE")) b->profile = std::atoi(e) != 0;
  if (const char* e = std::getenv("MDE_BATCH_EARLY")) b->early_handoff = std::atoi(e) != 0;
  b->max_parts = max_partitions ? max_partitions : 256;
  b->max_wait_us = max_wait_us;
  *out = b;
  return MDE_OK;
}

void mde_batcher_destroy(mde_batcher* b) {
  if (!b) return;
  if (b->profile && b->n_batches)
    std::fprintf(stderr,
                 "{\"batcher_profile\": {\"batches\": %llu, \"requests\": %llu, \"stage_launch_us\": %.2f, "
                 "\"device_wait_us\": %.2f, \"copy_out_us_per_batch\": %.2f, \"handoffs\": %llu, \"handoff_us\": %.2f}}\n",
                 (unsigned long long)b->n_batches, (unsigned long long)b->n_requests, 1e6 * b->t_stage / b->n_batches,
                 1e6 * b->t_device / b->n_batches, 1e6 * b->t_scatter / b->n_batches, (unsigned long long)b->n_handoff,
                 b->n_handoff ? 1e6 * b->t_handoff / b->n_handoff : 0.0);
  DeviceScope ds(b->device);
  for (auto& sl : b->slots) {
    if (!sl.ctx) continue;
    (void)mde_synchronize(sl.ctx);
    if (sl.pin_in.p) (void)hipHostFree(sl.pin_in.p);
    if (sl.pin_out.p) (void)hipHostFree(sl.pin_out.p);
    if (sl.dev_in.p) (void)hipFree(sl.dev_in.p);
    if (sl.dev_out.p) (void)hipFree(sl.dev_out.p);
    if (sl.done) (void)hipEventDestroy(sl.done);
    mde_destroy(sl.ctx);
  }
  delete b;
}

mde_ctx* mde_batcher_ctx(mde_batcher* b, uint32_t i) {
  return b && i < (uint32_t)b->n_slots ? b->slots[i].ctx : nullptr;
}

uint32_t mde_batcher_contexts(const mde_batcher* b) { return b ? (uint32_t)b->n_slots : 0u; }

int mde_batcher_stats(mde_batcher* b, uint64_t* batches, uint64_t* requests, uint64_t* partitions) {
  if (!b) return MDE_E_INVAL;
  std::lock_guard<std::mutex> lk(b->m);
  if (batches) *batches = b->n_batches;
  if (requests) *requests = b->n_requests;
  if (partitions) *partitions = b->n_partitions;
  return MDE_OK;
}

int mde_batch_build(mde_batcher* b, const mde_records* rec, const mde_tree_out* out, char* err, uint64_t err_cap) {
  put_msg(err, err_cap, "");
  if (!b || !rec || !out) {
    put_msg(err, err_cap, "null batcher, records or out");
    return MDE_E_INVAL;
  }
  Req q;
  q.kind = Kind::Build;
  q.rec = *rec;
  q.out = *out;
  q.err = err;
  q.err_cap = err_cap;
  int rc = check_build(&q);
  if (rc) return rc;
  return submit(b, &q);
}

int mde_batch_verify(mde_batcher* b, uint32_t n_buckets, int32_t partition, int64_t epoch, const uint64_t* digest,
                     const int32_t* size, uint32_t n_peers, const uint8_t* peer_bytes, const uint64_t* peer_off,
                     uint32_t replica_count, uint8_t* valid, int32_t* valid_count, int32_t* diff_ids,
                     int32_t* diff_count, int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                     uint32_t* object_len, char* err, uint64_t err_cap) {
  put_msg(err, err_cap, "");
  if (!b) {
    put_msg(err, err_cap, "null batcher");
    return MDE_E_INVAL;
  }
  Req q;
  q.kind = Kind::Verify;
  q.B = n_buckets;
  q.partition = partition;
  q.epoch = epoch;
  q.digest = digest;
  q.size = size;
  q.R = n_peers;
  q.peer_bytes = peer_bytes;
  q.peer_off = peer_off;
  q.replica_count = replica_count;
  q.valid = valid;
  q.valid_count = valid_count;
  q.diff_ids = diff_ids;
  q.diff_count = diff_count;
  q.peer_status = peer_status;
  q.object_out = object_out;
  q.object_len = object_len;
  q.err = err;
  q.err_cap = err_cap;
  int rc = check_verify(&q, object_stride);
  if (rc) return rc;
  return submit(b, &q);
}

}  // extern "C"
