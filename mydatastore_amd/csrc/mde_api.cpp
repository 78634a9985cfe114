// mde_api.cpp -- C ABI of the MI355X Merkle engine (include/mde.h).
//
// One context = one HIP device + one stream + grow-only device scratch. Every entry point takes
// the context lock and makes the context's device current on the calling thread, so a context can
// be shared by many goroutine-backed OS threads (VerifyEpoch runs on any of WORKERS_COUNT workers,
// main/manager.go:166-170) or each thread can own one. Errors are returned as MDE_E_* codes with
// the message kept per context; nothing throws or aborts across the ABI.
#include "../../include/mde.h"
#include "device_scope.hpp"

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "mde_internal.hpp"

// Digest-kernel tuning defaults (tools/digest_sweep.sh, profiles/r01_digest_sweep.json).
constexpr int kDefaultDigestVariant = 11;  // U=4 nontemporal, register-prefetched (first step before
                                           // the bucket search), s_setprio 2
constexpr int kDefaultDigestCap = 2;      // 2 workgroups (8 waves) per CU
constexpr int kDefaultDigestOversub = 1;  // grid = resident slots x oversub
// Interleaved pieces (digest variant 12): by default a wave whose share of
// the arena is at least kAutoPieceMinShare streams it as kAutoPieces interleaved pieces, so the
// grid sweeps the arena front to back together (same-box A/B, profiles/r02g_pieces_*.jsonl: C4
// fused +1.0 %, C3 +3.6 %; the N=8 shard, 0.6 MB per wave, loses 2-10 % to the per-piece search
// and pipeline drain, so small shares keep one range).
constexpr uint64_t kAutoPieceBytes = UINT64_MAX;  // digest_piece_bytes value: the policy above
constexpr uint64_t kAutoPieceMinShare = 4ull << 20;
constexpr uint64_t kAutoPieces = 5;
constexpr int kWindowDigestVariant = 13;                 // SegWindow + true double buffer (plan_digest)
constexpr int kRec8DigestVariant = 15;  // fixed 8-byte records: record-space prefix scan (plan_digest)
constexpr uint64_t kWindowMaxAvgBucketBytes = 64ull << 10;  // average bucket bytes below which it runs

struct mde_ctx {
  int device = 0;
  int cus = 256;
  int digest_blocks_per_cu = 0;  // resident workgroups per CU for the digest kernel (queried)
  int variant_blocks[32] = {0};  // the same per digest variant (plan_digest queries the one it runs)
  int digest_variant = kDefaultDigestVariant;
  bool digest_auto = true;  // no explicit variant: plan_digest picks the window / pieces forms
  int digest_cap = kDefaultDigestCap;
  int digest_oversub = kDefaultDigestOversub;
  uint64_t digest_piece_bytes = kAutoPieceBytes;
  bool direct_out = true;  // packed host calls: kernels store write-once outputs into pinned memory
  char arch[64] = {0};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::string err;
  // Byte-sum accumulators: zero between builds (the tree kernel clears what it reads).
  unsigned long long* sums = nullptr;
  uint32_t* counts = nullptr;  // layout-B record counts, same lifecycle as sums
  uint64_t sums_cap = 0;
  bool sums_dirty = false;
  // Host-API staging (device) and a scratch node array for B > kTreeLdsMaxBuckets.
  struct Buf { void* p = nullptr; uint64_t cap = 0; };
  Buf stage[16];
  Buf nodes_scratch;
  // Small host-API calls (mde_build): inputs and outputs each travel as ONE copy between a
  // pinned host region (pin_*) and a device region (packed_*).
  Buf packed_in, packed_out, pin_in, pin_out;
  Buf extract_scratch;
  Buf verify_scratch;
  Buf deep_scratch;  // spill area of deeply nested unknown groups (WireDecodeLaunch::deep)
  bool verify_chain = false;  // mde_set_verify_mode(1): the five-launch chain even when fusable
  // Host-ingest ring (mde_build_streamed): two slots of values / value_off / seg_rec.
  Buf ring_vals[2], ring_voff[2], ring_seg[2];
  hipStream_t copy_stream = nullptr;
  hipEvent_t ev_loaded[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  // Software-pipelined builds (mde_build_pipelined_async): two scratch slots of their own, so the
  // standalone entry points keep using `sums`, and the build whose trees are still owed.
  struct Slot {
    unsigned long long* sums = nullptr;
    uint32_t* counts = nullptr;
    uint64_t cap = 0;
    bool dirty = false;
  };
  Slot pipe[2];
  // Work accounting (mde_ctx_stats): builds enqueued on this context, their partitions and value
  // bytes -- which GPU of a group built what.
  uint64_t st_builds = 0, st_parts = 0, st_bytes = 0;
  struct Pending {
    bool active = false;
    int slot = 0;
    mde_records rec{};
    mde_tree_out out{};
  } pending;
};

namespace {

int set_err(mde_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define MDE_HIP(c, expr)                                                                  \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      if (c) c->sums_dirty = true;                                                        \
      return set_err((c), MDE_E_DEVICE, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),  \
                     __FILE__, __LINE__);                                                 \
    }                                                                                     \
  } while (0)

int ensure_buf(mde_ctx* c, mde_ctx::Buf& b, uint64_t bytes) {
  if (b.cap >= bytes && b.p) return MDE_OK;
  if (b.p) {
    MDE_HIP(c, hipStreamSynchronize(c->stream));
    MDE_HIP(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  uint64_t cap = bytes < 256 ? 256 : bytes;
  if (hipMalloc(&b.p, cap) != hipSuccess) {
    b.p = nullptr;
    return set_err(c, MDE_E_NOMEM, "device allocation of %llu bytes failed", (unsigned long long)cap);
  }
  b.cap = cap;
  return MDE_OK;
}

int ensure_pinned(mde_ctx* c, mde_ctx::Buf& b, uint64_t bytes) {
  if (b.cap >= bytes && b.p) return MDE_OK;
  if (b.p) {
    MDE_HIP(c, hipStreamSynchronize(c->stream));
    MDE_HIP(c, hipHostFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  uint64_t cap = bytes < 4096 ? 4096 : bytes;
  if (hipHostMalloc(&b.p, cap, hipHostMallocDefault) != hipSuccess) {
    b.p = nullptr;
    return set_err(c, MDE_E_NOMEM, "pinned host allocation of %llu bytes failed", (unsigned long long)cap);
  }
  b.cap = cap;
  return MDE_OK;
}

// 256-byte aligned pieces of one staging region.
struct Pack {
  uint64_t total = 0;
  uint64_t add(uint64_t bytes) {
    const uint64_t o = total;
    total += (bytes + 255) & ~255ull;
    return o;
  }
};

// Calls whose inputs and outputs each fit this go through the packed path: a pageable
// hipMemcpy costs ~10-20 us of fixed overhead per call, so the six to eight separate copies of
// a one-partition build cost more than the build itself; one pinned copy each way plus host
// memcpys does not. Larger calls keep the direct copies (the runtime pipelines those).
constexpr uint64_t kPackedCallMax = 8ull << 20;

// Staging of one synchronous host-API call: declare the inputs (host source, device bytes) and
// outputs (host destination, bytes), then upload() -> launch on dev_in/dev_out -> download().
// Packed calls use the context's packed_* / pin_* regions; larger ones one stage[] buffer per
// piece (inputs first, then outputs) with direct copies. A NULL host pointer skips its copy.
// An output declared write_once (the launch stores each of its bytes at most once and never reads
// it back, no atomics) is, in a packed call, stored by the kernels straight into the pinned
// staging area: no D2H copy for it, and none at all when every output is write-once -- a D2H copy
// above ~16 KB otherwise starts ~11 us after the kernel ends (profiles/r03q_call_trace.txt).
class HostIo {
 public:
  explicit HostIo(mde_ctx* c) : c_(c) {}
  // a call that returns between upload() and download() (an error) still waits for the copies
  // it issued: they read the caller's buffers and the entry point's host vectors
  ~HostIo() {
    if (issued_) (void)hipStreamSynchronize(c_->stream);
  }
  int in(const void* src, uint64_t copy_bytes, uint64_t dev_bytes) {
    pieces_[n_] = {const_cast<void*>(src), copy_bytes, dev_bytes, pin_.add(dev_bytes), true, false};
    return n_++;
  }
  int out(void* dst, uint64_t bytes, bool write_once = false) {
    const bool direct = write_once && c_->direct_out;
    pieces_[n_] = {dst, bytes, bytes, (direct ? pdir_ : pcopy_).add(bytes), false, direct};
    return n_++;
  }
  void* dev(int i) const { return dev_[i]; }
  int upload() {
    const uint64_t out_total = pcopy_.total + pdir_.total;
    packed_ = pin_.total <= kPackedCallMax && out_total <= kPackedCallMax;
    int rc;
    if (packed_) {
      if ((rc = ensure_buf(c_, c_->packed_in, pin_.total)) || (rc = ensure_buf(c_, c_->packed_out, out_total)) ||
          (rc = ensure_pinned(c_, c_->pin_in, pin_.total)) || (rc = ensure_pinned(c_, c_->pin_out, out_total)))
        return rc;
      void* out_dev = nullptr;
      if (pdir_.total && hipHostGetDevicePointer(&out_dev, c_->pin_out.p, 0) != hipSuccess) {
        (void)hipGetLastError();
        out_dev = nullptr;
      }
      copy_bytes_ = out_dev ? pcopy_.total : out_total;  // no mapping: every output is copied
      uint8_t* hi = static_cast<uint8_t*>(c_->pin_in.p);
      for (int i = 0; i < n_; i++) {
        const Piece& q = pieces_[i];
        if (q.input) dev_[i] = static_cast<uint8_t*>(c_->packed_in.p) + q.off;
        else if (q.direct) dev_[i] = static_cast<uint8_t*>(out_dev ? out_dev : c_->packed_out.p) + pcopy_.total + q.off;
        else dev_[i] = static_cast<uint8_t*>(c_->packed_out.p) + q.off;
        if (q.input && q.host && q.copy) std::memcpy(hi + q.off, q.host, q.copy);
      }
      issued_ = true;
      MDE_HIP(c_, hipMemcpyAsync(c_->packed_in.p, hi, pin_.total, hipMemcpyHostToDevice, c_->stream));
      return MDE_OK;
    }
    for (int i = 0; i < n_; i++) {
      const Piece& q = pieces_[i];
      if ((rc = ensure_buf(c_, c_->stage[i], q.dev))) return rc;
      dev_[i] = c_->stage[i].p;
      issued_ = true;
      if (q.input && q.host && q.copy)
        MDE_HIP(c_, hipMemcpyAsync(dev_[i], q.host, q.copy, hipMemcpyHostToDevice, c_->stream));
    }
    return MDE_OK;
  }
  int download() {
    if (packed_) {
      uint8_t* ho = static_cast<uint8_t*>(c_->pin_out.p);
      if (copy_bytes_) MDE_HIP(c_, hipMemcpyAsync(ho, c_->packed_out.p, copy_bytes_, hipMemcpyDeviceToHost, c_->stream));
      MDE_HIP(c_, hipStreamSynchronize(c_->stream));
      issued_ = false;
      for (int i = 0; i < n_; i++) {
        const Piece& q = pieces_[i];
        if (!q.input && q.host && q.copy) std::memcpy(q.host, ho + (q.direct ? pcopy_.total : 0) + q.off, q.copy);
      }
      return MDE_OK;
    }
    for (int i = 0; i < n_; i++) {
      const Piece& q = pieces_[i];
      if (!q.input && q.host && q.copy)
        MDE_HIP(c_, hipMemcpyAsync(q.host, dev_[i], q.copy, hipMemcpyDeviceToHost, c_->stream));
    }
    MDE_HIP(c_, hipStreamSynchronize(c_->stream));
    issued_ = false;
    return MDE_OK;
  }

 private:
  struct Piece {
    void* host;
    uint64_t copy, dev, off;
    bool input, direct;
  };
  mde_ctx* c_;
  uint64_t copy_bytes_ = 0;
  Piece pieces_[16];
  void* dev_[16] = {};
  int n_ = 0;
  Pack pin_, pcopy_, pdir_;
  bool packed_ = false;
  bool issued_ = false;  // copies issued that download() has not waited for
};

int ensure_sums(mde_ctx* c, uint64_t S) {
  if (c->sums_cap < S || !c->sums) {
    if (c->sums) {
      MDE_HIP(c, hipStreamSynchronize(c->stream));
      MDE_HIP(c, hipFree(c->sums));
      MDE_HIP(c, hipFree(c->counts));
      c->sums = nullptr;
      c->counts = nullptr;
    }
    uint64_t cap = S < 1024 ? 1024 : S;
    if (hipMalloc(&c->sums, cap * 8) != hipSuccess || hipMalloc(&c->counts, cap * 4) != hipSuccess) {
      if (c->sums) (void)hipFree(c->sums);
      c->sums = nullptr;
      c->counts = nullptr;
      c->sums_cap = 0;
      return set_err(c, MDE_E_NOMEM, "sums allocation failed");
    }
    c->sums_cap = cap;
    c->sums_dirty = true;
  }
  if (c->sums_dirty) {
    MDE_HIP(c, hipMemsetAsync(c->sums, 0, c->sums_cap * 8, c->stream));
    MDE_HIP(c, hipMemsetAsync(c->counts, 0, c->sums_cap * 4, c->stream));
    c->sums_dirty = false;
  }
  return MDE_OK;
}

int ensure_slot(mde_ctx* c, mde_ctx::Slot& sl, uint64_t S) {
  if (sl.cap < S || !sl.sums) {
    if (sl.sums) {
      MDE_HIP(c, hipStreamSynchronize(c->stream));
      MDE_HIP(c, hipFree(sl.sums));
      MDE_HIP(c, hipFree(sl.counts));
      sl.sums = nullptr;
      sl.counts = nullptr;
    }
    uint64_t cap = S < 1024 ? 1024 : S;
    if (hipMalloc(&sl.sums, cap * 8) != hipSuccess || hipMalloc(&sl.counts, cap * 4) != hipSuccess) {
      if (sl.sums) (void)hipFree(sl.sums);
      sl.sums = nullptr;
      sl.counts = nullptr;
      sl.cap = 0;
      return set_err(c, MDE_E_NOMEM, "pipeline scratch allocation failed");
    }
    sl.cap = cap;
    sl.dirty = true;
  }
  if (sl.dirty) {
    MDE_HIP(c, hipMemsetAsync(sl.sums, 0, sl.cap * 8, c->stream));
    MDE_HIP(c, hipMemsetAsync(sl.counts, 0, sl.cap * 4, c->stream));
    sl.dirty = false;
  }
  return MDE_OK;
}

// An entry point's critical section: the context lock, and the context's device selected for the
// call (the caller thread's device restored after it).
struct Guard {
  mde_ctx* c;
  std::lock_guard<std::mutex> lk;
  DeviceScope ds;
  explicit Guard(mde_ctx* ctx) : c(ctx), lk(ctx->mu), ds(ctx->device) { c->err.clear(); }
};

// Waits for the context stream when it goes out of scope: a synchronous entry point that returns
// early (an error) must not leave copies in flight from host memory about to be freed.
struct SyncOnReturn {
  hipStream_t s;
  ~SyncOnReturn() { (void)hipStreamSynchronize(s); }
};

int check_records(mde_ctx* c, const mde_records* r) {
  if (!r) return set_err(c, MDE_E_INVAL, "records is NULL");
  if (r->n_buckets == 0) return set_err(c, MDE_E_INVAL, "n_buckets must be >= 1");
  if (r->layout > MDE_LAYOUT_TAGGED) return set_err(c, MDE_E_INVAL, "unknown layout %u", r->layout);
  if (r->layout == MDE_LAYOUT_TAGGED) {
    if (!r->part_rec || (!r->bucket_tag && r->n_records)) return set_err(c, MDE_E_INVAL, "layout B needs part_rec and bucket_tag");
    if (!r->value_stride || r->value_stride > (1u << 30))
      return set_err(c, MDE_E_INVAL, "layout B needs fixed-length values of 1 B .. 1 GiB");
    if (r->n_buckets > 65536) return set_err(c, MDE_E_INVAL, "layout B supports n_buckets <= 65536");
  } else if (!r->seg_rec) {
    return set_err(c, MDE_E_INVAL, "seg_rec is NULL");
  }
  if ((uint64_t)r->n_partitions * r->n_buckets > 0xffffffffull)
    return set_err(c, MDE_E_INVAL, "n_partitions * n_buckets exceeds 2^32");
  if (r->value_stride == 0 && !r->value_off && r->n_records)
    return set_err(c, MDE_E_INVAL, "variable-length values need value_off");
  if (!r->values && r->values_bytes) return set_err(c, MDE_E_INVAL, "values is NULL");
  if (r->value_stride && (uint64_t)r->value_stride * r->n_records > r->values_bytes)
    return set_err(c, MDE_E_INVAL, "n_records * value_stride exceeds values_bytes");
  return MDE_OK;
}

mde::SegDesc seg_desc(const mde_records* r) {
  mde::SegDesc d{};
  const uintptr_t v = reinterpret_cast<uintptr_t>(r->values);
  d.base = reinterpret_cast<const uint8_t*>(v & ~uintptr_t(15));
  d.shift = v & 15u;
  d.stride = r->value_stride;
  d.value_off = r->value_off;
  d.seg_rec = r->seg_rec;
  d.S = (uint32_t)((uint64_t)r->n_partitions * r->n_buckets);
  d.n_records = r->n_records;
  d.end = d.shift + r->values_bytes;
  return d;
}

int plan_digest(mde_ctx* c, uint64_t bytes, mde::DigestLaunch* a) {
  // Short buckets (a boundary every few KiB, e.g. the reference's default B = 1000): the
  // register-window kernel (variant 13). Same-box A/B (profiles/r02u_window.jsonl): C4 at
  // B = 1000 (10 KiB buckets) 2,685 -> 1,493 us, its N=8 shard 376 -> 192 us; at B = 64 (156 KiB
  // buckets) it costs 0.3-0.8 %, so longer buckets keep variant 11.
  if (c->digest_auto && a->seg.S && bytes / a->seg.S < kWindowMaxAvgBucketBytes) {
    a->variant = kWindowDigestVariant;
    // the production epoch-index value: 8-byte LE timestamps (main/manager.go:816), a bucket start
    // every ~100 records at B = 1,000; the record-space scan (digest.hip digest_range_rec8)
    if (a->seg.stride == 8 && (a->seg.shift & 7) == 0) a->variant = kRec8DigestVariant;
  }
  // an explicitly chosen rec8 variant needs 8-byte records: the window kernel instead (decided
  // before the grid is planned, so the occupancy below is the one of the kernel that runs)
  if (mde::bucket_digest_rec8(a->variant) && (a->seg.stride != 8 || (a->seg.shift & 7)))
    a->variant = mde::bucket_digest_pieces(a->variant) ? mde::bucket_digest_pieces_sibling(kWindowDigestVariant)
                                                       : kWindowDigestVariant;
  uint64_t piece_bytes = 0;
  if (c->digest_piece_bytes == kAutoPieceBytes) {
    // automatic pieces: the default's (or an explicitly chosen pieces variant's) pieces form
    const int sib = c->digest_auto || mde::bucket_digest_pieces(a->variant)
                        ? mde::bucket_digest_pieces_sibling(a->variant) : a->variant;
    if (mde::bucket_digest_pieces(sib)) {
      const uint64_t waves = (uint64_t)c->cus * (uint64_t)(c->digest_blocks_per_cu > 0 ? c->digest_blocks_per_cu : 4) * 4u *
                             (uint64_t)(c->digest_oversub > 0 ? c->digest_oversub : 1);
      const uint64_t share = bytes / waves;
      if (c->digest_oversub <= 1 && share >= kAutoPieceMinShare) {
        piece_bytes = share / kAutoPieces;
        a->variant = sib;
      }
    }
  } else if (mde::bucket_digest_pieces(a->variant)) {
    piece_bytes = c->digest_piece_bytes;
  }
  // grid from the resident workgroups of the variant that actually runs (the window and rec8
  // kernels may fit fewer per CU than the default under a raised cap: then every wave of the
  // equal-range grid is still co-resident, no tail)
  int& vb = c->variant_blocks[a->variant & 31];
  if (!vb) vb = mde::bucket_digest_blocks_per_cu(a->variant, c->digest_cap);
  const int blocks_per_cu = std::min(vb, c->digest_blocks_per_cu > 0 ? c->digest_blocks_per_cu : vb);
  mde::plan_bucket_digest(bytes, c->cus, blocks_per_cu, c->digest_oversub, piece_bytes,
                          &a->wave_bytes, &a->n_waves, &a->pieces);
  a->piece_stride = (uint64_t)a->n_waves * a->wave_bytes;
  a->lds_bytes = c->digest_oversub > 1 ? (uint32_t)((160u * 1024u) / (uint32_t)c->digest_blocks_per_cu) & ~255u : 0u;
  if (mde::bucket_digest_rec8(a->variant)) a->lds_bytes = std::max(a->lds_bytes, mde::bucket_digest_rec8_lds_bytes(a->variant));
  return MDE_OK;
}

// Full validation of host-resident inputs (mde_build): the device API trusts its inputs but the
// kernels clamp every index, so bad device input gives wrong digests, never a fault.
int check_host_records(mde_ctx* c, const mde_records* r) {
  if (r->layout == MDE_LAYOUT_TAGGED) {
    for (uint32_t p = 0; p < r->n_partitions; p++)
      if (r->part_rec[p] > r->part_rec[p + 1]) return set_err(c, MDE_E_INVAL, "part_rec not nondecreasing");
    if (r->part_rec[r->n_partitions] > r->n_records) return set_err(c, MDE_E_INVAL, "part_rec exceeds n_records");
    for (uint64_t i = r->part_rec[0]; i < r->part_rec[r->n_partitions]; i++)
      if (r->bucket_tag[i] >= r->n_buckets) return set_err(c, MDE_E_INVAL, "bucket_tag[%llu] out of range", (unsigned long long)i);
    return MDE_OK;
  }
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  for (uint64_t s = 0; s < S; s++)
    if (r->seg_rec[s] > r->seg_rec[s + 1])
      return set_err(c, MDE_E_INVAL, "seg_rec not nondecreasing at %llu", (unsigned long long)s);
  if (r->seg_rec[S] > r->n_records)
    return set_err(c, MDE_E_INVAL, "seg_rec[%llu] = %llu exceeds n_records %llu",
                   (unsigned long long)S, (unsigned long long)r->seg_rec[S],
                   (unsigned long long)r->n_records);
  if (!r->value_stride && r->n_records) {
    for (uint64_t i = 0; i < r->n_records; i++)
      if (r->value_off[i] > r->value_off[i + 1])
        return set_err(c, MDE_E_INVAL, "value_off not nondecreasing at %llu", (unsigned long long)i);
    if (r->value_off[r->n_records] > r->values_bytes)
      return set_err(c, MDE_E_INVAL, "value_off[n_records] exceeds values_bytes");
  }
  return MDE_OK;
}

// span: bytes the records cover (0 = values_bytes); a streamed chunk passes a biased values
// pointer whose values_bytes includes the bias.
void plan_tagged_launch(mde_ctx* c, const mde_records* r, uint64_t span, unsigned long long* sums,
                        uint32_t* counts, mde::TaggedLaunch* out) {
  mde::TaggedLaunch& t = *out;
  t = mde::TaggedLaunch{};
  const uintptr_t v = reinterpret_cast<uintptr_t>(r->values);
  t.base = reinterpret_cast<const uint8_t*>(v & ~uintptr_t(15));
  t.shift = v & 15u;
  t.stride = r->value_stride;
  t.inv_stride = 1.0 / (double)r->value_stride;
  t.part_rec = r->part_rec;
  t.tag = r->bucket_tag;
  t.P = r->n_partitions;
  t.B = r->n_buckets;
  t.sums = sums;
  t.counts = counts;
  mde::plan_tagged((span ? span + 16 : r->values_bytes) + t.shift, c->cus, 8, &t.wave_bytes, &t.n_waves);
}

int tagged_async(mde_ctx* c, const mde_records* r, uint64_t span = 0, unsigned long long* sums = nullptr,
                 uint32_t* counts = nullptr) {
  mde::TaggedLaunch t;
  plan_tagged_launch(c, r, span, sums ? sums : c->sums, counts ? counts : c->counts, &t);
  MDE_HIP(c, mde::launch_tagged_digest(t, c->stream));
  return MDE_OK;
}

// Digest launch into explicit (zeroed) scratch.
int digest_into(mde_ctx* c, const mde_records* r, unsigned long long* sums, uint32_t* counts) {
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  if (S == 0 || r->n_records == 0 || r->values_bytes == 0) return MDE_OK;
  if (r->layout == MDE_LAYOUT_TAGGED) return tagged_async(c, r, 0, sums, counts);
  mde::DigestLaunch a{};
  a.seg = seg_desc(r);
  a.sums = sums;
  if (!c->digest_blocks_per_cu)
    c->digest_blocks_per_cu = mde::bucket_digest_blocks_per_cu(c->digest_variant, c->digest_cap);
  a.variant = c->digest_variant;
  int rc = plan_digest(c, r->values_bytes + a.seg.shift, &a);
  if (rc) return rc;
  MDE_HIP(c, mde::launch_bucket_digest(a, c->stream));
  return MDE_OK;
}

int digest_async(mde_ctx* c, const mde_records* r) {
  int rc = ensure_sums(c, (uint64_t)r->n_partitions * r->n_buckets);
  if (rc) return rc;
  return digest_into(c, r, c->sums, c->counts);
}

// Digest launch for a chunk whose values pointer is biased (mde_build_streamed): positions are
// global byte offsets, `end` is the chunk's end position, and the arena range actually read is
// [segpos(first bucket), end) -- inside the slot.
int digest_async_biased(mde_ctx* c, const mde_records* r, uint64_t end_pos, uint64_t span) {
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  int rc = ensure_sums(c, S);
  if (rc) return rc;
  if (S == 0 || r->n_records == 0) return MDE_OK;
  if (r->layout == MDE_LAYOUT_TAGGED) return tagged_async(c, r, span);
  mde::DigestLaunch a{};
  a.seg = seg_desc(r);
  a.seg.end = a.seg.shift + end_pos;
  a.sums = c->sums;
  if (!c->digest_blocks_per_cu)
    c->digest_blocks_per_cu = mde::bucket_digest_blocks_per_cu(c->digest_variant, c->digest_cap);
  a.variant = c->digest_variant;
  // plan over the bytes this chunk actually covers (span is known on the host)
  rc = plan_digest(c, span + 16, &a);
  if (rc) return rc;
  MDE_HIP(c, mde::launch_bucket_digest(a, c->stream));
  return MDE_OK;
}

// Tree launch of a build whose byte sums (and layout-B counts) sit in `sums` / `counts`.
int tree_launch_for(mde_ctx* c, const mde_records* r, const mde_tree_out* o, unsigned long long* sums,
                    uint32_t* counts, mde::TreeLaunch* t) {
  *t = mde::TreeLaunch{};
  t->P = r->n_partitions;
  t->B = r->n_buckets;
  t->sums_in = sums;
  t->sums_clear = sums;
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  t->seg_rec = tagged ? nullptr : r->seg_rec;
  t->counts_in = tagged ? counts : nullptr;
  t->digest_out = o->digest;
  t->size_out = o->size;
  t->items_out = o->items;
  t->root_out = o->root;
  t->nodes_out = o->nodes;
  t->n_int = mde::tree_internal(r->n_buckets);
  if (!t->nodes_out && o->root && r->n_buckets > mde::kTreeLdsMaxBuckets) {
    int rc = ensure_buf(c, c->nodes_scratch, (uint64_t)t->P * t->n_int * 32);
    if (rc) return rc;
    t->nodes_out = static_cast<uint8_t*>(c->nodes_scratch.p);
  }
  return MDE_OK;
}

// Outputs of a build: any pointer may be NULL; root == NULL (nodes then NULL too) is a digest-only
// build -- digests, sizes and items without the SHA-256 tree.
int check_out(mde_ctx* c, const mde_tree_out* o) {
  if (!o) return set_err(c, MDE_E_INVAL, "out is NULL");
  if (!o->root && o->nodes) return set_err(c, MDE_E_INVAL, "out/nodes needs out/root");
  return MDE_OK;
}

int tree_async(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  int rc0 = check_out(c, o);
  if (rc0) return rc0;
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  int rc = ensure_sums(c, S);
  if (rc) return rc;
  mde::TreeLaunch t;
  rc = tree_launch_for(c, r, o, c->sums, c->counts, &t);
  if (rc) return rc;
  MDE_HIP(c, mde::launch_tree(t, c->stream));
  return MDE_OK;
}

// digest + tree of one build on the context stream: one launch for a small layout-A arena
// (latency of the one-partition calls), else the digest kernel then the tree kernel.
void count_build(mde_ctx* c, const mde_records* r, uint64_t bytes) {
  c->st_builds++;
  c->st_parts += r->n_partitions;
  c->st_bytes += bytes;
}

int build_async_impl(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  count_build(c, r, r->values_bytes);
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  if (r->layout == MDE_LAYOUT_SORTED && S && r->n_records && r->values_bytes &&
      mde::small_build_fits(r->values_bytes + 16, r->n_partitions, r->n_buckets)) {
    int rc = ensure_sums(c, S);
    if (rc) return rc;
    mde::TreeLaunch t;
    if ((rc = tree_launch_for(c, r, o, c->sums, c->counts, &t))) return rc;
    MDE_HIP(c, mde::launch_small_build(seg_desc(r), t, c->stream));
    return MDE_OK;
  }
  int rc = digest_async(c, r);
  return rc ? rc : tree_async(c, r, o);
}

// The trees still owed by the pipeline, as a standalone launch.
int pipeline_drain(mde_ctx* c) {
  if (!c->pending.active) return MDE_OK;
  mde_ctx::Pending& pd = c->pending;
  pd.active = false;
  mde_ctx::Slot& sl = c->pipe[pd.slot];
  mde::TreeLaunch t;
  int rc = tree_launch_for(c, &pd.rec, &pd.out, sl.sums, sl.counts, &t);
  if (rc) return rc;
  hipError_t e = mde::launch_tree(t, c->stream);
  if (e != hipSuccess) sl.dirty = true;
  MDE_HIP(c, e);
  return MDE_OK;
}

// One pipelined build: digest `r` into the free slot and, in the same launch, build the trees of
// the pending build; `r` becomes the pending build. Layout B and B too wide for the fused step's
// LDS budget run as separate launches on the same stream (same results, no overlap).
int build_pipelined(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  const uint64_t S = (uint64_t)r->n_partitions * r->n_buckets;
  mde_ctx::Pending& pd = c->pending;
  const int slot = pd.active ? 1 - pd.slot : 0;
  mde_ctx::Slot& sl = c->pipe[slot];
  int rc = ensure_slot(c, sl, S);
  if (rc) return rc;
  // The digest role follows this build's layout (bucket_digest / tagged binning); the tree role
  // only needs the pending build's B to fit the packed trees' LDS budget.
  const bool fused = !pd.active || mde::build_step_fusable(pd.rec.n_buckets);
  if (!fused) {
    rc = pipeline_drain(c);
    if (rc) return rc;
    // digest into the slot through the standalone kernel, then make it pending
    rc = digest_into(c, r, sl.sums, sl.counts);
    if (rc) {
      sl.dirty = true;
      return rc;
    }
  } else if (r->layout == MDE_LAYOUT_TAGGED) {
    mde::TaggedLaunch a;
    plan_tagged_launch(c, r, 0, sl.sums, sl.counts, &a);
    if (!(S && r->n_records && r->values_bytes)) a.n_waves = 0;
    mde::TreeLaunch t;
    if (pd.active) {
      mde_ctx::Slot& ps = c->pipe[pd.slot];
      rc = tree_launch_for(c, &pd.rec, &pd.out, ps.sums, ps.counts, &t);
      if (rc) return rc;
    }
    hipError_t e = mde::launch_tagged_step(a, pd.active ? &t : nullptr, c->stream);
    if (e != hipSuccess) {
      sl.dirty = true;
      if (pd.active) c->pipe[pd.slot].dirty = true;
      pd.active = false;
    }
    MDE_HIP(c, e);
  } else {
    mde::DigestLaunch a{};
    if (S && r->n_records && r->values_bytes) {
      a.seg = seg_desc(r);
      if (!c->digest_blocks_per_cu)
        c->digest_blocks_per_cu = mde::bucket_digest_blocks_per_cu(c->digest_variant, c->digest_cap);
      a.variant = c->digest_variant;
      rc = plan_digest(c, r->values_bytes + a.seg.shift, &a);
      if (rc) return rc;
    }
    a.sums = sl.sums;
    mde::TreeLaunch t;
    if (pd.active) {
      mde_ctx::Slot& ps = c->pipe[pd.slot];
      rc = tree_launch_for(c, &pd.rec, &pd.out, ps.sums, ps.counts, &t);
      if (rc) return rc;
    }
    hipError_t e = mde::launch_build_step(a, pd.active ? &t : nullptr, c->stream);
    if (e != hipSuccess) {
      sl.dirty = true;
      if (pd.active) c->pipe[pd.slot].dirty = true;
      pd.active = false;
    }
    MDE_HIP(c, e);
  }
  pd.active = true;
  pd.slot = slot;
  pd.rec = *r;
  pd.out = *o;
  return MDE_OK;
}

// ordered: mde_stream_buckets' request-order contract (ExtractLaunch::ordered); else mde_extract's
// deduplicated ascending set
int extract_async(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                  const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                  uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap, int32_t* status,
                  bool ordered) {
  if (r->n_buckets > mde::kExtractMaxBuckets)
    return set_err(c, MDE_E_INVAL, "extract supports n_buckets <= %u", mde::kExtractMaxBuckets);
  if (ordered && r->layout == MDE_LAYOUT_TAGGED)
    return set_err(c, MDE_E_INVAL, "mde_stream_buckets needs layout A (a bucket's records in LSM order)");
  if (!ids || !counts || !part_off || !out_rec || !status || (out_values && !r->values))
    return set_err(c, MDE_E_INVAL, "bad extract arguments");
  int rc = ensure_buf(c, c->extract_scratch, 3 * ((uint64_t)r->n_partitions + 1) * 8);
  if (rc) return rc;
  mde::ExtractLaunch a{};
  if (r->layout == MDE_LAYOUT_TAGGED) {
    a.tag = r->bucket_tag;
    a.part_rec = r->part_rec;
    a.stride = r->value_stride;
  } else {
    a.seg = seg_desc(r);
  }
  a.values = r->values;
  a.P = r->n_partitions;
  a.B = r->n_buckets;
  a.ids = ids;
  a.ids_stride = ids_stride;
  a.counts = counts;
  a.part_off = part_off;
  a.out_rec = out_rec;
  a.rec_cap = rec_cap;
  a.out_values = out_values;
  a.out_value_off = out_value_off;
  a.bytes_cap = bytes_cap;
  a.status = status;
  a.scratch = static_cast<uint64_t*>(c->extract_scratch.p);
  a.ordered = ordered;
  MDE_HIP(c, mde::launch_extract(a, c->stream));
  return MDE_OK;
}

int tree_digests_async(mde_ctx* c, uint32_t n_trees, uint32_t B, const uint64_t* digest,
                       uint8_t* root, uint8_t* nodes) {
  if (B == 0 || !digest || !root) return set_err(c, MDE_E_INVAL, "bad tree_from_digests arguments");
  mde::TreeLaunch t{};
  t.P = n_trees;
  t.B = B;
  t.digest_in = digest;
  t.root_out = root;
  t.nodes_out = nodes;
  t.n_int = mde::tree_internal(B);
  if (!t.nodes_out && B > mde::kTreeLdsMaxBuckets) {
    int rc = ensure_buf(c, c->nodes_scratch, (uint64_t)n_trees * t.n_int * 32);
    if (rc) return rc;
    t.nodes_out = static_cast<uint8_t*>(c->nodes_scratch.p);
  }
  MDE_HIP(c, mde::launch_tree(t, c->stream));
  return MDE_OK;
}

// Default spill area for async decodes (objects of up to this many bytes in all never rescan).
constexpr uint64_t kDefaultDeepObjectBytes = 8ull << 20;

// The decode's spill area: at least the entries `n` objects of `bytes` bytes need (exact for the
// host-buffer calls), else whatever the context holds (async calls; mde_reserve_decode_scratch).
int attach_deep(mde_ctx* c, mde::WireDecodeLaunch* d, uint64_t n, uint64_t bytes) {
  const uint64_t want = mde::wire_deep_entries(n, bytes) * 4;
  int rc = ensure_buf(c, c->deep_scratch, std::max(want, c->deep_scratch.cap));
  if (rc) return rc;
  d->deep = static_cast<uint32_t*>(c->deep_scratch.p);
  d->deep_cap = c->deep_scratch.cap / 4;
  return MDE_OK;
}

}  // namespace

extern "C" {

int mde_abi_version(void) { return MDE_ABI_VERSION; }

int mde_device_list(int* ordinals, int cap) {
  int n = 0, k = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  for (int d = 0; d < n; d++) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) {
      if (ordinals && k < cap) ordinals[k] = d;
      k++;
    }
  }
  return k;
}

int mde_device_count(void) { return mde_device_list(nullptr, 0); }

int mde_reserve_decode_scratch(mde_ctx* c, uint64_t n_objects, uint64_t object_bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return ensure_buf(c, c->deep_scratch, std::max(mde::wire_deep_entries(n_objects, object_bytes) * 4,
                                                  c->deep_scratch.cap));
}

const char* mde_strerror(int code) {
  switch (code) {
    case MDE_OK: return "ok";
    case MDE_E_INVAL: return "invalid argument";
    case MDE_E_NOMEM: return "out of memory";
    case MDE_E_DEVICE: return "device error";
    case MDE_E_TREE: return "merkle trees do not match in shape";
    case MDE_E_CAPACITY: return "output capacity too small";
    case MDE_E_DECODE: return "byte slice should be 8 bytes long for int64 decoding";
    default: return "unknown error";
  }
}

int mde_create(int device, mde_ctx** out) {
  if (!out) return MDE_E_INVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MDE_E_DEVICE;
  if (device < 0 || device >= n) return MDE_E_INVAL;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return MDE_E_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MDE_E_DEVICE;  // gfx950-only code objects
  mde_ctx* c = new (std::nothrow) mde_ctx();
  if (!c) return MDE_E_NOMEM;
  c->device = device;
  c->cus = prop.multiProcessorCount;
  std::snprintf(c->arch, sizeof c->arch, "%s", prop.gcnArchName);
  DeviceScope ds(device);
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault) != hipSuccess) {
    delete c;
    return MDE_E_DEVICE;
  }
  c->stream = c->own_stream;
  if (const char* e = std::getenv("MDE_DIRECT_OUT")) c->direct_out = std::atoi(e) != 0;  // A/B switch
  *out = c;
  return MDE_OK;
}

void mde_destroy(mde_ctx* c) {
  if (!c) return;
  // MDE_TEARDOWN_TRACE=1: one stderr line before each step (a teardown that hangs names its step)
  static const bool trace = std::getenv("MDE_TEARDOWN_TRACE") != nullptr;
  auto step = [&](const char* what) {
    if (trace) std::fprintf(stderr, "mde_destroy(%p): %s\n", static_cast<void*>(c), what), std::fflush(stderr);
  };
  {
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceScope ds(c->device);
    step("synchronize the stream");
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    step("free device buffers");
    if (c->sums) (void)hipFree(c->sums);
    if (c->counts) (void)hipFree(c->counts);
    for (auto& sl : c->pipe) {
      if (sl.sums) (void)hipFree(sl.sums);
      if (sl.counts) (void)hipFree(sl.counts);
    }
    for (auto& b : c->stage)
      if (b.p) (void)hipFree(b.p);
    if (c->nodes_scratch.p) (void)hipFree(c->nodes_scratch.p);
    if (c->packed_in.p) (void)hipFree(c->packed_in.p);
    if (c->packed_out.p) (void)hipFree(c->packed_out.p);
    step("free pinned host buffers");
    if (c->pin_in.p) (void)hipHostFree(c->pin_in.p);
    if (c->pin_out.p) (void)hipHostFree(c->pin_out.p);
    step("free scratch");
    if (c->extract_scratch.p) (void)hipFree(c->extract_scratch.p);
    if (c->verify_scratch.p) (void)hipFree(c->verify_scratch.p);
    if (c->deep_scratch.p) (void)hipFree(c->deep_scratch.p);
    step("free rings and events");
    for (int i = 0; i < 2; i++) {
      for (auto* b : {&c->ring_vals[i], &c->ring_voff[i], &c->ring_seg[i]})
        if (b->p) (void)hipFree(b->p);
      if (c->ev_loaded[i]) (void)hipEventDestroy(c->ev_loaded[i]);
      if (c->ev_done[i]) (void)hipEventDestroy(c->ev_done[i]);
    }
    step(c->copy_stream ? "destroy the copy stream" : "no copy stream");
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    step("destroy the own stream");
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    step("done");
  }
  delete c;
}

const char* mde_last_error(mde_ctx* c) { return c ? c->err.c_str() : "null context"; }

namespace {
uint64_t copy_message(const std::string& m, char* buf, uint64_t cap) {
  if (buf && cap) {
    const uint64_t n = std::min<uint64_t>(m.size(), cap - 1);
    std::memcpy(buf, m.data(), n);
    buf[n] = 0;
  }
  return m.size();
}
}  // namespace

uint64_t mde_last_error_copy(mde_ctx* c, char* buf, uint64_t cap) {
  if (!c) return copy_message("null context", buf, cap);
  std::lock_guard<std::mutex> lk(c->mu);
  return copy_message(c->err, buf, cap);
}

int mde_set_tuning(mde_ctx* c, int digest_variant, int digest_blocks_per_cu, int digest_oversub) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (digest_variant >= 0 && !mde::bucket_digest_variant_valid(digest_variant))
    return set_err(c, MDE_E_INVAL, "digest variant %d is not one of 11..16", digest_variant);
  c->digest_variant = digest_variant < 0 ? kDefaultDigestVariant : digest_variant;
  c->digest_auto = digest_variant < 0;
  c->digest_cap = digest_blocks_per_cu < 0 ? kDefaultDigestCap : digest_blocks_per_cu;
  c->digest_oversub = digest_oversub < 0 ? kDefaultDigestOversub : (digest_oversub ? digest_oversub : 1);
  c->digest_blocks_per_cu = 0;  // re-query
  for (int& x : c->variant_blocks) x = 0;
  return MDE_OK;
}

int mde_ctx_stats(mde_ctx* c, uint64_t* builds, uint64_t* partitions, uint64_t* value_bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (builds) *builds = c->st_builds;
  if (partitions) *partitions = c->st_parts;
  if (value_bytes) *value_bytes = c->st_bytes;
  return MDE_OK;
}

int mde_set_digest_piece_bytes(mde_ctx* c, uint64_t piece_bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  c->digest_piece_bytes = piece_bytes;  // UINT64_MAX = kAutoPieceBytes
  return MDE_OK;
}

int mde_set_verify_mode(mde_ctx* c, int mode) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (mode < 0 || mode > 1) return set_err(c, MDE_E_INVAL, "verify mode %d out of range", mode);
  c->verify_chain = mode == 1;
  return MDE_OK;
}

int mde_use_own_stream(mde_ctx* c) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  c->stream = c->own_stream;
  return MDE_OK;
}

int mde_set_stream(mde_ctx* c, void* s) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  c->stream = static_cast<hipStream_t>(s);  // NULL = the null stream (torch's default stream)
  return MDE_OK;
}

void* mde_get_stream(mde_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int mde_synchronize(mde_ctx* c) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_device_info(mde_ctx* c, int* cu_count, char* arch, int cap) {
  if (!c) return MDE_E_INVAL;
  if (cu_count) *cu_count = c->cus;
  if (arch && cap > 0) std::snprintf(arch, (size_t)cap, "%s", c->arch);
  return MDE_OK;
}

uint32_t mde_tree_depth(uint32_t B) { return B ? mde::tree_levels(B, nullptr) - 1 : 0; }
uint64_t mde_tree_internal_nodes(uint32_t B) { return B ? mde::tree_internal(B) : 0; }
uint64_t mde_tree_prefix_nodes(uint32_t B, uint32_t top_nodes) {
  if (!B) return 0;
  uint64_t t = 0;
  uint32_t n = (B + 1) / 2;  // level 1 (the duplicate leaf of an odd B included)
  const uint32_t stop = top_nodes ? top_nodes : 1u;
  for (;;) {
    t += n;
    if (n <= stop) return t;
    n = (n + 1) / 2;
  }
}
uint64_t mde_diff_capacity(uint32_t a, uint32_t b) {
  if (!a || !b) return 0;
  uint32_t d = mde_tree_depth(a) < mde_tree_depth(b) ? mde_tree_depth(a) : mde_tree_depth(b);
  return 1ull << d;
}

int mde_digest_async(mde_ctx* c, const mde_records* r) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  return rc ? rc : digest_async(c, r);
}

int mde_tree_async(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  return rc ? rc : tree_async(c, r, o);
}

int mde_build_async(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  if (rc) return rc;
  if ((rc = check_out(c, o))) return rc;
  return build_async_impl(c, r, o);
}

int mde_build_pipelined_async(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  if (rc) return rc;
  if (!o || !o->root) return set_err(c, MDE_E_INVAL, "out/root is NULL");
  count_build(c, r, r->values_bytes);
  return build_pipelined(c, r, o);
}

int mde_build_pipeline_drain_async(mde_ctx* c) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return pipeline_drain(c);
}

int mde_build(mde_ctx* c, const mde_records* r, const mde_tree_out* o) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  if (rc) return rc;
  if ((rc = check_host_records(c, r))) return rc;
  if ((rc = check_out(c, o))) return rc;
  const uint64_t P = r->n_partitions, S = P * r->n_buckets, NI = mde::tree_internal(r->n_buckets);
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  const uint64_t nvo = r->value_stride ? 0 : (r->n_records + 1);
  const uint64_t nseg = (tagged ? P + 1 : S + 1) * 8, ntag = tagged ? r->n_records * 2 : 0;
  HostIo io(c);
  const int i_val = io.in(r->values, r->values_bytes, r->values_bytes);
  const int i_voff = io.in(r->value_off, nvo * 8, nvo * 8);
  const int i_seg = io.in(tagged ? r->part_rec : r->seg_rec, nseg, nseg);
  const int i_tag = io.in(r->bucket_tag, ntag, ntag);
  // every output is stored once by the tree pass (wider trees re-read their node levels)
  const bool wo = r->n_buckets <= mde::kTreeLdsMaxBuckets;
  const int o_dig = io.out(o->digest, S * 8, wo), o_size = io.out(o->size, S * 4, wo),
            o_items = io.out(o->items, P * 4, wo);
  const int o_root = io.out(o->root, o->root ? P * 32 : 0, wo), o_nodes = io.out(o->nodes, o->nodes ? P * NI * 32 : 0, wo);
  if ((rc = io.upload())) return rc;
  mde_records dr = *r;
  dr.values = static_cast<const uint8_t*>(io.dev(i_val));
  dr.value_off = nvo ? static_cast<const uint64_t*>(io.dev(i_voff)) : nullptr;
  dr.seg_rec = tagged ? nullptr : static_cast<const uint64_t*>(io.dev(i_seg));
  dr.part_rec = tagged ? static_cast<const uint64_t*>(io.dev(i_seg)) : nullptr;
  dr.bucket_tag = tagged ? static_cast<const uint16_t*>(io.dev(i_tag)) : nullptr;
  mde_tree_out dout{static_cast<uint64_t*>(io.dev(o_dig)), static_cast<int32_t*>(io.dev(o_size)),
                    static_cast<int32_t*>(io.dev(o_items)), o->root ? static_cast<uint8_t*>(io.dev(o_root)) : nullptr,
                    o->nodes ? static_cast<uint8_t*>(io.dev(o_nodes)) : nullptr};
  if ((rc = build_async_impl(c, &dr, &dout))) return rc;
  return io.download();
}

int mde_build_streamed(mde_ctx* c, const mde_records* r, const mde_tree_out* o, uint64_t chunk_bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  if (rc) return rc;
  if ((rc = check_host_records(c, r))) return rc;
  if (!o || !o->root) return set_err(c, MDE_E_INVAL, "out/root is NULL");
  if (!chunk_bytes) chunk_bytes = 256ull << 20;
  if (!c->copy_stream) {
    MDE_HIP(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
      MDE_HIP(c, hipEventCreateWithFlags(&c->ev_loaded[i], hipEventDisableTiming));
      MDE_HIP(c, hipEventCreateWithFlags(&c->ev_done[i], hipEventDisableTiming));
    }
  }
  // every return waits for the copies and builds this call issued (they read the caller's arena)
  SyncOnReturn drain_copy{c->copy_stream}, drain{c->stream};
  const uint32_t P = r->n_partitions, B = r->n_buckets;
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  const uint64_t NI = mde::tree_internal(B);
  auto pos = [&](uint64_t rr) { return r->value_stride ? rr * r->value_stride : r->value_off[rr]; };
  // first record of partition p (p <= P); layout A: of its first bucket segment
  auto prec = [&](uint64_t p) { return tagged ? r->part_rec[p] : r->seg_rec[p * B]; };
  const uint64_t per_part = tagged ? 1 : B;  // index entries per partition
  // Chunks of whole partitions, ~chunk_bytes each.
  std::vector<uint32_t> cuts{0};
  uint64_t max_bytes = 0, max_recs = 0, max_parts = 0;
  for (uint32_t p = 0; p < P;) {
    const uint64_t b0 = pos(prec(p));
    uint32_t q = p + 1;
    while (q < P && pos(prec(q + 1)) - b0 <= chunk_bytes) q++;
    cuts.push_back(q);
    max_bytes = std::max(max_bytes, pos(prec(q)) - b0);
    max_recs = std::max(max_recs, prec(q) - prec(p));
    max_parts = std::max<uint64_t>(max_parts, q - p);
    p = q;
  }
  for (int i = 0; i < 2; i++) {
    if ((rc = ensure_buf(c, c->ring_vals[i], max_bytes + 32))) return rc;
    if ((rc = ensure_buf(c, c->ring_seg[i], (max_parts * per_part + 1) * 8))) return rc;
    if (!r->value_stride && (rc = ensure_buf(c, c->ring_voff[i], (max_recs + 1) * 8))) return rc;
    if (tagged && (rc = ensure_buf(c, c->ring_voff[i], max_recs * 2 + 16))) return rc;  // tags
  }
  // Device outputs for the whole build (host copies at the end).
  const uint64_t S = (uint64_t)P * B;
  const uint64_t osz[5] = {S * 8, S * 4, (uint64_t)P * 4, (uint64_t)P * 32, o->nodes ? P * NI * 32 : 0};
  for (int i = 0; i < 5; i++)
    if ((rc = ensure_buf(c, c->stage[11 + i], osz[i]))) return rc;
  uint64_t* d_digest = static_cast<uint64_t*>(c->stage[11].p);
  int32_t* d_size = static_cast<int32_t*>(c->stage[12].p);
  int32_t* d_items = static_cast<int32_t*>(c->stage[13].p);
  uint8_t* d_root = static_cast<uint8_t*>(c->stage[14].p);
  uint8_t* d_nodes = o->nodes ? static_cast<uint8_t*>(c->stage[15].p) : nullptr;
  MDE_HIP(c, hipEventRecord(c->ev_done[0], c->stream));
  MDE_HIP(c, hipEventRecord(c->ev_done[1], c->stream));
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    const int slot = (int)(k & 1);
    const uint32_t p0 = cuts[k], p1 = cuts[k + 1];
    const uint64_t r0 = prec(p0), r1 = prec(p1);
    const uint64_t byte0 = pos(r0), byte1 = pos(r1);
    uint8_t* vslot = static_cast<uint8_t*>(c->ring_vals[slot].p);
    // copy stream: wait until the build two chunks back released this slot, then load
    MDE_HIP(c, hipStreamWaitEvent(c->copy_stream, c->ev_done[slot], 0));
    if (byte1 > byte0)
      MDE_HIP(c, hipMemcpyAsync(vslot + (byte0 & 15), r->values + byte0, byte1 - byte0,
                                hipMemcpyHostToDevice, c->copy_stream));
    MDE_HIP(c, hipMemcpyAsync(c->ring_seg[slot].p, tagged ? r->part_rec + p0 : r->seg_rec + (uint64_t)p0 * B,
                              ((uint64_t)(p1 - p0) * per_part + 1) * 8, hipMemcpyHostToDevice, c->copy_stream));
    if (tagged && r1 > r0)
      MDE_HIP(c, hipMemcpyAsync(c->ring_voff[slot].p, r->bucket_tag + r0, (r1 - r0) * 2, hipMemcpyHostToDevice,
                                c->copy_stream));
    if (!r->value_stride)
      MDE_HIP(c, hipMemcpyAsync(c->ring_voff[slot].p, r->value_off + r0, (r1 - r0 + 1) * 8,
                                hipMemcpyHostToDevice, c->copy_stream));
    MDE_HIP(c, hipEventRecord(c->ev_loaded[slot], c->copy_stream));
    // compute stream: build the chunk. Record indices stay global; the value and value_off
    // pointers are biased so that global offsets land in the slot (never dereferenced outside).
    MDE_HIP(c, hipStreamWaitEvent(c->stream, c->ev_loaded[slot], 0));
    mde_records cr = *r;
    cr.values = vslot - (byte0 & ~uint64_t(15));
    cr.values_bytes = byte1 - (byte0 & ~uint64_t(15));
    cr.value_off = r->value_stride ? nullptr : static_cast<const uint64_t*>(c->ring_voff[slot].p) - r0;
    cr.n_partitions = p1 - p0;
    if (tagged) {  // part_rec keeps global record indices; the tags pointer is biased like values
      cr.part_rec = static_cast<const uint64_t*>(c->ring_seg[slot].p);
      cr.bucket_tag = static_cast<const uint16_t*>(c->ring_voff[slot].p) - r0;
    } else {
      cr.seg_rec = static_cast<const uint64_t*>(c->ring_seg[slot].p);
    }
    mde_tree_out co{d_digest + (uint64_t)p0 * B, d_size + (uint64_t)p0 * B, d_items + p0,
                    d_root + (uint64_t)p0 * 32, d_nodes ? d_nodes + (uint64_t)p0 * NI * 32 : nullptr};
    count_build(c, &cr, byte1 - byte0);
    if (byte1 > byte0 && (rc = digest_async_biased(c, &cr, byte1, byte1 - byte0))) return rc;
    if ((rc = tree_async(c, &cr, &co))) return rc;
    MDE_HIP(c, hipEventRecord(c->ev_done[slot], c->stream));
  }
  if (o->digest) MDE_HIP(c, hipMemcpyAsync(o->digest, d_digest, S * 8, hipMemcpyDeviceToHost, c->stream));
  if (o->size) MDE_HIP(c, hipMemcpyAsync(o->size, d_size, S * 4, hipMemcpyDeviceToHost, c->stream));
  if (o->items) MDE_HIP(c, hipMemcpyAsync(o->items, d_items, (uint64_t)P * 4, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipMemcpyAsync(o->root, d_root, (uint64_t)P * 32, hipMemcpyDeviceToHost, c->stream));
  if (o->nodes) MDE_HIP(c, hipMemcpyAsync(o->nodes, d_nodes, P * NI * 32, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_tree_from_digests_async(mde_ctx* c, uint32_t n_trees, uint32_t B, const uint64_t* digest,
                                uint8_t* root, uint8_t* nodes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return tree_digests_async(c, n_trees, B, digest, root, nodes);
}

int mde_tree_from_digests(mde_ctx* c, uint32_t n_trees, uint32_t B, const uint64_t* digest,
                          uint8_t* root, uint8_t* nodes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  SyncOnReturn drain{c->stream};  // every return waits for the copies this call issued
  if (B == 0 || !digest || !root) return set_err(c, MDE_E_INVAL, "bad tree_from_digests arguments");
  const uint64_t T = n_trees, NI = mde::tree_internal(B);
  int rc;
  if ((rc = ensure_buf(c, c->stage[8], T * B * 8))) return rc;
  if ((rc = ensure_buf(c, c->stage[9], T * 32))) return rc;
  if ((rc = ensure_buf(c, c->stage[10], nodes ? T * NI * 32 : 0))) return rc;
  MDE_HIP(c, hipMemcpyAsync(c->stage[8].p, digest, T * B * 8, hipMemcpyHostToDevice, c->stream));
  rc = tree_digests_async(c, n_trees, B, static_cast<const uint64_t*>(c->stage[8].p),
                          static_cast<uint8_t*>(c->stage[9].p),
                          nodes ? static_cast<uint8_t*>(c->stage[10].p) : nullptr);
  if (rc) return rc;
  MDE_HIP(c, hipMemcpyAsync(root, c->stage[9].p, T * 32, hipMemcpyDeviceToHost, c->stream));
  if (nodes) MDE_HIP(c, hipMemcpyAsync(nodes, c->stage[10].p, T * NI * 32, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_decode_bucket_hashes(const uint8_t* const* hashes, const uint32_t* lens, uint32_t n,
                             uint64_t* out) {
  if ((!hashes || !lens || !out) && n) return MDE_E_INVAL;
  for (uint32_t i = 0; i < n; i++) {
    if (lens[i] != 8 || !hashes[i]) return MDE_E_DECODE;  // utils.DecodeBytesToInt64
    uint64_t v = 0;
    for (int k = 7; k >= 0; k--) v = (v << 8) | hashes[i][k];
    out[i] = v;
  }
  return MDE_OK;
}

int mde_diff_async(mde_ctx* c, uint32_t n_pairs, uint32_t Ba, const uint64_t* da,
                   const uint8_t* na, uint32_t Bb, const uint64_t* db, const uint8_t* nb,
                   int32_t* out_ids, uint64_t out_stride, int32_t* out_count) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!Ba || !Bb || !da || !db || !na || !nb || !out_ids || !out_count)
    return set_err(c, MDE_E_INVAL, "bad diff arguments");
  if (out_stride < mde_diff_capacity(Ba, Bb))
    return set_err(c, MDE_E_CAPACITY, "out_stride %llu < mde_diff_capacity %llu",
                   (unsigned long long)out_stride, (unsigned long long)mde_diff_capacity(Ba, Bb));
  mde::DiffLaunch a{n_pairs, Ba, Bb, da, na, db, nb, out_ids, out_stride, out_count};
  MDE_HIP(c, mde::launch_diff(a, c->stream));
  return MDE_OK;
}

int mde_diff(mde_ctx* c, uint32_t n_pairs, uint32_t Ba, const uint64_t* da, const uint8_t* na,
             uint32_t Bb, const uint64_t* db, const uint8_t* nb, int32_t* out_ids,
             uint64_t out_stride, int32_t* out_count) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!Ba || !Bb || !da || !db || !na || !nb || !out_ids || !out_count)
    return set_err(c, MDE_E_INVAL, "bad diff arguments");
  if (out_stride < mde_diff_capacity(Ba, Bb))
    return set_err(c, MDE_E_CAPACITY, "out_stride too small");
  const uint64_t T = n_pairs, NA = mde::tree_internal(Ba), NB = mde::tree_internal(Bb);
  HostIo io(c);
  const int i_da = io.in(da, T * Ba * 8, T * Ba * 8), i_na = io.in(na, T * NA * 32, T * NA * 32);
  const int i_db = io.in(db, T * Bb * 8, T * Bb * 8), i_nb = io.in(nb, T * NB * 32, T * NB * 32);
  const int o_ids = io.out(out_ids, T * out_stride * 4), o_cnt = io.out(out_count, T * 4);
  int rc = io.upload();
  if (rc) return rc;
  mde::DiffLaunch a{n_pairs,
                    Ba,
                    Bb,
                    static_cast<const uint64_t*>(io.dev(i_da)),
                    static_cast<const uint8_t*>(io.dev(i_na)),
                    static_cast<const uint64_t*>(io.dev(i_db)),
                    static_cast<const uint8_t*>(io.dev(i_nb)),
                    static_cast<int32_t*>(io.dev(o_ids)),
                    out_stride,
                    static_cast<int32_t*>(io.dev(o_cnt))};
  MDE_HIP(c, mde::launch_diff(a, c->stream));
  return io.download();
}

int mde_diff_digests(mde_ctx* c, uint32_t n_pairs, uint32_t Ba, const uint64_t* da, uint32_t Bb,
                     const uint64_t* db, int32_t* out_ids, uint64_t out_stride, int32_t* out_count) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  SyncOnReturn drain{c->stream};  // every return waits for the copies this call issued
  if (!Ba || !Bb || !da || !db || !out_ids || !out_count)
    return set_err(c, MDE_E_INVAL, "bad diff arguments");
  if (out_stride < mde_diff_capacity(Ba, Bb))
    return set_err(c, MDE_E_CAPACITY, "out_stride too small");
  const uint64_t T = n_pairs, NA = mde::tree_internal(Ba), NB = mde::tree_internal(Bb);
  const uint64_t sz[8] = {T * Ba * 8, T * NA * 32, T * Bb * 8, T * NB * 32, T * out_stride * 4, T * 4,
                          T * 32, T * 32};
  int rc;
  for (int i = 0; i < 8; i++)
    if ((rc = ensure_buf(c, c->stage[i], sz[i]))) return rc;
  MDE_HIP(c, hipMemcpyAsync(c->stage[0].p, da, sz[0], hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(c->stage[2].p, db, sz[2], hipMemcpyHostToDevice, c->stream));
  if ((rc = tree_digests_async(c, n_pairs, Ba, static_cast<const uint64_t*>(c->stage[0].p),
                               static_cast<uint8_t*>(c->stage[6].p), static_cast<uint8_t*>(c->stage[1].p))))
    return rc;
  if ((rc = tree_digests_async(c, n_pairs, Bb, static_cast<const uint64_t*>(c->stage[2].p),
                               static_cast<uint8_t*>(c->stage[7].p), static_cast<uint8_t*>(c->stage[3].p))))
    return rc;
  mde::DiffLaunch a{n_pairs,
                    Ba,
                    Bb,
                    static_cast<const uint64_t*>(c->stage[0].p),
                    static_cast<const uint8_t*>(c->stage[1].p),
                    static_cast<const uint64_t*>(c->stage[2].p),
                    static_cast<const uint8_t*>(c->stage[3].p),
                    static_cast<int32_t*>(c->stage[4].p),
                    out_stride,
                    static_cast<int32_t*>(c->stage[5].p)};
  MDE_HIP(c, mde::launch_diff(a, c->stream));
  MDE_HIP(c, hipMemcpyAsync(out_ids, c->stage[4].p, sz[4], hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipMemcpyAsync(out_count, c->stage[5].p, sz[5], hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_extract_async(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                      const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                      uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap,
                      int32_t* status) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  return rc ? rc : extract_async(c, r, ids, ids_stride, counts, part_off, out_rec, rec_cap, out_values,
                                 out_value_off, bytes_cap, status, false);
}

int mde_stream_buckets_async(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                             const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                             uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap,
                             int32_t* status) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  int rc = check_records(c, r);
  return rc ? rc : extract_async(c, r, ids, ids_stride, counts, part_off, out_rec, rec_cap, out_values,
                                 out_value_off, bytes_cap, status, true);
}

namespace {
// mde_extract / mde_stream_buckets over host buffers: stage, extract, copy back.
int extract_host(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                 const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                 uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap, bool ordered) {
  SyncOnReturn drain{c->stream};  // every return waits for the copies this call issued
  int rc = check_records(c, r);
  if (rc) return rc;
  if ((rc = check_host_records(c, r))) return rc;
  if (!ids || !counts || !part_off || !out_rec) return set_err(c, MDE_E_INVAL, "bad extract arguments");
  const uint64_t P = r->n_partitions, S = P * r->n_buckets;
  const bool tagged = r->layout == MDE_LAYOUT_TAGGED;
  const uint64_t nvo = r->value_stride ? 0 : (r->n_records + 1);
  const uint64_t sz[11] = {r->values_bytes, nvo * 8, tagged ? (P + 1) * 8 : (S + 1) * 8, P * ids_stride * 4, P * 4,
                           (P + 1) * 8, rec_cap * 8, out_values ? bytes_cap : 0,
                           out_value_off ? (rec_cap + 1) * 8 : 0, 4, tagged ? r->n_records * 2 : 0};
  for (int i = 0; i < 11; i++)
    if ((rc = ensure_buf(c, c->stage[i], sz[i]))) return rc;
  auto dp = [&](int i) { return c->stage[i].p; };
  if (r->values_bytes)
    MDE_HIP(c, hipMemcpyAsync(dp(0), r->values, r->values_bytes, hipMemcpyHostToDevice, c->stream));
  if (nvo) MDE_HIP(c, hipMemcpyAsync(dp(1), r->value_off, nvo * 8, hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(dp(2), tagged ? r->part_rec : r->seg_rec, sz[2], hipMemcpyHostToDevice, c->stream));
  if (tagged && sz[10]) MDE_HIP(c, hipMemcpyAsync(dp(10), r->bucket_tag, sz[10], hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(dp(3), ids, sz[3], hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(dp(4), counts, sz[4], hipMemcpyHostToDevice, c->stream));
  mde_records dr = *r;
  dr.values = static_cast<const uint8_t*>(dp(0));
  dr.value_off = nvo ? static_cast<const uint64_t*>(dp(1)) : nullptr;
  dr.seg_rec = tagged ? nullptr : static_cast<const uint64_t*>(dp(2));
  dr.part_rec = tagged ? static_cast<const uint64_t*>(dp(2)) : nullptr;
  dr.bucket_tag = tagged ? static_cast<const uint16_t*>(dp(10)) : nullptr;
  rc = extract_async(c, &dr, static_cast<const int32_t*>(dp(3)), ids_stride,
                     static_cast<const int32_t*>(dp(4)), static_cast<uint64_t*>(dp(5)),
                     static_cast<uint64_t*>(dp(6)), rec_cap,
                     out_values ? static_cast<uint8_t*>(dp(7)) : nullptr,
                     out_value_off ? static_cast<uint64_t*>(dp(8)) : nullptr, bytes_cap,
                     static_cast<int32_t*>(dp(9)), ordered);
  if (rc) return rc;
  int32_t status = 0;
  MDE_HIP(c, hipMemcpyAsync(&status, dp(9), 4, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipMemcpyAsync(part_off, dp(5), (P + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  if (status != 0) return set_err(c, MDE_E_CAPACITY, "extract needs %llu records",
                                  (unsigned long long)part_off[P]);
  const uint64_t n = part_off[P];
  if (n) MDE_HIP(c, hipMemcpyAsync(out_rec, dp(6), n * 8, hipMemcpyDeviceToHost, c->stream));
  if (out_value_off)
    MDE_HIP(c, hipMemcpyAsync(out_value_off, dp(8), (n + 1) * 8, hipMemcpyDeviceToHost, c->stream));
  if (out_values) {
    uint64_t nbytes = 0;
    if (out_value_off) {
      MDE_HIP(c, hipStreamSynchronize(c->stream));
      nbytes = out_value_off[n];
    } else {
      nbytes = bytes_cap;  // copy the whole buffer (unused tail is unspecified)
    }
    if (nbytes) MDE_HIP(c, hipMemcpyAsync(out_values, dp(7), nbytes, hipMemcpyDeviceToHost, c->stream));
  }
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}
}  // namespace

int mde_extract(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return extract_host(c, r, ids, ids_stride, counts, part_off, out_rec, rec_cap, out_values, out_value_off,
                      bytes_cap, false);
}

int mde_stream_buckets(mde_ctx* c, const mde_records* r, const int32_t* ids, uint64_t ids_stride,
                       const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                       uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return extract_host(c, r, ids, ids_stride, counts, part_off, out_rec, rec_cap, out_values, out_value_off,
                      bytes_cap, true);
}

uint64_t mde_epoch_tree_object_max_bytes(uint32_t B) { return mde::wire_max_bytes(B); }

int mde_encode_epoch_tree_objects_async(mde_ctx* c, uint32_t n, uint32_t B, const int32_t* partition,
                                        int64_t lower, int64_t upper, const uint64_t* digest,
                                        const int32_t* size, const uint8_t* valid, const int32_t* items,
                                        uint8_t* out, uint64_t out_stride, uint32_t* out_len) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if ((B && (!digest || !size)) || !out || !out_len) return set_err(c, MDE_E_INVAL, "bad encode arguments");
  if (out_stride < mde::wire_max_bytes(B)) return set_err(c, MDE_E_CAPACITY, "out_stride too small");
  mde::WireEncodeLaunch a{n, B, partition, lower, upper, digest, size, valid, items, out, out_stride, out_len};
  MDE_HIP(c, mde::launch_wire_encode(a, c->stream));
  return MDE_OK;
}

int mde_encode_epoch_tree_objects(mde_ctx* c, uint32_t n, uint32_t B, const int32_t* partition,
                                  int64_t lower, int64_t upper, const uint64_t* digest, const int32_t* size,
                                  const uint8_t* valid, const int32_t* items, uint8_t* out,
                                  uint64_t out_stride, uint32_t* out_len) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  SyncOnReturn drain{c->stream};  // every return waits for the copies this call issued
  if ((B && (!digest || !size)) || !out || !out_len) return set_err(c, MDE_E_INVAL, "bad encode arguments");
  if (out_stride < mde::wire_max_bytes(B)) return set_err(c, MDE_E_CAPACITY, "out_stride too small");
  const uint64_t N = n;
  const uint64_t sz[7] = {N * 4, N * B * 8, N * B * 4, N, N * 4, N * out_stride, N * 4};
  int rc;
  for (int i = 0; i < 7; i++)
    if ((rc = ensure_buf(c, c->stage[i], sz[i]))) return rc;
  auto up = [&](int i, const void* src) -> int {
    if (!src) return MDE_OK;
    MDE_HIP(c, hipMemcpyAsync(c->stage[i].p, src, sz[i], hipMemcpyHostToDevice, c->stream));
    return MDE_OK;
  };
  if ((rc = up(0, partition)) || (rc = up(1, digest)) || (rc = up(2, size)) || (rc = up(3, valid)) ||
      (rc = up(4, items)))
    return rc;
  mde::WireEncodeLaunch a{n,
                          B,
                          partition ? static_cast<const int32_t*>(c->stage[0].p) : nullptr,
                          lower,
                          upper,
                          static_cast<const uint64_t*>(c->stage[1].p),
                          static_cast<const int32_t*>(c->stage[2].p),
                          valid ? static_cast<const uint8_t*>(c->stage[3].p) : nullptr,
                          items ? static_cast<const int32_t*>(c->stage[4].p) : nullptr,
                          static_cast<uint8_t*>(c->stage[5].p),
                          out_stride,
                          static_cast<uint32_t*>(c->stage[6].p)};
  MDE_HIP(c, mde::launch_wire_encode(a, c->stream));
  MDE_HIP(c, hipMemcpyAsync(out, c->stage[5].p, sz[5], hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipMemcpyAsync(out_len, c->stage[6].p, sz[6], hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_decode_epoch_tree_objects_async(mde_ctx* c, uint32_t n, const uint8_t* bytes, const uint64_t* off,
                                        uint32_t cap, int32_t* partition, int64_t* lower, int64_t* upper,
                                        uint64_t* digest, int32_t* size, uint8_t* valid, int32_t* items,
                                        int32_t* n_buckets) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!off || !digest || !size || !n_buckets || (n && !bytes))
    return set_err(c, MDE_E_INVAL, "bad decode arguments");
  mde::WireDecodeLaunch a{n, bytes, off, cap, partition, lower, upper, digest, size, valid, items, n_buckets};
  int rc = attach_deep(c, &a, 0, kDefaultDeepObjectBytes);
  if (rc) return rc;
  MDE_HIP(c, mde::launch_wire_decode(a, c->stream));
  return MDE_OK;
}

int mde_decode_epoch_tree_objects(mde_ctx* c, uint32_t n, const uint8_t* bytes, const uint64_t* off,
                                  uint32_t cap, int32_t* partition, int64_t* lower, int64_t* upper,
                                  uint64_t* digest, int32_t* size, uint8_t* valid, int32_t* items,
                                  int32_t* n_buckets) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!off || !digest || !size || !n_buckets || (n && !bytes))
    return set_err(c, MDE_E_INVAL, "bad decode arguments");
  for (uint32_t i = 0; i < n; i++)
    if (off[i] > off[i + 1]) return set_err(c, MDE_E_INVAL, "off not nondecreasing");
  const uint64_t N = n, nbytes = off[n] - off[0];
  const uint64_t sz[11] = {nbytes + 1, (N + 1) * 8, N * 4, N * 8, N * 8, N * cap * 8, N * cap * 4, N, N * 4, N * 4, 0};
  int rc;
  for (int i = 0; i < 10; i++)
    if ((rc = ensure_buf(c, c->stage[i], sz[i]))) return rc;
  std::vector<uint64_t> rel(N + 1);
  SyncOnReturn drain{c->stream};  // declared after rel: an early return waits before rel is freed
  for (uint64_t i = 0; i <= N; i++) rel[i] = off[i] - off[0];
  if (nbytes) MDE_HIP(c, hipMemcpyAsync(c->stage[0].p, bytes + off[0], nbytes, hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(c->stage[1].p, rel.data(), (N + 1) * 8, hipMemcpyHostToDevice, c->stream));
  auto dp = [&](int i) { return c->stage[i].p; };
  mde::WireDecodeLaunch a{n,
                          static_cast<const uint8_t*>(dp(0)),
                          static_cast<const uint64_t*>(dp(1)),
                          cap,
                          static_cast<int32_t*>(dp(2)),
                          static_cast<int64_t*>(dp(3)),
                          static_cast<int64_t*>(dp(4)),
                          static_cast<uint64_t*>(dp(5)),
                          static_cast<int32_t*>(dp(6)),
                          static_cast<uint8_t*>(dp(7)),
                          static_cast<int32_t*>(dp(8)),
                          static_cast<int32_t*>(dp(9))};
  if ((rc = attach_deep(c, &a, N, nbytes))) return rc;
  MDE_HIP(c, mde::launch_wire_decode(a, c->stream));
  auto down = [&](void* dst, int i) -> int {
    if (!dst) return MDE_OK;
    MDE_HIP(c, hipMemcpyAsync(dst, dp(i), sz[i], hipMemcpyDeviceToHost, c->stream));
    return MDE_OK;
  };
  if ((rc = down(partition, 2)) || (rc = down(lower, 3)) || (rc = down(upper, 4)) || (rc = down(digest, 5)) ||
      (rc = down(size, 6)) || (rc = down(valid, 7)) || (rc = down(items, 8)) || (rc = down(n_buckets, 9)))
    return rc;
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

uint32_t mde_verify_peer_capacity(uint32_t B) {
  if (!B) return 0;
  const uint32_t d = mde_tree_depth(B);
  return d >= 31 ? 0u : (1u << d);
}

namespace {

// Manager.VerifyEpoch, device pointers (see include/mde.h). Peer object (p, r) is
// peer_bytes[peer_off[p*R+r] .. peer_off[p*R+r+1]); an empty range is an absent peer (an empty
// object gives no tree, exactly like a missing one contributes nothing).
int verify_async(mde_ctx* c, uint32_t P, uint32_t B, const int32_t* partition, int64_t epoch,
                 const uint64_t* digest, const int32_t* size, const uint8_t* nodes, uint32_t R,
                 const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                 uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                 int32_t* peer_status, uint8_t* object_out, uint64_t object_stride, uint32_t* object_len) {
  if (!B || B > mde::kVerifyMaxBuckets || !digest || !valid || !valid_count || !diff_ids ||
      !diff_count || (R && (!peer_off || !peer_bytes)) || (object_out && (!size || !object_len)))
    return set_err(c, MDE_E_INVAL, "bad verify arguments");
  if (object_out && object_stride < mde::wire_max_bytes(B))
    return set_err(c, MDE_E_CAPACITY, "object_stride too small");
  if (!P) return MDE_OK;
  const uint64_t T = (uint64_t)P * R;
  const uint32_t cap = mde_verify_peer_capacity(B);
  if (!cap) return set_err(c, MDE_E_INVAL, "n_buckets too large");
  const uint64_t NI = mde::tree_internal(cap), idcap = mde_diff_capacity(B, cap);
  // scratch: digests, sizes, bucket counts, valid flags, nodes, roots, diff ids, statuses, the
  // partitions' valid flags (the encoder reads them; the caller's `valid` and `peer_status` are
  // stored once by the fold, so they may be pinned host memory); without local nodes
  // (nodes == NULL) also the local trees' nodes and roots, built where needed
  const uint64_t NL = mde::tree_internal(B);
  const uint64_t part[11] = {T * cap * 8, T * cap * 4, T * 4, T, T * NI * 32, T * 32, T * idcap * 4, T * 4,
                             nodes ? 0 : (uint64_t)P * NL * 32, nodes ? 0 : (uint64_t)P * 32, P};
  uint64_t off[12] = {0};
  for (int i = 0; i < 11; i++) off[i + 1] = off[i] + ((part[i] + 255) & ~255ull);
  int rc = ensure_buf(c, c->verify_scratch, off[11]);
  if (rc) return rc;
  uint8_t* base = static_cast<uint8_t*>(c->verify_scratch.p);
  auto at = [&](int i) { return static_cast<void*>(base + off[i]); };
  uint64_t* pd = static_cast<uint64_t*>(at(0));
  int32_t* nbk = static_cast<int32_t*>(at(2));
  uint8_t* pvalid = static_cast<uint8_t*>(at(3));
  uint8_t* pnodes = static_cast<uint8_t*>(at(4));
  int32_t* pids = static_cast<int32_t*>(at(6));
  int32_t* pst = static_cast<int32_t*>(at(7));
  uint8_t* const valid_user = valid;
  valid = static_cast<uint8_t*>(at(10));
  const bool build_local = !nodes;
  if (build_local) nodes = static_cast<const uint8_t*>(at(8));
  mde::TreeLaunch lt{};
  lt.P = build_local ? P : 0;
  lt.B = B;
  lt.digest_in = digest;
  lt.root_out = static_cast<uint8_t*>(at(9));
  lt.nodes_out = static_cast<uint8_t*>(at(8));
  lt.n_int = NL;
  if (mde::verify_fused_fits(R, cap) && !c->verify_chain) {
    // one launch: decode (LDS-staged) -> trees of other-shape peers -> diffs -> fold -> encode
    mde::VerifyFusedLaunch f{};
    f.dec = mde::WireDecodeLaunch{(uint32_t)T, peer_bytes, peer_off, cap, nullptr, nullptr, nullptr, pd,
                                  static_cast<int32_t*>(at(1)), pvalid, nullptr, nbk};
    if ((rc = attach_deep(c, &f.dec, 0, kDefaultDeepObjectBytes))) return rc;
    f.tree.B = cap;
    f.tree.digest_in = pd;
    f.tree.root_out = static_cast<uint8_t*>(at(5));
    f.tree.nodes_out = pnodes;
    f.tree.n_int = NI;
    f.diff = mde::DiffLaunch{(uint32_t)T, B, cap, digest, nodes, pd, pnodes, pids, idcap, pst, R, nbk};
    f.fold = mde::VerifyLaunch{P, R, B, pst, pids, idcap, pvalid, replica_count, valid, valid_count, diff_ids,
                               diff_count, valid_user, peer_status};
    if (object_out)
      f.enc = mde::WireEncodeLaunch{P, B, partition, epoch, epoch + 1, digest, size, valid, nullptr,
                                    object_out, object_stride, object_len};
    f.local = lt;
    MDE_HIP(c, mde::launch_verify_fused(f, c->stream));
    return MDE_OK;
  }
  if (T && build_local) MDE_HIP(c, mde::launch_tree(lt, c->stream));  // the chain diffs read every node
  if (T) {
    // EpochTreeObjectToMerkleTree: decode (>cap buckets can only diff with an error: deeper tree)
    mde::WireDecodeLaunch d{(uint32_t)T, peer_bytes, peer_off, cap, nullptr, nullptr, nullptr, pd,
                            static_cast<int32_t*>(at(1)), pvalid, nullptr, nbk};
    if ((rc = attach_deep(c, &d, 0, kDefaultDeepObjectBytes))) return rc;
    MDE_HIP(c, mde::launch_wire_decode(d, c->stream));
    mde::TreeLaunch t{};
    t.P = (uint32_t)T;
    t.B = cap;
    t.digest_in = pd;
    t.root_out = static_cast<uint8_t*>(at(5));
    t.nodes_out = pnodes;
    t.n_int = NI;
    t.n_in = nbk;
    MDE_HIP(c, mde::launch_tree(t, c->stream));
    // DifferentMerkleTreeBuckets(myTree, otherTree)
    mde::DiffLaunch df{(uint32_t)T, B, cap, digest, nodes, pd, pnodes, pids, idcap, pst, R, nbk};
    MDE_HIP(c, mde::launch_diff(df, c->stream));
  }
  mde::VerifyLaunch v{P, R, B, pst, pids, idcap, pvalid, replica_count, valid, valid_count, diff_ids, diff_count,
                      valid_user, peer_status};
  MDE_HIP(c, mde::launch_verify(v, c->stream));
  if (object_out) {
    // the object VerifyEpoch persists: MerkleTreeToPartitionEpochObject(myTree, p, E, E+1) with Valid
    mde::WireEncodeLaunch e{P, B, partition, epoch, epoch + 1, digest, size, valid, nullptr,
                            object_out, object_stride, object_len};
    MDE_HIP(c, mde::launch_wire_encode(e, c->stream));
  }
  return MDE_OK;
}

}  // namespace

int mde_verify_epochs_async(mde_ctx* c, uint32_t P, uint32_t B, const int32_t* partition, int64_t epoch,
                            const uint64_t* digest, const int32_t* size, const uint8_t* nodes, uint32_t R,
                            const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                            uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                            int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                            uint32_t* object_len) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  return verify_async(c, P, B, partition, epoch, digest, size, nodes, R, peer_bytes, peer_off, replica_count,
                      valid, valid_count, diff_ids, diff_count, peer_status, object_out, object_stride,
                      object_len);
}

int mde_verify_epochs(mde_ctx* c, uint32_t P, uint32_t B, const int32_t* partition, int64_t epoch,
                      const uint64_t* digest, const int32_t* size, const uint8_t* nodes, uint32_t R,
                      const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                      uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                      int32_t* peer_status, uint8_t* object_out, uint64_t object_stride, uint32_t* object_len) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!B || !digest || !valid || !valid_count || !diff_ids || !diff_count ||
      (R && P && !peer_off) || (object_out && (!size || !object_len)))
    return set_err(c, MDE_E_INVAL, "bad verify arguments");
  const uint64_t N = P, T = N * R, NI = mde::tree_internal(B);
  for (uint64_t i = 0; i < T; i++)
    if (peer_off[i] > peer_off[i + 1]) return set_err(c, MDE_E_INVAL, "peer_off not nondecreasing");
  const uint64_t nbytes = T ? peer_off[T] - peer_off[0] : 0;
  if (nbytes && !peer_bytes) return set_err(c, MDE_E_INVAL, "peer_bytes is NULL");
  const uint64_t ostride = object_out ? object_stride : 0;
  std::vector<uint64_t> rel(T + 1, 0);
  for (uint64_t i = 0; i <= T && T; i++) rel[i] = peer_off[i] - peer_off[0];
  HostIo io(c);
  const int i_part = io.in(partition, partition ? N * 4 : 0, N * 4);
  const int i_dig = io.in(digest, N * B * 8, N * B * 8);
  const int i_size = io.in(size, size ? N * B * 4 : 0, N * B * 4);
  const int i_nodes = io.in(nodes, nodes ? N * NI * 32 : 0, nodes ? N * NI * 32 : 0);
  const int i_peer = io.in(nbytes ? peer_bytes + peer_off[0] : nullptr, nbytes, nbytes + 1);
  const int i_rel = io.in(rel.data(), (T + 1) * 8, (T + 1) * 8);
  // every output is stored once (valid and the peer statuses are also kept in device scratch for
  // the fold and the encode to read back)
  const int o_valid = io.out(valid, N, true), o_vc = io.out(valid_count, N * 4, true),
            o_ids = io.out(diff_ids, N * B * 4, true);
  const int o_dc = io.out(diff_count, N * 4, true), o_ps = io.out(T ? peer_status : nullptr, T * 4, true);
  const int o_obj = io.out(object_out, N * ostride, true),
            o_olen = io.out(object_out ? object_len : nullptr, N * 4, true);
  int rc = io.upload();
  if (rc) return rc;
  // the spill area covers every object of this call (no rescans, whatever they nest)
  rc = ensure_buf(c, c->deep_scratch, std::max(mde::wire_deep_entries(T, nbytes) * 4, c->deep_scratch.cap));
  if (rc) return rc;
  rc = verify_async(c, P, B, partition ? static_cast<const int32_t*>(io.dev(i_part)) : nullptr, epoch,
                    static_cast<const uint64_t*>(io.dev(i_dig)),
                    size ? static_cast<const int32_t*>(io.dev(i_size)) : nullptr,
                    nodes ? static_cast<const uint8_t*>(io.dev(i_nodes)) : nullptr, R,
                    static_cast<const uint8_t*>(io.dev(i_peer)),
                    static_cast<const uint64_t*>(io.dev(i_rel)), replica_count,
                    static_cast<uint8_t*>(io.dev(o_valid)), static_cast<int32_t*>(io.dev(o_vc)),
                    static_cast<int32_t*>(io.dev(o_ids)), static_cast<int32_t*>(io.dev(o_dc)),
                    static_cast<int32_t*>(io.dev(o_ps)),
                    object_out ? static_cast<uint8_t*>(io.dev(o_obj)) : nullptr, ostride,
                    object_out ? static_cast<uint32_t*>(io.dev(o_olen)) : nullptr);
  if (rc) return rc;
  return io.download();
}

int mde_tag_keys_async(mde_ctx* c, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                       uint32_t B, uint32_t P, uint32_t* bucket, uint32_t* partition) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if ((bucket && !B) || (partition && !P) || (n && (!keys || !key_off)))
    return set_err(c, MDE_E_INVAL, "bad tag_keys arguments");
  MDE_HIP(c, mde::launch_tag_keys(keys, key_off, n, B, P, bucket, partition, c->stream));
  return MDE_OK;
}

int mde_tag_keys(mde_ctx* c, const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t B,
                 uint32_t P, uint32_t* bucket, uint32_t* partition) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  SyncOnReturn drain{c->stream};  // every return waits for the copies this call issued
  if ((bucket && !B) || (partition && !P) || (n && (!keys || !key_off)))
    return set_err(c, MDE_E_INVAL, "bad tag_keys arguments");
  if (n == 0) return MDE_OK;
  const uint64_t kb = key_off[n];
  const uint64_t sz[4] = {kb, (n + 1) * 8, n * 4, n * 4};
  int rc;
  for (int i = 0; i < 4; i++)
    if ((rc = ensure_buf(c, c->stage[i], sz[i]))) return rc;
  if (kb) MDE_HIP(c, hipMemcpyAsync(c->stage[0].p, keys, kb, hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipMemcpyAsync(c->stage[1].p, key_off, sz[1], hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, mde::launch_tag_keys(static_cast<const uint8_t*>(c->stage[0].p),
                                  static_cast<const uint64_t*>(c->stage[1].p), n, B, P,
                                  bucket ? static_cast<uint32_t*>(c->stage[2].p) : nullptr,
                                  partition ? static_cast<uint32_t*>(c->stage[3].p) : nullptr,
                                  c->stream));
  if (bucket) MDE_HIP(c, hipMemcpyAsync(bucket, c->stage[2].p, sz[2], hipMemcpyDeviceToHost, c->stream));
  if (partition) MDE_HIP(c, hipMemcpyAsync(partition, c->stage[3].p, sz[3], hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_synth_tags_async(mde_ctx* c, const uint64_t* gids, uint64_t n, uint32_t P, uint32_t B,
                         int mode, uint64_t kpp, uint32_t* part, uint32_t* bucket) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!B || !P || mode < 0 || mode > 2 || (mode == 0 && !kpp) || (n && (!gids || !part || !bucket)))
    return set_err(c, MDE_E_INVAL, "bad synth_tags arguments");
  MDE_HIP(c, mde::launch_synth_tags(gids, n, P, B, mode, kpp, part, bucket, c->stream));
  return MDE_OK;
}

int mde_synth_values_async(mde_ctx* c, uint8_t* dst, const uint64_t* gids, uint64_t n,
                           uint32_t len, uint64_t seed) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (n && len && (!dst || !gids)) return set_err(c, MDE_E_INVAL, "bad synth_values arguments");
  MDE_HIP(c, mde::launch_synth_values(dst, gids, n, len, seed, c->stream));
  return MDE_OK;
}

int mde_dev_alloc(mde_ctx* c, uint64_t bytes, void** p) {
  if (!c || !p) return MDE_E_INVAL;
  Guard g(c);
  if (hipMalloc(p, bytes ? bytes : 1) != hipSuccess) {
    *p = nullptr;
    return set_err(c, MDE_E_NOMEM, "hipMalloc(%llu) failed", (unsigned long long)bytes);
  }
  return MDE_OK;
}

int mde_dev_free(mde_ctx* c, void* p) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (p) {
    MDE_HIP(c, hipStreamSynchronize(c->stream));
    MDE_HIP(c, hipFree(p));
  }
  return MDE_OK;
}

int mde_memcpy_h2d(mde_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!bytes) return MDE_OK;
  MDE_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

int mde_memcpy_d2h(mde_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return MDE_E_INVAL;
  Guard g(c);
  if (!bytes) return MDE_OK;
  MDE_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  MDE_HIP(c, hipStreamSynchronize(c->stream));
  return MDE_OK;
}

}  // extern "C"

// Device groups (mde_group_*, mde_multi_build*): group.cpp.
