// verify.hip -- the decision step of Manager.VerifyEpoch, batched over partitions.
//
// Reference (main/manager.go:1072-1118): for each peer EpochTreeObject, rebuild its tree and diff
// it against this node's tree; a peer whose object or diff fails is skipped (logrus.Error +
// continue); every successful diff is merged into diffSet (utils.Int32Set); an empty diff counts
// toward validCount, a non-empty diff against a peer object marked Valid sets validDiff. The
// epoch object is valid iff validCount >= ReplicaCount or validDiff; otherwise the node requests
// diffSet.List() from its peers (PoliteStreamRequest).
//
// One 256-thread workgroup per partition: the diff ids of its R peers are OR-ed into an LDS
// bitmap of B bits (the Int32Set), then compacted in ascending order with a block prefix sum over
// the bitmap words. Go's map iteration order is unspecified; ascending is the canonical order.
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {
namespace {

constexpr int kThreads = 256;
constexpr uint32_t kWords = kVerifyMaxBuckets / 32;

__global__ __launch_bounds__(kThreads) void verify_kernel(VerifyLaunch a) {
  __shared__ uint32_t bits[kWords];
  __shared__ uint32_t wave_tot[kThreads / 64];
  const uint32_t p = blockIdx.x, t = threadIdx.x;
  const uint32_t W = (a.B + 31) / 32;
  for (uint32_t w = t; w < W; w += kThreads) bits[w] = 0;
  __syncthreads();
  int32_t valid_count = 0;
  bool valid_diff = false;
  for (uint32_t r = 0; r < a.R; r++) {
    const uint64_t i = (uint64_t)p * a.R + r;
    const int32_t n = a.peer_status[i];
    if (n < 0) continue;  // EpochTreeObjectToMerkleTree / DifferentMerkleTreeBuckets error
    if (n == 0) {
      valid_count++;
    } else if (a.peer_valid[i]) {
      valid_diff = true;
    }
    const int32_t* ids = a.peer_ids + i * a.ids_stride;
    for (uint32_t j = t; j < (uint32_t)n; j += kThreads) {
      const uint32_t id = (uint32_t)ids[j];
      if (id < a.B) atomicOr(&bits[id >> 5], 1u << (id & 31));
    }
  }
  __syncthreads();
  // Ascending compaction: thread t owns words [t*per, (t+1)*per).
  const uint32_t per = (W + kThreads - 1) / kThreads;
  const uint32_t w0 = min(t * per, W), w1 = min(w0 + per, W);
  uint32_t mine = 0;
  for (uint32_t w = w0; w < w1; w++) mine += __popc(bits[w]);
  const int lane = t & 63, wid = t >> 6;
  uint32_t incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o);
    if (lane >= o) incl += x;
  }
  if (lane == 63) wave_tot[wid] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < kThreads / 64; w++) {
    base += w < wid ? wave_tot[w] : 0u;
    total += wave_tot[w];
  }
  uint32_t pos = base + incl - mine;
  int32_t* out = a.diff_ids + (uint64_t)p * a.B;
  for (uint32_t w = w0; w < w1; w++) {
    uint32_t m = bits[w];
    while (m) {
      const uint32_t b = __ffs(m) - 1;
      m &= m - 1;
      out[pos++] = (int32_t)(w * 32 + b);
    }
  }
  if (t == 0) {
    a.diff_count[p] = (int32_t)total;
    a.valid_count[p] = valid_count;
    a.valid[p] = (valid_count >= (int32_t)a.replica_count || valid_diff) ? 1 : 0;
  }
}

}  // namespace

hipError_t launch_verify(const VerifyLaunch& a, hipStream_t st) {
  if (a.P == 0) return hipSuccess;
  if (a.B == 0 || a.B > kVerifyMaxBuckets) return hipErrorInvalidValue;
  hipLaunchKernelGGL(verify_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace mde
