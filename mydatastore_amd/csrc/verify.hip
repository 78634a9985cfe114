// verify.hip -- the decision step of Manager.VerifyEpoch, batched over partitions.
//
// Reference (main/manager.go:1072-1118): for each peer EpochTreeObject, rebuild its tree and diff
// it against this node's tree; a peer whose object or diff fails is skipped (logrus.Error +
// continue); every successful diff is merged into diffSet (utils.Int32Set); an empty diff counts
// toward validCount, a non-empty diff against a peer object marked Valid sets validDiff. The
// epoch object is valid iff validCount >= ReplicaCount or validDiff; otherwise the node requests
// diffSet.List() from its peers (PoliteStreamRequest).
//
// Fold (verify_body): one 256-thread workgroup per partition; the diff ids of its R peers are
// OR-ed into an LDS bitmap of B bits (the Int32Set), then compacted in ascending order with a
// block prefix sum over the bitmap words. Go's map iteration order is unspecified; ascending is
// the canonical order.
//
// Two launch shapes:
//   * verify_kernel: the fold alone, after the decode / tree / diff kernels of the chain
//     (mde_api.cpp verify_async) -- any R and B;
//   * verify_fused_kernel: the whole step in one launch per call. A one-partition VerifyEpoch
//     spent ~93 us in the chain on the device, 52 us of it in the decoder's lane-0 byte walk over
//     global memory (one dependent load per varint byte) and 28 us rebuilding the peer trees (11
//     dependent SHA-256 compressions). Here each wave stages one peer object into LDS with wide
//     loads and parses it there with all 64 lanes (wire_body.hpp), and a peer tree is rebuilt
//     only when its shape differs from the local tree's: same-shape peers diff on the leaf
//     digests alone (diff_body<true>).
#include "verify_body.hpp"

namespace mde {
namespace {

constexpr int kThreads = kVerifyThreads;

__global__ __launch_bounds__(kThreads) void verify_kernel(VerifyLaunch a) {
  __shared__ uint32_t bits[kVerifyWords];
  __shared__ uint32_t wave_tot[kThreads / 64];
  verify_body(a, blockIdx.x, bits, wave_tot);
}

template <bool kDeep>
__global__ __launch_bounds__(kThreads) void verify_fused_kernel(VerifyFusedLaunch f, uint32_t G, uint32_t words,
                                                                uint32_t stage_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ VerifyShared sh;
  verify_fused_body<kDeep>(f, blockIdx.x, G, words, stage_bytes, dyn, sh);
}

}  // namespace

hipError_t launch_verify(const VerifyLaunch& a, hipStream_t st) {
  if (a.P == 0) return hipSuccess;
  if (a.B == 0 || a.B > kVerifyMaxBuckets) return hipErrorInvalidValue;
  hipLaunchKernelGGL(verify_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

bool verify_fused_fits(uint32_t R, uint32_t cap) {
  return R <= kVerifyFusedMaxPeers && cap >= 1 && cap <= kVerifyFusedMaxCap;
}

hipError_t launch_verify_fused(const VerifyFusedLaunch& a, hipStream_t st) {
  const uint32_t P = a.fold.P, cap = a.dec.cap;
  if (P == 0) return hipSuccess;
  if (!verify_fused_fits(a.fold.R, cap) || a.fold.B == 0 || a.fold.B > cap) return hipErrorInvalidValue;
  uint32_t G, words, stage;
  const size_t lds = verify_fused_lds(cap, &G, &words, &stage);
  if (a.fold.B > 64)
    hipLaunchKernelGGL(verify_fused_kernel<true>, dim3(P), dim3(kThreads), lds, st, a, G, words, stage);
  else
    hipLaunchKernelGGL(verify_fused_kernel<false>, dim3(P), dim3(kThreads), lds, st, a, G, words, stage);
  return hipGetLastError();
}

size_t verify_fused_lds(uint32_t cap, uint32_t* G, uint32_t* words, uint32_t* stage_bytes) {
  TreeGeometry g;
  tree_geometry(cap, &g);
  const uint32_t tree_bytes = g.words * 4u * ((uint32_t)kThreads / g.G);
  uint64_t stage = (wire_max_bytes(cap) + 4 + 15) / 16 * 16;
  if (stage > kVerifyStageMaxBytes) stage = kVerifyStageMaxBytes;
  const uint64_t stage_all = stage * (kThreads / 64);
  *G = g.G;
  *words = g.words;
  *stage_bytes = (uint32_t)stage;
  return tree_bytes > stage_all ? tree_bytes : stage_all;
}

}  // namespace mde
