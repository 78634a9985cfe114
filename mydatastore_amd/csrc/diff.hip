// diff.hip -- DifferentMerkleTreeBuckets on device, one workgroup per tree pair.
//
// The per-pair DFS (reference semantics, path enumeration) is diff_body() in diff_body.hpp, shared
// with the fused verify kernel (verify.hip).
#include "diff_body.hpp"

namespace mde {
namespace {

__global__ __launch_bounds__(kDiffThreads) void diff_kernel(DiffLaunch a) {
  __shared__ DiffLds s;
  diff_body<false>(a, blockIdx.x, s);
}

}  // namespace

hipError_t launch_diff(const DiffLaunch& a, hipStream_t st) {
  if (a.n_pairs == 0) return hipSuccess;
  hipLaunchKernelGGL(diff_kernel, dim3(a.n_pairs), dim3(kDiffThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace mde
