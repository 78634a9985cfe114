// shaprobe.hip -- SHA-256 compression latency / throughput probe for the tree kernels (not
// product code). Times the engine's own sha256_node_pair (mde_device.hpp) in dependent chains:
//   * one wave alone on the chip: shader cycles and wall time per node hash (the latency that
//     bounds a tree's critical path);
//   * W waves per SIMD on every SIMD, each lane an independent chain: node hashes per second
//     for the whole chip (the throughput that bounds a build's tree work).
//   hipcc -O3 --offload-arch=gfx950 -I include -I mydatastore_amd/csrc tools/shaprobe.hip -o tools/shaprobe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "mde_device.hpp"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

using namespace mde;

__global__ __launch_bounds__(256) void chain(uint32_t k, uint32_t active, uint32_t* out, unsigned long long* cyc) {
  uint32_t h[8], r[8];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; i++) { h[i] = t * 2654435761u + i; r[i] = ~h[i]; }
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  if ((threadIdx.x & 63) < active) {
    for (uint32_t j = 0; j < k; j++) {
      uint32_t st[8];
      sha256_node_pair(h, r, st);
#pragma unroll
      for (int i = 0; i < 8; i++) { r[i] = h[i]; h[i] = st[i]; }
    }
  }
  const uint64_t c1 = clock64(), w1 = wall_clock64();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x ^= h[i];
  out[t] = x;
  if (t == 0) { cyc[0] = c1 - c0; cyc[1] = w1 - w0; }
}

int main(int argc, char** argv) {
  const uint32_t k = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int wall_khz = 0;
  CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  uint32_t* out;
  unsigned long long* cyc;
  CK(hipMalloc(&out, (size_t)cus * 256 * 16 * 4));
  CK(hipMalloc(&cyc, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // one wave alone: lanes active 64 and 1 (an upper tree level's single node)
  for (uint32_t active : {64u, 1u}) {
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, k, active, out, cyc);
      CK(hipDeviceSynchronize());
    }
    unsigned long long h[2];
    CK(hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost));
    printf("{\"mode\": \"one_wave\", \"active_lanes\": %u, \"node_hashes\": %u, \"cycles_per_node\": %.1f, "
           "\"ns_per_node\": %.1f}\n",
           active, k, (double)h[0] / k, (double)h[1] * 1e6 / wall_khz / k);
  }
  // every SIMD: W waves each (256-thread workgroups, W per CU... W x cus workgroups)
  for (uint32_t W : {1u, 2u, 4u, 8u}) {
    const uint32_t blocks = (uint32_t)cus * W;
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(chain, dim3(blocks), dim3(256), 0, 0, k, 64u, out, cyc);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double nodes = (double)blocks * 256 * k;
    printf("{\"mode\": \"all_simds\", \"waves_per_simd\": %u, \"node_hashes\": %.0f, \"ms\": %.3f, "
           "\"node_hashes_per_us\": %.0f, \"us_per_node_per_wave\": %.3f}\n",
           W, nodes, best, nodes / (best * 1e3), best * 1e3 / k);
  }
  return 0;
}
