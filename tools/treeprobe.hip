// treeprobe.hip -- workgroup shapes for the standalone tree kernel (not product code).
// Times tree_body (tree_body.hpp, the product's builder) from digests under several launch
// shapes -- partitions per wave (G) and threads per workgroup -- at B = 64 and 1,000 for 1,024 and
// 128 partitions (or a B x P sweep), and checks that every shape's roots and nodes equal the
// product geometry's. Two more probes ran on a modified tree_body and were dropped (no change,
// profiles/r02ad_treeprobe*.jsonl): rotating the narrow upper levels over the workgroup's waves,
// and barriers that order LDS only (no wait for the global node stores).
//   hipcc -O3 --offload-arch=gfx950 -I include -I mydatastore_amd/csrc tools/treeprobe.hip -o tools/treeprobe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "tree_body.hpp"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

using namespace mde;

__global__ __launch_bounds__(256) void probe_tree(TreeLaunch a, uint32_t G, uint32_t words, uint32_t threads,
                                                  uint32_t rotate) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  (void)rotate;
  tree_body<true>(a, G, words, blockIdx.x, lds, threads);
}

namespace mde {
uint64_t tree_internal_host(uint32_t B) {
  uint32_t n = B + (B & 1u);
  uint64_t t = 0;
  while (n > 1) {
    n = (n + 1) / 2;
    t += n;
  }
  return t;
}
}  // namespace mde

struct Shape {
  const char* name;
  uint32_t G, threads, rotate;
};

// treeprobe            -- every shape at B = 64 / 1,000, P = 1,024 / 128
// treeprobe sweep      -- product vs 128- and 64-thread groups over B and P
int main(int argc, char** argv) {
  const bool wide = !(argc > 1 && strcmp(argv[1], "sweep") == 0);
  std::vector<uint32_t> Bs = wide ? std::vector<uint32_t>{64u, 1000u} : std::vector<uint32_t>{200u, 500u, 1000u, 2000u, 4096u};
  std::vector<uint32_t> Ps = wide ? std::vector<uint32_t>{1024u, 128u} : std::vector<uint32_t>{64u, 128u, 256u, 512u, 1024u, 4096u};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint32_t B : Bs) {
    const uint32_t n1 = (B + 1) / 2;
    uint32_t Gp = 8;
    while (Gp < n1 && Gp < 256) Gp <<= 1;
    const uint32_t Tp = n1 > 64 ? 256 : 64;
    std::vector<Shape> shapes = {{"product", n1 > 64 ? 256u : Gp, Tp, 0}};
    if (wide) {
      if (n1 > 64) {
        shapes.push_back({"g128_t128", 128, 128, 0});
        shapes.push_back({"g128_t256", 128, 256, 0});
        shapes.push_back({"g64_t64", 64, 64, 0});
        shapes.push_back({"g64_t256", 64, 256, 0});
      } else {
        shapes.push_back({"g32_t128", Gp, 128, 0});
        shapes.push_back({"g32_t256", Gp, 256, 0});
        shapes.push_back({"g64_t64", 64, 64, 0});
        shapes.push_back({"g64_t256", 64, 256, 0});
      }
    } else if (n1 > 64) {
      shapes.push_back({"g128_t128", 128, 128, 0});
      if (n1 <= 1024) shapes.push_back({"g64_t64", 64, 64, 0});
    }
    for (uint32_t P : Ps) {
      const uint64_t nint = tree_internal_host(B);
      std::vector<uint64_t> h((size_t)P * B);
      uint64_t x = 88172645463325252ull ^ (B * 131 + P);
      for (auto& v : h) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = x % 999999;
      }
      uint64_t* d;
      uint8_t *root, *nodes;
      CK(hipMalloc(&d, h.size() * 8));
      CK(hipMalloc(&root, (size_t)P * 32));
      CK(hipMalloc(&nodes, (size_t)P * nint * 32));
      CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
      std::vector<uint8_t> ref_root, ref_nodes;
      for (const Shape& s : shapes) {
        TreeLaunch a{};
        a.P = P;
        a.B = B;
        a.digest_in = d;
        a.root_out = root;
        a.nodes_out = nodes;
        a.n_int = nint;
        const uint32_t words = 4 + (n1 + (n1 + 1) / 2) * 8;
        const uint32_t groups = s.threads / s.G;
        const size_t lds = (size_t)words * 4 * groups;
        const uint32_t blocks = (P + groups - 1) / groups;
        float best = 1e30f, sum = 0;
        const int reps = wide ? 20 : 8;
        for (int r = -2; r < reps; r++) {
          CK(hipMemset(root, 0, (size_t)P * 32));
          CK(hipEventRecord(e0, 0));
          hipLaunchKernelGGL(probe_tree, dim3(blocks), dim3(s.threads), lds, 0, a, s.G, words, s.threads, s.rotate);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (r >= 0) {
            sum += ms;
            if (ms < best) best = ms;
          }
        }
        std::vector<uint8_t> rr((size_t)P * 32), nn((size_t)P * nint * 32);
        CK(hipMemcpy(rr.data(), root, rr.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(nn.data(), nodes, nn.size(), hipMemcpyDeviceToHost));
        bool same = true;
        if (ref_root.empty()) {
          ref_root = rr;
          ref_nodes = nn;
        } else {
          same = rr == ref_root && nn == ref_nodes;
        }
        printf("{\"B\": %u, \"P\": %u, \"shape\": \"%s\", \"G\": %u, \"threads\": %u, \"rotate\": %u, "
               "\"us_min\": %.2f, \"us_mean\": %.2f, \"same_as_product\": %s}\n",
               B, P, s.name, s.G, s.threads, s.rotate, best * 1e3, sum / reps * 1e3, same ? "true" : "false");
        fflush(stdout);
      }
      CK(hipFree(d));
      CK(hipFree(root));
      CK(hipFree(nodes));
    }
  }
  return 0;
}
