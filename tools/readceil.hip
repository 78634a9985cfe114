// readceil.hip -- HBM read-ceiling probe for the digest kernel's roofline (not product code).
//
// Streams a 10.24 GB buffer (the C4 arena size) with the same per-lane work as
// bucket_digest_kernel's fast path (16-B loads, one v_sad_u8 per dword, one atomic per wave) but
// none of its bucket bookkeeping, under several access shapes, to measure what a read-only stream
// achieves on this chip. The digest kernel's roofline.frac is quoted against the 8 TB/s spec; this
// gives the measured ceiling beside it.
//
//   hipcc -O3 --offload-arch=gfx950 tools/readceil.hip -o tools/readceil && tools/readceil
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// Contiguous range per wave (the digest kernel's shape). U 16-B loads per lane per step.
template <int U, bool NT, bool PIPE>
__global__ __launch_bounds__(256) void read_contig(const u32x4* __restrict__ buf, uint64_t n16,
                                                   uint64_t per_wave16, unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t beg = wave * per_wave16, end = std::min(beg + per_wave16, n16);
  uint32_t acc = 0;
  constexpr uint64_t kStep = 64ull * U;
  u32x4 cur[U];
  if (PIPE && beg < end) {
#pragma unroll
    for (int u = 0; u < U; u++) cur[u] = NT ? __builtin_nontemporal_load(buf + beg + u * 64 + lane) : buf[beg + u * 64 + lane];
  }
  for (uint64_t p = beg; p + kStep <= end; p += kStep) {
    u32x4 v[U];
    if (PIPE) {
      u32x4 nx[U];
      if (p + 2 * kStep <= end) {
#pragma unroll
        for (int u = 0; u < U; u++)
          nx[u] = NT ? __builtin_nontemporal_load(buf + p + kStep + u * 64 + lane) : buf[p + kStep + u * 64 + lane];
      }
#pragma unroll
      for (int u = 0; u < U; u++) { v[u] = cur[u]; cur[u] = nx[u]; }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(buf + p + u * 64 + lane) : buf[p + u * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
    }
  }
  unsigned long long s = acc;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) atomicAdd(out, s);
}

// Grid-stride: consecutive waves read consecutive KiB (all waves sweep the buffer together).
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_stride(const u32x4* __restrict__ buf, uint64_t n16,
                                                   unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (uint64_t p = wave * 64 * U; p + 64 * U <= n16; p += nw * 64 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(buf + p + u * 64 + lane) : buf[p + u * 64 + lane];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
    }
  }
  unsigned long long s = acc;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) atomicAdd(out, s);
}

// Contiguous range per WORKGROUP: its W waves interleave at U KiB granularity (wave w takes steps
// w, w+W, ...), so the workgroup sweeps one region front to back with W*U KiB in flight -- W times
// fewer concurrent streams than read_contig at the same wave count.
template <int U, int W>
__global__ __launch_bounds__(64 * W) void read_wgcontig(const u32x4* __restrict__ buf, uint64_t n16,
                                                       uint64_t per_wg16, unsigned long long* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t beg = (uint64_t)blockIdx.x * per_wg16, end = std::min(beg + per_wg16, n16);
  uint32_t acc = 0;
  constexpr uint64_t kStep = 64ull * U;
  for (uint64_t p = beg + wid * kStep; p + kStep <= end; p += W * kStep) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(buf + p + u * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
      acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
    }
  }
  unsigned long long s = acc;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) atomicAdd(out, s);
}

// Chunked grid-stride: the buffer is cut into chunks of C16 16-B vectors; wave w streams chunks
// w, w + nw, w + 2nw, ... front to back (U KiB steps, next step's loads issued before the current
// step is reduced). All waves sweep the buffer together in a window of nw * C bytes, as the
// grid-stride shape does, while each wave still reads C contiguous bytes at a time.
template <int U>
__global__ __launch_bounds__(256) void read_chunk(const u32x4* __restrict__ buf, uint64_t n16, uint64_t c16,
                                                  unsigned long long* out) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  constexpr uint64_t kStep = 64ull * U;
  const uint64_t nchunks = (n16 + c16 - 1) / c16;
  uint32_t acc = 0;
  for (uint64_t c = wave; c < nchunks; c += nw) {
    const uint64_t beg = c * c16, end = std::min(beg + c16, n16) / kStep * kStep;
    if (beg >= end) break;
    u32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; u++) cur[u] = __builtin_nontemporal_load(buf + beg + u * 64 + lane);
    for (uint64_t p = beg; p < end; p += kStep) {
      u32x4 v[U], nx[U];
      if (p + kStep < end) {
#pragma unroll
        for (int u = 0; u < U; u++) nx[u] = __builtin_nontemporal_load(buf + p + kStep + u * 64 + lane);
      }
#pragma unroll
      for (int u = 0; u < U; u++) { v[u] = cur[u]; cur[u] = nx[u]; }
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
      }
    }
  }
  unsigned long long s = acc;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) atomicAdd(out, s);
}

// Contiguous range per wave through buffer loads with cache-policy bits AUX (gfx950: 1 = sc0,
// 2 = nt, 16 = sc1): one descriptor per wave based at its range (ranges < 4 GiB).
template <int AUX>
__global__ __launch_bounds__(256) void read_buf(const u32x4* __restrict__ buf, uint64_t n16, uint64_t per_wave16,
                                                unsigned long long* out) {
  constexpr int U = 4;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t beg = wave * per_wave16, end = std::min(beg + per_wave16, n16);
  uint32_t acc = 0;
  if (beg < end) {
    const uint32_t nbytes = (uint32_t)((end - beg) * 16);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(buf + beg), (short)0, (int)nbytes, 0x00020000);
    const uint32_t steps = (uint32_t)((end - beg) / (64 * U));
    u32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      cur[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (u * 64 + lane) * 16, 0, AUX));
    for (uint32_t t = 0; t < steps; t++) {
      u32x4 v[U], nx[U];
      if (t + 1 < steps) {
#pragma unroll
        for (int u = 0; u < U; u++)
          nx[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((t + 1) * 64 * U + u * 64 + lane) * 16, 0, AUX));
      }
#pragma unroll
      for (int u = 0; u < U; u++) { v[u] = cur[u]; cur[u] = nx[u]; }
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
      }
    }
  }
  unsigned long long s = acc;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) atomicAdd(out, s);
}

__global__ void fill(uint32_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u);
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 10240000000ull;
  const uint64_t n16 = bytes / 16;
  u32x4* buf;
  unsigned long long* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 8));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint32_t*)buf, bytes / 4);
  CK(hipDeviceSynchronize());
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));

  auto time_it = [&](auto launch) {
    for (int i = 0; i < 2; i++) launch();
    std::vector<float> ms;
    for (int r = 0; r < 10; r++) {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float t;
      CK(hipEventElapsedTime(&t, a, b));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
  };
  if (argc > 2 && std::string(argv[2]) == "cumask") {
    // Streaming on a subset of the CUs (hipExtStreamCreateWithCUMask): is HBM still saturated
    // when a few CUs are set aside? off CUs masked, either the last ones or one per 32.
    for (int spread = 0; spread < 2; spread++)
      for (int off : {0, 8, 16, 32}) {
        std::vector<uint32_t> mask((cus + 31) / 32, 0u);
        int on = 0;
        for (int c = 0; c < cus; c++) {
          const bool masked = spread ? (off && (c % (cus / off)) == (cus / off) - 1) : c >= cus - off;
          if (!masked) { mask[c / 32] |= 1u << (c % 32); on++; }
        }
        hipStream_t st;
        CK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
        for (int wpc : {2, 3}) {
          const uint64_t waves = (uint64_t)on * wpc * 4;
          uint64_t per = (n16 + waves - 1) / waves;
          per = (per + 255) / 256 * 256;
          const uint32_t blocks = (uint32_t)((n16 + per * 4 - 1) / (per * 4));
          std::vector<float> ms;
          for (int r = 0; r < 12; r++) {
            CK(hipEventRecord(a, st));
            hipLaunchKernelGGL((read_contig<4, true, true>), dim3(blocks), dim3(256), 0, st, buf, n16, per, out);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            if (r >= 2) ms.push_back(t);
          }
          std::sort(ms.begin(), ms.end());
          const float m = ms[ms.size() / 2];
          printf("{\"shape\": \"contig U4 nt pipe, CU mask\", \"cus_on\": %d, \"spread\": %d, \"wg_per_cu\": %d, "
                 "\"ms\": %.4f, \"GBps\": %.1f}\n", on, spread, wpc, m, bytes / (m * 1e-3) / 1e9);
          fflush(stdout);
        }
        CK(hipStreamDestroy(st));
      }
    return 0;
  }
  auto report = [&](const char* name, int wg_per_cu, float ms) {
    printf("{\"shape\": \"%s\", \"wg_per_cu\": %d, \"bytes\": %llu, \"ms\": %.4f, \"GBps\": %.1f}\n", name,
           wg_per_cu, (unsigned long long)bytes, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  if (argc > 2 && std::string(argv[2]) == "policy") {
    // cache-policy bits of the streaming loads: buffer loads with aux = sc0 / nt / sc1 combos
    for (int wpc : {1, 2}) {
      const uint64_t waves = (uint64_t)cus * wpc * 4;
      uint64_t per = (n16 + waves - 1) / waves;
      per = (per + 255) / 256 * 256;
      const uint32_t blocks = (uint32_t)((n16 + per * 4 - 1) / (per * 4));
      report("contig U4 nt pipe (global)", wpc, time_it([&] {
               hipLaunchKernelGGL((read_contig<4, true, true>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
             }));
#define RB(AUX)                                                                                         \
  report("buffer U4 pipe aux " #AUX, wpc, time_it([&] {                                                 \
           hipLaunchKernelGGL((read_buf<AUX>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);     \
         }));
      RB(0) RB(1) RB(2) RB(3) RB(16) RB(17) RB(18) RB(19)
#undef RB
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "chunk") {
    // chunked grid-stride vs the two end points (contiguous range per wave, plain grid-stride);
    // chunk sizes divide the byte count only approximately: the reported rate uses the bytes read
    for (int wpc : {1, 2, 3}) {
      const uint64_t waves = (uint64_t)cus * wpc * 4;
      uint64_t per = (n16 + waves - 1) / waves;
      per = (per + 255) / 256 * 256;
      const uint32_t blocks = (uint32_t)((n16 + per * 4 - 1) / (per * 4));
      report("contig U4 nt pipe", wpc, time_it([&] {
               hipLaunchKernelGGL((read_contig<4, true, true>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
             }));
      report("stride U4 nt", wpc, time_it([&] {
               hipLaunchKernelGGL((read_stride<4, true>), dim3(cus * wpc), dim3(256), 0, 0, buf, n16, out);
             }));
      // k pieces per wave: the wave's share cut into k chunks placed k grid-strides apart
      for (uint64_t k : {2ull, 4ull, 16ull, 64ull, 256ull}) {
        uint64_t c16 = (n16 + waves * k - 1) / (waves * k);
        c16 = (c16 + 255) / 256 * 256;
        const float ms = time_it([&] {
          hipLaunchKernelGGL((read_chunk<4>), dim3(cus * wpc), dim3(256), 0, 0, buf, n16, c16, out);
        });
        printf("{\"shape\": \"chunk k%llu (%llu KiB) U4 nt pipe\", \"wg_per_cu\": %d, \"bytes\": %llu, "
               "\"ms\": %.4f, \"GBps\": %.1f}\n", (unsigned long long)k, (unsigned long long)(c16 / 64), wpc,
               (unsigned long long)bytes, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
      }
    }
    return 0;
  }

  for (int wpc : {1, 2, 3, 4, 8}) {
    const uint64_t waves = (uint64_t)cus * wpc * 4;
    uint64_t per = (n16 + waves - 1) / waves;
    per = (per + 255) / 256 * 256;
    const uint32_t blocks = (uint32_t)((n16 + per * 4 - 1) / (per * 4));
    report("contig U4 nt pipe", wpc, time_it([&] {
             hipLaunchKernelGGL((read_contig<4, true, true>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
           }));
    report("contig U8 nt", wpc, time_it([&] {
             hipLaunchKernelGGL((read_contig<8, true, false>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
           }));
    report("contig U8 default", wpc, time_it([&] {
             hipLaunchKernelGGL((read_contig<8, false, false>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
           }));
    report("contig U16 nt", wpc, time_it([&] {
             hipLaunchKernelGGL((read_contig<16, true, false>), dim3(blocks), dim3(256), 0, 0, buf, n16, per, out);
           }));
    report("stride U4 nt", wpc, time_it([&] {
             hipLaunchKernelGGL((read_stride<4, true>), dim3(cus * wpc), dim3(256), 0, 0, buf, n16, out);
           }));
    report("stride U8 default", wpc, time_it([&] {
             hipLaunchKernelGGL((read_stride<8, false>), dim3(cus * wpc), dim3(256), 0, 0, buf, n16, out);
           }));
    {  // one stream per 4-wave / 8-wave workgroup (wpc = 4-wave workgroups per CU, as above)
      const uint64_t per4 = ((n16 + (uint64_t)cus * wpc - 1) / ((uint64_t)cus * wpc) + 255) / 256 * 256;
      const uint32_t b4 = (uint32_t)((n16 + per4 - 1) / per4);
      report("wgcontig W4 U4 nt", wpc, time_it([&] {
               hipLaunchKernelGGL((read_wgcontig<4, 4>), dim3(b4), dim3(256), 0, 0, buf, n16, per4, out);
             }));
      report("wgcontig W4 U8 nt", wpc, time_it([&] {
               hipLaunchKernelGGL((read_wgcontig<8, 4>), dim3(b4), dim3(256), 0, 0, buf, n16, per4, out);
             }));
      if (wpc % 2 == 0) {
        const uint64_t per8 = ((n16 + (uint64_t)cus * wpc / 2 - 1) / ((uint64_t)cus * wpc / 2) + 255) / 256 * 256;
        const uint32_t b8 = (uint32_t)((n16 + per8 - 1) / per8);
        report("wgcontig W8 U4 nt", wpc, time_it([&] {
                 hipLaunchKernelGGL((read_wgcontig<4, 8>), dim3(b8), dim3(512), 0, 0, buf, n16, per8, out);
               }));
      }
    }
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
