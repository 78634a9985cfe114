// wire.hip -- EpochTreeObject protobuf wire bytes on device.
//
// The per-object encoder/decoder (reference semantics, field layout) is in wire_body.hpp, shared
// with the fused verify kernel (verify.hip).
//
// Encode: one wave per object, lanes write the 10-byte bucket entries and the size varints at
// offsets from a wave prefix sum. Decode: one wave per object, staged into LDS (objects up to
// 8 KiB) and parsed by the whole wave (bucket-entry and packed-size runs 64 at a time; 256 when
// cap > 64, the same results in a quarter of the dependent cursor steps).
#include "wire_body.hpp"

namespace mde {
namespace {

__global__ __launch_bounds__(64) void encode_kernel(WireEncodeLaunch a) {
  encode_object(a, blockIdx.x, threadIdx.x);
}

constexpr uint32_t kDecodeStageBytes = 8u * 1024u;

template <uint32_t kWin>
__global__ __launch_bounds__(64) void decode_kernel(WireDecodeLaunch a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[kDecodeStageBytes];
  __shared__ uint32_t gstack[kWireGroupDepth];
  const uint32_t i = blockIdx.x, lane = threadIdx.x;
  const uint8_t* obj = a.bytes + a.off[i];
  const uint64_t n = a.off[i + 1] - a.off[i];
  if (n + 4 <= kDecodeStageBytes) {
    const uint8_t* staged = stage_object(obj, n, stage, lane);
    __syncthreads();
    decode_object<kWin>(a, i, staged, n, lane, gstack);
  } else {
    decode_object<kWin>(a, i, obj, n, lane, gstack);
  }
}

}  // namespace

hipError_t launch_wire_encode(const WireEncodeLaunch& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(encode_kernel, dim3(a.n), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_wire_decode(const WireDecodeLaunch& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  if (a.cap > 64)
    hipLaunchKernelGGL(decode_kernel<4>, dim3(a.n), dim3(64), 0, st, a);
  else
    hipLaunchKernelGGL(decode_kernel<1>, dim3(a.n), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace mde
