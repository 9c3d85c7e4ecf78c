// On-box peak measurements reported beside the rooflines (bench.py; SURVEY.md §8 asks for the
// datasheet figures re-measured on the box): the HBM bandwidth of a float4 streaming copy and
// the dense bf16 MFMA rate of back-to-back v_mfma_f32_32x32x16_bf16.
#include "common.h"

namespace rs {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// dst[i] = src[i] over n float4s, one float4 per lane and n / 256 workgroups: the shape that
// measured best on the box (6.25 TB/s for 2 GiB, against 5.2-5.5 TB/s for grid-stride loops with
// 4-16 float4s per lane, default or non-temporal policy; tools/copy_variants.hip)
__global__ __launch_bounds__(256) void copy_f4_kernel(const floatx4* __restrict__ src, floatx4* __restrict__ dst,
                                                      int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// every wave: `iters` x 4 back-to-back 32x32x16 bf16 MFMAs (4 accumulators), operands from
// registers; one lane's sum is stored so the chain is live
__global__ __launch_bounds__(256) void mfma_bf16_kernel(float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(1.0f + 0.001f * (lane + j));
    b[j] = (__bf16)(0.5f - 0.001f * (lane - j));
  }
  floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) s += c0[e] + c1[e] + c2[e] + c3[e];
  if (lane == 0) out[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = s;
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_peak_copy(const void* src, void* dst, int64_t bytes, void* stream) {
  RS_CHECK_ARG(src && dst && bytes >= 16 && bytes % 16 == 0 && aligned16(src) && aligned16(dst),
               "rs_peak_copy: needs 16-byte aligned buffers, bytes a multiple of 16");
  const int64_t n = bytes / 16;
  RS_CHECK_ARG(n <= (int64_t)256 * 0x7fffffff, "rs_peak_copy: too large");
  copy_f4_kernel<<<(unsigned)cdiv(n, (int64_t)256), 256, 0, as_stream(stream)>>>(reinterpret_cast<const floatx4*>(src),
                                                      reinterpret_cast<floatx4*>(dst), n);
  RS_CHECK_LAUNCH("rs_peak_copy");
  return 0;
}

extern "C" int64_t rs_peak_mfma_flops(int blocks, int iters) {
  // per wave and iteration: 4 MFMAs x (32 x 32 x 16 x 2) flops; 4 waves per 256-thread block
  return (int64_t)blocks * 4 * iters * 4 * (32 * 32 * 16 * 2);
}

extern "C" int rs_peak_mfma(float* out, int blocks, int iters, void* stream) {
  RS_CHECK_ARG(out && blocks >= 1 && iters >= 1, "rs_peak_mfma: bad args");
  mfma_bf16_kernel<<<blocks, 256, 0, as_stream(stream)>>>(out, iters);
  RS_CHECK_LAUNCH("rs_peak_mfma");
  return 0;
}
