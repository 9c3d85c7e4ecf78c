// Staging a small fp32 matrix (weights, <= 256 x 256) from HBM into LDS at kernel start.
// A plain `for (i = tid; i < n; i += blockDim) lds[..] = src[..]` loop issues one load, waits for
// it, stores, and repeats: one full global-memory latency per element per thread (tens of us per
// launch for a 256 x 64 weight). Here every thread issues a batch of 16-byte loads before it
// writes any of them, so their latencies overlap.
#pragma once
#include <stdint.h>

namespace rs {

typedef float stage_f4 __attribute__((ext_vector_type(4)));

// src [ROWS][COLS] fp32 with row stride ld (16-byte aligned rows, COLS % 4 == 0) ->
// put(row, col, float4 of columns col..col+3), NTHR threads, batches of BATCH loads per thread;
// ok(row, col) false -> zeros, no load (ragged edges)
struct stage_all {
  __device__ bool operator()(int, int) const { return true; }
};
template <int ROWS, int COLS, int NTHR, int BATCH = 8, typename Put, typename Ok = stage_all>
__device__ __forceinline__ void stage_batched(const float* src, int64_t ld, Put put, Ok ok = Ok()) {
  constexpr int C4 = COLS / 4, NV = ROWS * C4;
  constexpr int PER = (NV + NTHR - 1) / NTHR;
  typedef const __attribute__((address_space(1))) stage_f4* gp;
#pragma unroll
  for (int b0 = 0; b0 < PER; b0 += BATCH) {
    stage_f4 v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int idx = threadIdx.x + NTHR * (b0 + i);
      v[i] = stage_f4{0.f, 0.f, 0.f, 0.f};
      if (b0 + i < PER && idx < NV && ok(idx / C4, (idx % C4) * 4))
        v[i] = *(gp)(src + (int64_t)(idx / C4) * ld + (idx % C4) * 4);
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int idx = threadIdx.x + NTHR * (b0 + i);
      if (b0 + i < PER && idx < NV) put(idx / C4, (idx % C4) * 4, v[i]);
    }
  }
}

}  // namespace rs
