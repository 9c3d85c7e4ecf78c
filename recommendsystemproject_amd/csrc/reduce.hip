// Deterministic column / full reductions (bias gradients, positional-embedding gradients,
// LayerNorm gamma/beta gradients, mean loss). Two passes with a fixed summation order so that
// repeated runs are bitwise identical (no float atomics).
#include "common.h"

namespace rs {

int colsum_chunks(int M) {
  int s = cdiv(M, 256);
  if (s < 1) s = 1;
  if (s > 512) s = 512;
  return s;
}

namespace {

template <int TPR>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ X, int M,
                                                             int N, int ldx, int rows_per_chunk,
                                                             float* __restrict__ ws) {
  constexpr int RL = 256 / TPR;
  __shared__ float red[256];
  const int c = blockIdx.x * TPR + (threadIdx.x % TPR);
  const int rl = threadIdx.x / TPR;
  const int s = blockIdx.y;
  const int r0 = s * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  float acc = 0.f;
  if (c < N)
    for (int m = r0 + rl; m < r1; m += RL) acc += X[(int64_t)m * ldx + c];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rl == 0 && c < N) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < RL; ++i) v += red[i * TPR + (threadIdx.x % TPR)];
    ws[(int64_t)s * N + c] = v;
  }
}

__global__ void colsum_final_kernel(const float* __restrict__ ws, int S, int N, float scale,
                                    float beta, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += ws[(int64_t)s * N + c];
  out[c] = (beta != 0.f ? beta * out[c] : 0.f) + scale * v;
}

__global__ __launch_bounds__(1024) void sum_kernel(const float* __restrict__ x, int n, float scale,
                                                   float* __restrict__ out) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    *out = (float)(t * (double)scale);
  }
}

}  // namespace

int colsum_launch(const float* X, int M, int N, int ldx, float scale, float beta, float* out,
                  float* ws, hipStream_t st) {
  const int S = colsum_chunks(M);
  const int rpc = cdiv(M, S);
  if (N <= 64) {
    colsum_partial_kernel<64><<<dim3(cdiv(N, 64), S), 256, 0, st>>>(X, M, N, ldx, rpc, ws);
  } else if (N <= 128) {
    colsum_partial_kernel<128><<<dim3(cdiv(N, 128), S), 256, 0, st>>>(X, M, N, ldx, rpc, ws);
  } else {
    colsum_partial_kernel<256><<<dim3(cdiv(N, 256), S), 256, 0, st>>>(X, M, N, ldx, rpc, ws);
  }
  RS_CHECK_LAUNCH("colsum partial");
  colsum_final_kernel<<<cdiv(N, 256), 256, 0, st>>>(ws, S, N, scale, beta, out);
  RS_CHECK_LAUNCH("colsum final");
  return 0;
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_colsum_ws_bytes(int M, int N) {
  return (int64_t)colsum_chunks(M) * N * (int64_t)sizeof(float);
}

extern "C" int rs_colsum(const float* X, int M, int N, int ldx, float scale, float beta,
                         float* out, float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && N >= 0 && ldx >= N, "rs_colsum: bad shape M=%d N=%d ldx=%d", M, N, ldx);
  if (N == 0) return 0;
  RS_CHECK_ARG(X && out && ws, "rs_colsum: null pointer");
  if (M == 0) M = 0;
  return colsum_launch(X, M, N, ldx, scale, beta, out, ws, as_stream(stream));
}

extern "C" int rs_sum(const float* x, int n, float scale, float* out, void* stream) {
  RS_CHECK_ARG(n >= 0 && x && out, "rs_sum: bad args");
  sum_kernel<<<1, 1024, 0, as_stream(stream)>>>(x, n, scale, out);
  RS_CHECK_LAUNCH("rs_sum");
  return 0;
}
