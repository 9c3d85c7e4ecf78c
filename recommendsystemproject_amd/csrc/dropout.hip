// Dropout (nn.Dropout / F.dropout in training mode) for the sites the reference has outside the
// fused kernels: the sequence input (projection dropout, + positional embedding, second dropout:
// SequenceFeatureProcessor.py:77-83, trap T5), the FFN inner dropout and the MLP dropouts
// (Tower.py:19). Attention-probability dropout and the two residual dropouts of the encoder
// layer are fused into rs_attn_* and rs_add_layernorm_* (same mask function, rng.h).
#include "common.h"
#include "rng.h"

namespace rs {
namespace {

__global__ void rng_next_kernel(int64_t* state, int64_t* key) {
  key[0] = state[0];
  key[1] = state[1];
  state[1] = state[1] + 1;
}

__global__ void dropout_fwd_kernel(float* __restrict__ x, int64_t n, int N,
                                   const float* __restrict__ aux, int ld_aux, int aux_mod, float p,
                                   const int64_t* __restrict__ key, int site) {
  const DropKey k = make_key(key, site, p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i];
    if (aux) {
      const int64_t row = i / N;
      v += aux[(row % aux_mod) * ld_aux + (i - row * N)];
    }
    x[i] = v * keep_mult(k, (uint64_t)i);
  }
}

__global__ void dropout_bwd_kernel(float* __restrict__ dx, int64_t n, float p,
                                   const int64_t* __restrict__ key, int site) {
  const DropKey k = make_key(key, site, p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] *= keep_mult(k, (uint64_t)i);
}

// Backward of the sequence input's two dropouts around the positional-embedding add
// (SequenceFeatureProcessor.py:77-83: x = drop_b(drop_a(cat W^T + b) + pos[l])) in one pass over
// dx [rows, N] (N = L * d): v = dx * mask_b, pos_grad[n] += sum over rows of v (fixed-order
// per-workgroup partials), dx = v * mask_a. The three-pass form (rs_dropout_bwd, rs_colsum,
// rs_dropout_bwd) read and wrote dx twice more. Element i = row * N + n draws exactly as
// rs_dropout_* (keep4: two pair hashes per 4 elements).
constexpr int kSeqDropCols = 4;  // float4 groups per thread and row (N <= 4 * 4 * 256)

__global__ __launch_bounds__(256) void seq_input_dropout_bwd_kernel(float* __restrict__ dx, int rows, int N,
                                                                    int rows_per_block, float p,
                                                                    const int64_t* __restrict__ key,
                                                                    int site_a, int site_b,
                                                                    float* __restrict__ ws) {
  const DropKey ka = make_key(key, site_a, p), kb = make_key(key, site_b, p);
  const int G4 = N / 4;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float4 acc[kSeqDropCols];
#pragma unroll
  for (int u = 0; u < kSeqDropCols; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  // the next row's loads are issued before this row's hashes and stores (one row in flight
  // behind the other: the loop was a load round trip per row)
  // (unconditional loads -- row and column clamped, the extra values unused: a guarded load
  // would make the join wait for it)
  float4 nx[kSeqDropCols];
  if (r0 >= r1) return;
#pragma unroll
  for (int u = 0; u < kSeqDropCols; ++u) {
    const int g = min(threadIdx.x + 256 * u, G4 - 1);
    nx[u] = *reinterpret_cast<const float4*>(dx + (int64_t)r0 * N + 4 * g);
  }
  for (int row = r0; row < r1; ++row) {
    float4 v[kSeqDropCols];
#pragma unroll
    for (int u = 0; u < kSeqDropCols; ++u) v[u] = nx[u];
    const int rn = min(row + 1, r1 - 1);
#pragma unroll
    for (int u = 0; u < kSeqDropCols; ++u) {
      const int g = min(threadIdx.x + 256 * u, G4 - 1);
      nx[u] = *reinterpret_cast<const float4*>(dx + (int64_t)rn * N + 4 * g);
    }
#pragma unroll
    for (int u = 0; u < kSeqDropCols; ++u) {
      const int g = threadIdx.x + 256 * u;
      if (g >= G4) continue;
      const uint64_t i0 = (uint64_t)row * N + 4 * g;
      float mb[4], ma[4];
      keep4(kb, i0, mb);
      keep4(ka, i0, ma);
      float4 t = v[u];
      t.x *= mb[0]; t.y *= mb[1]; t.z *= mb[2]; t.w *= mb[3];
      acc[u].x += t.x; acc[u].y += t.y; acc[u].z += t.z; acc[u].w += t.w;
      t.x *= ma[0]; t.y *= ma[1]; t.z *= ma[2]; t.w *= ma[3];
      *reinterpret_cast<float4*>(dx + (int64_t)row * N + 4 * g) = t;
    }
  }
#pragma unroll
  for (int u = 0; u < kSeqDropCols; ++u) {
    const int g = threadIdx.x + 256 * u;
    if (g < G4) *reinterpret_cast<float4*>(ws + (int64_t)blockIdx.x * N + 4 * g) = acc[u];
  }
}

int seq_drop_blocks(int rows) {
  int b = cdiv(rows, 8);  // >= 8 rows per workgroup
  return b > 512 ? 512 : (b < 1 ? 1 : b);
}

int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return b < 1 ? 1 : (int)b;
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_rng_next(int64_t* state, int64_t* key, void* stream) {
  RS_CHECK_ARG(state && key, "rs_rng_next: null pointer");
  rng_next_kernel<<<1, 1, 0, as_stream(stream)>>>(state, key);
  RS_CHECK_LAUNCH("rs_rng_next");
  return 0;
}

extern "C" int rs_dropout_fwd(float* x, int64_t n, int N, const float* aux, int ld_aux,
                              int aux_mod, float p, const int64_t* key, int site, void* stream) {
  RS_CHECK_ARG(x && key && n >= 0 && p >= 0.f && p <= 1.f, "rs_dropout_fwd: bad args");
  RS_CHECK_ARG(!aux || (N > 0 && aux_mod > 0 && ld_aux >= N), "rs_dropout_fwd: bad aux");
  if (n == 0) return 0;
  dropout_fwd_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(x, n, N > 0 ? N : 1, aux, ld_aux,
                                                                  aux_mod, p, key, site);
  RS_CHECK_LAUNCH("rs_dropout_fwd");
  return 0;
}

extern "C" int64_t rs_seq_input_dropout_bwd_ws_bytes(int rows, int N) {
  return (int64_t)seq_drop_blocks(rows) * N * (int64_t)sizeof(float);
}

extern "C" int rs_seq_input_dropout_bwd(float* dx, int rows, int N, float p, const int64_t* key, int site_a,
                                        int site_b, float* pos_grad, float* ws, void* stream) {
  RS_CHECK_ARG(dx && key && pos_grad && ws && rows >= 0 && N > 0 && N % 4 == 0 &&
                   N <= 4 * kSeqDropCols * 256 && p >= 0.f && p < 1.f && aligned16(dx),
               "rs_seq_input_dropout_bwd: bad args (N=%d)", N);
  if (rows == 0) return 0;
  const int nb = seq_drop_blocks(rows);
  const int rpb = cdiv(rows, nb);
  hipStream_t st = as_stream(stream);
  seq_input_dropout_bwd_kernel<<<cdiv(rows, rpb), 256, 0, st>>>(dx, rows, N, rpb, p, key, site_a, site_b, ws);
  RS_CHECK_LAUNCH("rs_seq_input_dropout_bwd");
  return partials_reduce_any(ws, cdiv(rows, rpb), N, N, 1.f, 1.f, pos_grad, nullptr, st);
}

extern "C" int rs_dropout_bwd(float* dx, int64_t n, float p, const int64_t* key, int site,
                              void* stream) {
  RS_CHECK_ARG(dx && key && n >= 0 && p >= 0.f && p <= 1.f, "rs_dropout_bwd: bad args");
  if (n == 0) return 0;
  dropout_bwd_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(dx, n, p, key, site);
  RS_CHECK_LAUNCH("rs_dropout_bwd");
  return 0;
}
