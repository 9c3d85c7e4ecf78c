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

extern "C" int rs_dropout_bwd(float* dx, int64_t n, float p, const int64_t* key, int site,
                              void* stream) {
  RS_CHECK_ARG(dx && key && n >= 0 && p >= 0.f && p <= 1.f, "rs_dropout_bwd: bad args");
  if (n == 0) return 0;
  dropout_bwd_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(dx, n, p, key, site);
  RS_CHECK_LAUNCH("rs_dropout_bwd");
  return 0;
}
