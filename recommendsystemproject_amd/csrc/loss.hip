// In-batch sampled-softmax loss with hard negatives (TwoTowerModel.compute_loss,
// TwoTowerModel.py:81-140; K15-K17). The batch-similarity GEMM S = U I^T runs on the MFMA GEMM;
// these kernels do the row-wise part fused: 1/T, off-diagonal equal-id collision mask (-1e9,
// trap T12), hard-negative logits U_i . H_in / T appended without masking, log-sum-exp,
// cross-entropy with labels arange(B). One workgroup per row; the row is streamed twice
// (max/sum, then value) from L2 and never copied. The backward turns S into dlogits / T in
// place so the two gradient GEMMs (dU = dS I, dI = dS^T U) need no extra scaling pass.
#include "common.h"

namespace rs {
namespace {

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max(v) : wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

__device__ __forceinline__ float logit_at(const float* Srow, const int64_t* ids, int64_t st,
                                          int64_t idi, int i, int j, float T) {
  if (ids && j != i && ids[(int64_t)j * st] == idi) return -1e9f;  // no ids: no collision mask
  return Srow[j] / T;
}

// hard-negative logit n of row i: dot(U_i, H[i, n]) / T computed by one wave; H element
// (i, n, c) at Hn[i*hs.row + n*hs.slot + c] ([B, N, D] contiguous, or the [N, B, D] output of one
// grouped item-tower pass viewed as [B, N, D])
struct HStride {
  int64_t row, slot;
};

__device__ float hard_logit(const float* U, const float* Hn, HStride hs, int i, int n, int D,
                            float T) {
  const int lane = threadIdx.x & 63;
  const float* h = Hn + (int64_t)i * hs.row + (int64_t)n * hs.slot;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += U[(int64_t)i * D + c] * h[c];
  return wave_sum(s) / T;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ S, int ld,
                                                     const float* __restrict__ U,
                                                     const float* __restrict__ Hn, HStride hs,
                                                     const int64_t* __restrict__ ids, int64_t st,
                                                     int B, int N, int D, float T,
                                                     float* __restrict__ lse,
                                                     float* __restrict__ row_loss) {
  __shared__ float red[8];
  __shared__ float hl[64];
  const int i = blockIdx.x;
  const float* Srow = S + (int64_t)i * ld;
  const int64_t idi = ids ? ids[(int64_t)i * st] : 0;
  const int wave = threadIdx.x >> 6;
  for (int n = wave; n < N; n += 4) {
    const float v = hard_logit(U, Hn, hs, i, n, D, T);
    if ((threadIdx.x & 63) == 0) hl[n] = v;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int j = threadIdx.x; j < B; j += 256) m = fmaxf(m, logit_at(Srow, ids, st, idi, i, j, T));
  for (int n = threadIdx.x; n < N; n += 256) m = fmaxf(m, hl[n]);
  m = block_reduce(m, red, true);
  float s = 0.f;
  for (int j = threadIdx.x; j < B; j += 256) s += expf(logit_at(Srow, ids, st, idi, i, j, T) - m);
  for (int n = threadIdx.x; n < N; n += 256) s += expf(hl[n] - m);
  s = block_reduce(s, red, false);
  if (threadIdx.x == 0) {
    const float l = m + logf(s);
    lse[i] = l;
    row_loss[i] = l - Srow[i] / T;
  }
}

// the logits matrix itself [B, B + N] (TwoTowerModel.py:95-136 before F.cross_entropy): one
// workgroup per row; the in-batch part from S, the hard-negative part by one wave per slot
__global__ __launch_bounds__(256) void logits_kernel(const float* __restrict__ S, int ld,
                                                     const float* __restrict__ U,
                                                     const float* __restrict__ Hn, HStride hs,
                                                     const int64_t* __restrict__ ids, int64_t st,
                                                     int B, int N, int D, float T,
                                                     float* __restrict__ out, int64_t ldo) {
  const int i = blockIdx.x;
  const float* Srow = S + (int64_t)i * ld;
  const int64_t idi = ids ? ids[(int64_t)i * st] : 0;
  float* o = out + (int64_t)i * ldo;
  for (int j = threadIdx.x; j < B; j += 256) o[j] = logit_at(Srow, ids, st, idi, i, j, T);
  for (int n = threadIdx.x >> 6; n < N; n += 4) {
    const float v = hard_logit(U, Hn, hs, i, n, D, T);
    if ((threadIdx.x & 63) == 0) o[B + n] = v;
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(float* __restrict__ S, int ld,
                                                     const float* __restrict__ U,
                                                     const float* __restrict__ Hn, HStride hs,
                                                     const int64_t* __restrict__ ids, int64_t st,
                                                     int B, int N, int D, float T,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ grad_out,
                                                     float* __restrict__ dhl) {
  const int i = blockIdx.x;
  float* Srow = S + (int64_t)i * ld;
  const int64_t idi = ids ? ids[(int64_t)i * st] : 0;
  const float l = lse[i];
  const float g = (grad_out ? *grad_out : 1.f) / (float)B / T;  // d loss / d S = dlogits / T
  for (int j = threadIdx.x; j < B; j += 256) {
    const float p = expf(logit_at(Srow, ids, st, idi, i, j, T) - l);
    Srow[j] = g * (p - (j == i ? 1.f : 0.f));
  }
  const int wave = threadIdx.x >> 6;
  for (int n = wave; n < N; n += 4) {
    const float v = hard_logit(U, Hn, hs, i, n, D, T);
    if ((threadIdx.x & 63) == 0) dhl[(int64_t)i * N + n] = g * expf(v - l);
  }
}

// dU += sum_n dhl[i,n] H[i,n,:]; dH[i,n,:] = dhl[i,n] U[i,:] (dH in the layout of H)
__global__ void hardneg_bwd_kernel(const float* __restrict__ U, const float* __restrict__ Hn,
                                   HStride hs, const float* __restrict__ dhl,
                                   float* __restrict__ dU, float* __restrict__ dH, int B, int N,
                                   int D) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * D) return;
  const int i = (int)(idx / D), c = (int)(idx % D);
  const float u = U[idx];
  float acc = 0.f;
  for (int n = 0; n < N; ++n) {
    const float w = dhl[(int64_t)i * N + n];
    const int64_t o = (int64_t)i * hs.row + (int64_t)n * hs.slot + c;
    acc += w * Hn[o];
    dH[o] = w * u;
  }
  dU[idx] += acc;
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_inbatch_ce_fwd(const float* S, int ld_s, const float* U, const float* Hn,
                                 int64_t h_row_stride, int64_t h_slot_stride,
                                 const int64_t* item_ids, int64_t id_stride, int B, int N, int D,
                                 float T, float* lse, float* row_loss, float* loss, void* stream) {
  RS_CHECK_ARG(S && lse && row_loss && loss, "rs_inbatch_ce_fwd: null pointer");
  RS_CHECK_ARG(B >= 1 && ld_s >= B && N >= 0 && N <= 64, "rs_inbatch_ce_fwd: bad shape B=%d N=%d", B, N);
  RS_CHECK_ARG(N == 0 || (U && Hn && D >= 1), "rs_inbatch_ce_fwd: hard negatives need U, H, D");
  hipStream_t st = as_stream(stream);
  const HStride hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
  ce_fwd_kernel<<<B, 256, 0, st>>>(S, ld_s, U, Hn, hs, item_ids, id_stride, B, N, D, T, lse, row_loss);
  RS_CHECK_LAUNCH("rs_inbatch_ce_fwd");
  return rs_sum(row_loss, B, 1.f / (float)B, loss, stream);
}

extern "C" int rs_inbatch_ce_bwd(float* S, int ld_s, const float* U, const float* Hn,
                                 int64_t h_row_stride, int64_t h_slot_stride,
                                 const int64_t* item_ids, int64_t id_stride, int B, int N, int D,
                                 float T, const float* lse, const float* grad_out, float* dhl,
                                 void* stream) {
  RS_CHECK_ARG(S && lse, "rs_inbatch_ce_bwd: null pointer");
  RS_CHECK_ARG(B >= 1 && ld_s >= B && N >= 0 && N <= 64, "rs_inbatch_ce_bwd: bad shape");
  RS_CHECK_ARG(N == 0 || (U && Hn && dhl && D >= 1), "rs_inbatch_ce_bwd: hard negatives need U, H, dhl");
  const HStride hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
  ce_bwd_kernel<<<B, 256, 0, as_stream(stream)>>>(S, ld_s, U, Hn, hs, item_ids, id_stride, B, N, D, T,
                                                  lse, grad_out, dhl);
  RS_CHECK_LAUNCH("rs_inbatch_ce_bwd");
  return 0;
}

extern "C" int rs_hardneg_bwd(const float* U, const float* Hn, int64_t h_row_stride,
                              int64_t h_slot_stride, const float* dhl, float* dU, float* dH, int B,
                              int N, int D, void* stream) {
  RS_CHECK_ARG(U && Hn && dhl && dU && dH && B >= 0 && N >= 1 && D >= 1, "rs_hardneg_bwd: bad args");
  const int64_t total = (int64_t)B * D;
  if (total == 0) return 0;
  const HStride hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
  hardneg_bwd_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(U, Hn, hs, dhl, dU, dH, B, N, D);
  RS_CHECK_LAUNCH("rs_hardneg_bwd");
  return 0;
}

extern "C" int rs_inbatch_logits(const float* S, int ld_s, const float* U, const float* Hn,
                                 int64_t h_row_stride, int64_t h_slot_stride,
                                 const int64_t* item_ids, int64_t id_stride, int B, int N, int D,
                                 float T, float* out, int64_t ld_out, void* stream) {
  RS_CHECK_ARG(S && out && B >= 1 && ld_s >= B && N >= 0 && ld_out >= B + N,
               "rs_inbatch_logits: bad args");
  RS_CHECK_ARG(N == 0 || (U && Hn && D >= 1), "rs_inbatch_logits: hard negatives need U, H, D");
  const HStride hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
  logits_kernel<<<B, 256, 0, as_stream(stream)>>>(S, ld_s, U, Hn, hs, item_ids, id_stride, B, N, D, T,
                                                  out, ld_out);
  RS_CHECK_LAUNCH("rs_inbatch_logits");
  return 0;
}
