// Validation / Recall@K on the device (the reference's validate(),
// training_utils.py:121-275): scores = U · I_allᵀ run on the MFMA GEMM (rs_gemm_f32), then
//   rs_mask_history  — each user's training items to -inf (the per-user Python loop :238-252),
//   rs_topk_rows     — the K best columns of every row, sorted (torch.topk :256),
//   rs_recall_hits   — hit counts of the target item within the first k of each list (:258-262).
// top-K is an exact radix select (4 passes of 8 bits on order-preserving uint32 keys) followed by
// an ordered collection and a bitonic sort in LDS; ties are broken by the lower column index, so
// the result is deterministic. Catalogs larger than one launch's row are handled by chunking
// columns and running rs_topk_rows again over the per-chunk candidates (idx_in maps them back).
#include "common.h"

namespace rs {
namespace {

constexpr int kTopkThreads = 256;
constexpr int kTopkMax = 256;  // K <= 256

__device__ __forceinline__ uint32_t order_key(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending uint order == ascending float
}
__device__ __forceinline__ float key_value(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// columns [c0, c0 + n) of the catalog live at S[b*ld + (c - c0)] (one column chunk)
__global__ void mask_history_kernel(float* __restrict__ S, int64_t ld, int B, int64_t c0, int64_t n,
                                    const int64_t* __restrict__ user_ids, int64_t uid_stride,
                                    const int64_t* __restrict__ off, const int32_t* __restrict__ idx,
                                    int64_t U) {
  const int b = blockIdx.x;
  if (b >= B) return;
  const int64_t uid = user_ids[(int64_t)b * uid_stride];
  if (uid < 0 || uid >= U) return;
  const int64_t j0 = off[uid], j1 = off[uid + 1];
  for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const int64_t c = (int64_t)idx[j] - c0;
    if (c >= 0 && c < n) S[(int64_t)b * ld + c] = -INFINITY;
  }
}

// one workgroup per row
__global__ __launch_bounds__(kTopkThreads) void topk_kernel(const float* __restrict__ S, int64_t ld,
                                                            int N, int K,
                                                            const int32_t* __restrict__ idx_in,
                                                            int64_t ld_idx_in, int col_offset,
                                                            int32_t* __restrict__ out_idx,
                                                            float* __restrict__ out_val,
                                                            int64_t ld_out) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_mask, s_need, s_above;
  __shared__ uint32_t skey[kTopkMax];
  __shared__ int32_t sidx[kTopkMax];
  __shared__ uint32_t s_cnt_above;
  __shared__ uint32_t wscan[kTopkThreads / 64];
  const int b = blockIdx.x;
  const float* row = S + (int64_t)b * ld;
  const int tid = threadIdx.x;
  if (tid == 0) { s_prefix = 0; s_mask = 0; s_need = (uint32_t)K; s_above = 0; s_cnt_above = 0; }
  __syncthreads();
  // radix select of the K-th largest key: after the passes, T = s_prefix is that key,
  // s_above = number of keys > T (< K), s_need = how many keys == T to take
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    const uint32_t pre = s_prefix, msk = s_mask;
    for (int j = tid; j < N; j += kTopkThreads) {
      const uint32_t k = order_key(row[j]);
      if ((k & msk) == pre) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t need = s_need, acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= need) break;
        acc += hist[d];
      }
      s_above += acc;
      s_need = need - acc;
      s_prefix = pre | ((uint32_t)d << shift);
      s_mask = msk | (255u << shift);
    }
    __syncthreads();
  }
  const uint32_t T = s_prefix;
  const uint32_t above = s_above, need_eq = s_need;
  // collect: keys > T anywhere (order fixed later by the sort), keys == T in column order
  const int chunk = (N + kTopkThreads - 1) / kTopkThreads;
  const int c0 = tid * chunk, c1 = min(N, c0 + chunk);
  uint32_t my_eq = 0;
  for (int j = c0; j < c1; ++j) {
    const uint32_t k = order_key(row[j]);
    if (k > T) {
      const uint32_t slot = atomicAdd(&s_cnt_above, 1u);
      skey[slot] = k;
      sidx[slot] = j;
    } else if (k == T) {
      ++my_eq;
    }
  }
  // exclusive scan of my_eq over threads (column order)
  uint32_t incl = my_eq;
  const int lane = tid & 63, w = tid >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wscan[w] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < w; ++i) base += wscan[i];
  uint32_t rank = base + incl - my_eq;
  for (int j = c0; j < c1 && rank < need_eq; ++j) {
    if (order_key(row[j]) == T) {
      skey[above + rank] = T;
      sidx[above + rank] = j;
      ++rank;
    }
  }
  __syncthreads();
  // bitonic sort of the K entries (padded to a power of two) by key desc, column asc
  int P = 1;
  while (P < K) P <<= 1;
  for (int i = K + tid; i < P; i += kTopkThreads) { skey[i] = 0; sidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += kTopkThreads) {
        const int jx = i ^ stride;
        if (jx > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ka = skey[i], kb = skey[jx];
          const int32_t ia = sidx[i], ib = sidx[jx];
          // "a before b" in the final order: larger key, then smaller column
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (desc ? !a_first : a_first) {
            skey[i] = kb; skey[jx] = ka;
            sidx[i] = ib; sidx[jx] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < K; i += kTopkThreads) {
    const int32_t c = sidx[i];
    out_idx[(int64_t)b * ld_out + i] = idx_in ? idx_in[(int64_t)b * ld_idx_in + c] : c + col_offset;
    if (out_val) out_val[(int64_t)b * ld_out + i] = key_value(skey[i]);
  }
}

__global__ void recall_hits_kernel(const int32_t* __restrict__ topk, int B, int K,
                                   const int64_t* __restrict__ item_ids,
                                   const int64_t* __restrict__ targets, int64_t t_stride,
                                   const int32_t* __restrict__ ks, int nk, int32_t* __restrict__ hits) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = targets[(int64_t)b * t_stride];
  int first = K;  // position of the first hit
  for (int j = 0; j < K; ++j)
    if (item_ids[topk[(int64_t)b * K + j]] == t) { first = j; break; }
  for (int i = 0; i < nk; ++i)
    if (first < ks[i]) atomicAdd(&hits[i], 1);
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_mask_history(float* S, int64_t ld, int B, int64_t col0, int64_t ncols,
                               const int64_t* user_ids, int64_t uid_stride, const int64_t* hist_off,
                               const int32_t* hist_idx, int64_t num_users, void* stream) {
  RS_CHECK_ARG(S && user_ids && hist_off && (hist_idx || num_users == 0) && B >= 0 && ld >= ncols &&
                   col0 >= 0,
               "rs_mask_history: bad args");
  if (B == 0 || num_users == 0) return 0;
  mask_history_kernel<<<B, 256, 0, as_stream(stream)>>>(S, ld, B, col0, ncols, user_ids, uid_stride,
                                                        hist_off, hist_idx, num_users);
  RS_CHECK_LAUNCH("rs_mask_history");
  return 0;
}

extern "C" int rs_topk_rows(const float* S, int64_t ld, int B, int N, int K, const int32_t* idx_in,
                            int64_t ld_idx_in, int col_offset, int32_t* out_idx, float* out_val,
                            int64_t ld_out, void* stream) {
  RS_CHECK_ARG(S && out_idx && B >= 0 && N >= 1 && K >= 1 && K <= kTopkMax && K <= N && ld >= N &&
                   ld_out >= K,
               "rs_topk_rows: bad args (B=%d N=%d K=%d; K <= min(N, 256))", B, N, K);
  if (B == 0) return 0;
  topk_kernel<<<B, kTopkThreads, 0, as_stream(stream)>>>(S, ld, N, K, idx_in, ld_idx_in, col_offset,
                                                         out_idx, out_val, ld_out);
  RS_CHECK_LAUNCH("rs_topk_rows");
  return 0;
}

extern "C" int rs_recall_hits(const int32_t* topk_idx, int B, int K, const int64_t* item_ids,
                              const int64_t* targets, int64_t target_stride, const int32_t* ks,
                              int nk, int32_t* hits, void* stream) {
  RS_CHECK_ARG(topk_idx && item_ids && targets && ks && hits && B >= 0 && K >= 1 && nk >= 1,
               "rs_recall_hits: bad args");
  if (B == 0) return 0;
  recall_hits_kernel<<<cdiv(B, 256), 256, 0, as_stream(stream)>>>(topk_idx, B, K, item_ids, targets,
                                                                   target_stride, ks, nk, hits);
  RS_CHECK_LAUNCH("rs_recall_hits");
  return 0;
}
