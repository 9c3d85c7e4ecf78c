// Lazy-exact Adam for large embedding tables (SURVEY.md §7.2 hard part 1, trap T16).
//
// The reference trains nn.Embedding with dense gradients, so torch.optim.Adam moves EVERY row of
// every table every step: a row whose exp_avg is non-zero keeps drifting after it was last
// looked up. At 10M-100M rows that is a 75-360 GB sweep per step. Here a large table keeps
// per-row `last` (the optimizer step the row was last brought to) and only rows looked up in a
// step are touched:
//   forward : rs_sparse_touch dedups the batch's ids into a row list; rs_sparse_catchup replays
//             the skipped zero-gradient Adam steps (last+1 .. t) for those rows before they are
//             gathered, so the forward sees exactly the weights dense Adam would have produced;
//   backward: the ordinary scatter-add writes their gradient rows;
//   step    : rs_sparse_adam applies step t to the listed rows with their (clipped) gradient,
//             zeroes the gradient rows and clears the list; rs_sparse_sqnorm contributes the
//             listed rows to the global clip norm;
//   flush   : rs_sparse_flush brings every row to step t (before state_dict / checkpoint).
// The replay runs the same fp32 operation sequence as the dense kernel (adam_step_elem) with the
// same per-step constants (consts[s] = {lr/bc1(s), sqrt(bc2(s))}, written once per step by
// rs_adam_prepare), so lazy and dense Adam are bitwise identical. With weight_decay == 0 a row
// whose exp_avg and exp_avg_sq are zero does not move, which is what makes skipping it exact.
#include "common.h"

// no fma contraction: the dense and the lazy (sparse.hip) Adam must round identically
#pragma clang fp contract(off)

namespace rs {
namespace {

struct Hyper {
  float b1, b2, one_m_b1, one_m_b2, eps, wd;
};

__device__ __forceinline__ void adam_step_elem(const Hyper& h, float step_size, float bc2_sqrt,
                                               float gs, float& p, float& m, float& v) {
  if (h.wd != 0.f) gs = gs + h.wd * p;
  m = m + h.one_m_b1 * (gs - m);
  v = v * h.b2 + h.one_m_b2 * gs * gs;
  const float denom = sqrtf(v) / bc2_sqrt + h.eps;
  p = p - step_size * (m / denom);
}

// replay zero-gradient steps s = from .. to (inclusive)
__device__ __forceinline__ void replay(const Hyper& h, const float2* __restrict__ consts, int from,
                                       int to, float& p, float& m, float& v) {
  if (h.wd == 0.f && m == 0.f && v == 0.f) return;  // exact: such an element does not move
  for (int s = from; s <= to; ++s) {
    const float2 c = consts[s];
    adam_step_elem(h, c.x, c.y, 0.f, p, m, v);
  }
}

// consts[0] (step 0 never runs) holds {cap as int bits, overflow flag as int bits}: every reader
// clamps its step index to cap - 1, so a graph replayed past the capacity reads no memory past the
// table (the constants it then uses are stale: Adam.check_errors raises on the overflow flag)
__global__ void adam_prepare_kernel(int64_t* step, float2* consts, int cap, float lr, float b1,
                                    float b2) {
  const int64_t t = *step + 1;
  *step = t;
  if (t < cap) {
    const double bc1 = 1.0 - pow((double)b1, (double)t), bc2 = 1.0 - pow((double)b2, (double)t);
    consts[t] = make_float2((float)((double)lr / bc1), (float)sqrt(bc2));
    if (t == 1) consts[0] = make_float2(__int_as_float(cap), __int_as_float(0));
  } else {
    consts[0] = make_float2(__int_as_float(cap), __int_as_float(1));
  }
}

// the step index clamped into the constants table (see adam_prepare_kernel)
__device__ __forceinline__ int clamp_step(const float2* consts, int64_t t) {
  const int cap = __float_as_int(consts[0].x);
  return t < cap ? (int)t : cap - 1;
}

__global__ void touch_kernel(const int64_t* __restrict__ ids, int rows, int bag, int64_t stride,
                             int64_t vocab, int64_t pad, int* __restrict__ flag,
                             int* __restrict__ list, int* __restrict__ count) {
  const int64_t total = (int64_t)rows * bag;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / bag, l = e - r * bag;
    const int64_t id = ids[r * stride + l];
    if (id < 0 || id >= vocab || id == pad) continue;
    // flag = lookups of the row this step (the gradient scatter stores instead of adding when 1)
    if (atomicAdd(&flag[id], 1) == 0) list[atomicAdd(count, 1)] = (int)id;
  }
}

// one 64-lane wave per listed row (D <= 256: each lane owns D/64 columns)
__global__ __launch_bounds__(256) void catchup_kernel(float* __restrict__ p, float* __restrict__ m,
                                                      float* __restrict__ v, int* __restrict__ last,
                                                      const int* __restrict__ list,
                                                      const int* __restrict__ count, int D,
                                                      const int64_t* __restrict__ step,
                                                      const float2* __restrict__ consts, Hyper h) {
  const int n = *count;
  const int target = clamp_step(consts, *step);
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
    const int row = list[i];
    const int from = last[row] + 1;
    if (from > target) continue;
    for (int c = lane; c < D; c += 64) {
      const int64_t o = (int64_t)row * D + c;
      float pp = p[o], mm = m[o], vv = v[o];
      replay(h, consts, from, target, pp, mm, vv);
      p[o] = pp; m[o] = mm; v[o] = vv;
    }
    if (lane == 0) last[row] = target;
  }
}

__global__ __launch_bounds__(256) void sparse_adam_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    int* __restrict__ last, int* __restrict__ flag, const int* __restrict__ list,
    const int* __restrict__ count, int D, const int64_t* __restrict__ step,
    const float2* __restrict__ consts, Hyper h, float scale, const float* __restrict__ coef) {
  const int n = *count;
  const int t = clamp_step(consts, *step);
  const float s = scale * (coef ? *coef : 1.f);
  const float2 ct = consts[t];
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
    const int row = list[i];
    const int from = last[row] + 1;
    for (int c = lane; c < D; c += 64) {
      const int64_t o = (int64_t)row * D + c;
      float pp = p[o], mm = m[o], vv = v[o];
      if (from <= t - 1) replay(h, consts, from, t - 1, pp, mm, vv);
      adam_step_elem(h, ct.x, ct.y, g[o] * s, pp, mm, vv);
      p[o] = pp; m[o] = mm; v[o] = vv;
      g[o] = 0.f;
    }
    if (lane == 0) {
      last[row] = t;
      flag[row] = 0;
    }
  }
}

__global__ __launch_bounds__(256) void sparse_sqnorm_kernel(const float* __restrict__ g,
                                                            const int* __restrict__ list,
                                                            const int* __restrict__ count, int D,
                                                            float scale, double* __restrict__ ws) {
  __shared__ double red[4];
  const int n = *count;
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {
    const int row = list[i];
    for (int c = lane; c < D; c += 64) {
      const float a = g[(int64_t)row * D + c] * scale;
      acc += (double)(a * a);
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void flush_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                             int* __restrict__ last, int64_t V, int D,
                             const int64_t* __restrict__ step, const float2* __restrict__ consts,
                             Hyper h) {
  const int target = clamp_step(consts, *step);
  const int lane = threadIdx.x & 63;
  for (int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6); row < V; row += (int64_t)gridDim.x * 4) {
    const int from = last[row] + 1;
    if (from > target) continue;
    for (int c = lane; c < D; c += 64) {
      const int64_t o = row * D + c;
      float pp = p[o], mm = m[o], vv = v[o];
      replay(h, consts, from, target, pp, mm, vv);
      p[o] = pp; m[o] = mm; v[o] = vv;
    }
    if (lane == 0) last[row] = target;
  }
}

__global__ void reset_kernel(int* count) { *count = 0; }

// ---- ordered row list from flags (deterministic order for the data-parallel union) ----------
constexpr int kCompactChunk = 4096;  // flags per block: 256 threads x 16

__global__ __launch_bounds__(256) void compact_count_kernel(const int* __restrict__ flag, int64_t V,
                                                            int* __restrict__ part) {
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk;
  int c = 0;
  for (int j = threadIdx.x; j < kCompactChunk; j += 256) {
    const int64_t i = base + j;
    c += (i < V && flag[i] != 0);
  }
  __shared__ int red[4];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// exclusive scan of the per-chunk counts in one block; total -> *count
__global__ __launch_bounds__(1024) void compact_scan_kernel(int* __restrict__ part, int nb,
                                                            int* __restrict__ count) {
  __shared__ int carry_s;
  __shared__ int wsum[16];
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < nb; base += 1024) {
    const int i = base + threadIdx.x;
    const int x = i < nb ? part[i] : 0;
    // inclusive wave scan
    int y = x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(y, o, 64);
      if (lane >= o) y += t;
    }
    if (lane == 63) wsum[w] = y;
    __syncthreads();
    int pre = carry_s;
    for (int k = 0; k < w; ++k) pre += wsum[k];
    if (i < nb) part[i] = pre + y - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry_s = pre + y;
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = carry_s;
}

__global__ __launch_bounds__(256) void compact_write_kernel(const int* __restrict__ flag, int64_t V,
                                                            const int* __restrict__ part,
                                                            int* __restrict__ list) {
  // each thread owns 16 consecutive flags; block-exclusive scan of thread counts keeps order
  const int64_t base = (int64_t)blockIdx.x * kCompactChunk + threadIdx.x * 16;
  int c = 0;
  for (int j = 0; j < 16; ++j) c += (base + j < V && flag[base + j] != 0);
  __shared__ int wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int y = c;
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(y, o, 64);
    if (lane >= o) y += t;
  }
  if (lane == 63) wsum[w] = y;
  __syncthreads();
  int pos = part[blockIdx.x] + y - c;
  for (int k = 0; k < w; ++k) pos += wsum[k];
  for (int j = 0; j < 16; ++j)
    if (base + j < V && flag[base + j] != 0) list[pos++] = (int)(base + j);
}

// ---- row-sparse gradient exchange buffers: [cap ids (int32 bits)][cap x D rows] --------------
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ g,
                                                   const int* __restrict__ list,
                                                   const int* __restrict__ count, int D, int cap,
                                                   float* __restrict__ buf) {
  const int n = min(*count, cap);
  int* ids = reinterpret_cast<int*>(buf);
  float* rows = buf + cap;
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < cap; i += gridDim.x * 4) {
    const int row = i < n ? list[i] : -1;
    if (lane == 0) ids[i] = row;
    if (row >= 0)
      for (int c = lane; c < D; c += 64) rows[(int64_t)i * D + c] = g[(int64_t)row * D + c];
  }
}

__global__ __launch_bounds__(256) void unpack_add_kernel(float* __restrict__ g,
                                                         int* __restrict__ flag,
                                                         const float* __restrict__ buf, int D,
                                                         int cap) {
  const int* ids = reinterpret_cast<const int*>(buf);
  const float* rows = buf + cap;
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < cap; i += gridDim.x * 4) {
    const int row = ids[i];
    if (row < 0) continue;
    for (int c = lane; c < D; c += 64) g[(int64_t)row * D + c] += rows[(int64_t)i * D + c];
    if (lane == 0) flag[row] = 1;
  }
}

__global__ void overflow_kernel(const int* count, int cap, int* err) {
  if (*count > cap) atomicOr(err, 2);
}

Hyper make_hyper(float b1, float b2, float eps, float wd) {
  Hyper h;
  h.b1 = b1; h.b2 = b2; h.one_m_b1 = 1.f - b1; h.one_m_b2 = 1.f - b2; h.eps = eps; h.wd = wd;
  return h;
}

constexpr int kSparseGrid = 2048;

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_adam_prepare(int64_t* step, float* consts, int cap, float lr, float beta1,
                               float beta2, void* stream) {
  RS_CHECK_ARG(step && consts && cap > 1, "rs_adam_prepare: bad args");
  adam_prepare_kernel<<<1, 1, 0, as_stream(stream)>>>(step, reinterpret_cast<float2*>(consts), cap,
                                                       lr, beta1, beta2);
  RS_CHECK_LAUNCH("rs_adam_prepare");
  return 0;
}

extern "C" int rs_sparse_touch(const int64_t* ids, int rows, int bag, int64_t row_stride,
                               int64_t vocab, int64_t pad, int* flag, int* list, int* count,
                               void* stream) {
  RS_CHECK_ARG(ids && flag && list && count && rows >= 0 && bag >= 1, "rs_sparse_touch: bad args");
  const int64_t total = (int64_t)rows * bag;
  if (total == 0) return 0;
  int blocks = cdiv(total, 256);
  if (blocks > 4096) blocks = 4096;
  touch_kernel<<<blocks, 256, 0, as_stream(stream)>>>(ids, rows, bag, row_stride, vocab, pad, flag,
                                                       list, count);
  RS_CHECK_LAUNCH("rs_sparse_touch");
  return 0;
}

extern "C" int rs_sparse_catchup(float* p, float* m, float* v, int* last, const int* list,
                                 const int* count, int D, const int64_t* step, const float* consts,
                                 float beta1, float beta2, float eps, float weight_decay,
                                 void* stream) {
  RS_CHECK_ARG(p && m && v && last && list && count && step && consts && D >= 1,
               "rs_sparse_catchup: bad args");
  catchup_kernel<<<kSparseGrid, 256, 0, as_stream(stream)>>>(
      p, m, v, last, list, count, D, step, reinterpret_cast<const float2*>(consts),
      make_hyper(beta1, beta2, eps, weight_decay));
  RS_CHECK_LAUNCH("rs_sparse_catchup");
  return 0;
}

extern "C" int rs_sparse_adam(float* p, float* g, float* m, float* v, int* last, int* flag,
                              const int* list, int* count, int D, const int64_t* step,
                              const float* consts, float beta1, float beta2, float eps,
                              float weight_decay, float scale, const float* coef, void* stream) {
  RS_CHECK_ARG(p && g && m && v && last && flag && list && count && step && consts && D >= 1,
               "rs_sparse_adam: bad args");
  hipStream_t st = as_stream(stream);
  sparse_adam_kernel<<<kSparseGrid, 256, 0, st>>>(p, g, m, v, last, flag, list, count, D, step,
                                                  reinterpret_cast<const float2*>(consts),
                                                  make_hyper(beta1, beta2, eps, weight_decay),
                                                  scale, coef);
  RS_CHECK_LAUNCH("rs_sparse_adam");
  reset_kernel<<<1, 1, 0, st>>>(count);
  RS_CHECK_LAUNCH("rs_sparse_adam reset");
  return 0;
}

extern "C" int rs_sparse_sqnorm_parts(void) { return kSparseGrid; }

extern "C" int rs_sparse_sqnorm(const float* g, const int* list, const int* count, int D,
                                float scale, double* ws, void* stream) {
  RS_CHECK_ARG(g && list && count && ws && D >= 1, "rs_sparse_sqnorm: bad args");
  sparse_sqnorm_kernel<<<kSparseGrid, 256, 0, as_stream(stream)>>>(g, list, count, D, scale, ws);
  RS_CHECK_LAUNCH("rs_sparse_sqnorm");
  return 0;
}

extern "C" int64_t rs_sparse_compact_ws_bytes(int64_t V) {
  return (int64_t)(cdiv(V, kCompactChunk) + 1) * sizeof(int);
}

extern "C" int rs_sparse_compact(const int* flag, int64_t V, int* list, int* count, int* ws,
                                 void* stream) {
  RS_CHECK_ARG(flag && list && count && ws && V >= 1 && V < (int64_t)1 << 31,
               "rs_sparse_compact: bad args");
  hipStream_t st = as_stream(stream);
  const int nb = (int)cdiv(V, kCompactChunk);
  compact_count_kernel<<<nb, 256, 0, st>>>(flag, V, ws);
  RS_CHECK_LAUNCH("rs_sparse_compact count");
  compact_scan_kernel<<<1, 1024, 0, st>>>(ws, nb, count);
  RS_CHECK_LAUNCH("rs_sparse_compact scan");
  compact_write_kernel<<<nb, 256, 0, st>>>(flag, V, ws, list);
  RS_CHECK_LAUNCH("rs_sparse_compact write");
  return 0;
}

extern "C" int rs_sparse_pack(const float* g, const int* list, const int* count, int D, int cap,
                              float* buf, int* err_flag, void* stream) {
  RS_CHECK_ARG(g && list && count && buf && D >= 1 && cap >= 1, "rs_sparse_pack: bad args");
  hipStream_t st = as_stream(stream);
  if (err_flag) {
    overflow_kernel<<<1, 1, 0, st>>>(count, cap, err_flag);
    RS_CHECK_LAUNCH("rs_sparse_pack overflow");
  }
  pack_kernel<<<std::min(cdiv(cap, 4), 8192), 256, 0, st>>>(g, list, count, D, cap, buf);
  RS_CHECK_LAUNCH("rs_sparse_pack");
  return 0;
}

extern "C" int rs_sparse_unpack_add(float* g, int* flag, const float* buf, int D, int cap,
                                    void* stream) {
  RS_CHECK_ARG(g && flag && buf && D >= 1 && cap >= 1, "rs_sparse_unpack_add: bad args");
  unpack_add_kernel<<<std::min(cdiv(cap, 4), 8192), 256, 0, as_stream(stream)>>>(g, flag, buf, D,
                                                                                 cap);
  RS_CHECK_LAUNCH("rs_sparse_unpack_add");
  return 0;
}

extern "C" int rs_sparse_flush(float* p, float* m, float* v, int* last, int64_t V, int D,
                               const int64_t* step, const float* consts, float beta1, float beta2,
                               float eps, float weight_decay, void* stream) {
  RS_CHECK_ARG(p && m && v && last && step && consts && V >= 0 && D >= 1, "rs_sparse_flush: bad args");
  if (V == 0) return 0;
  int64_t blocks = (V + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  flush_kernel<<<(int)blocks, 256, 0, as_stream(stream)>>>(p, m, v, last, V, D, step,
                                                           reinterpret_cast<const float2*>(consts),
                                                           make_hyper(beta1, beta2, eps, weight_decay));
  RS_CHECK_LAUNCH("rs_sparse_flush");
  return 0;
}
