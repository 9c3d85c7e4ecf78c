// Lazy-exact Adam for large embedding tables (SURVEY.md §7.2 hard part 1, trap T16): the per-step
// constants and the whole-table flush. The per-row work of a step (catch-up before the gather,
// the Adam step, clip-norm partials) walks the step's sorted lookups (lookup.hip).
//
// The reference trains nn.Embedding with dense gradients, so torch.optim.Adam moves EVERY row of
// every table every step: a row whose exp_avg is non-zero keeps drifting after it was last
// looked up. At 10M-100M rows that is a 75-360 GB sweep per step. Here a large table keeps
// per-row `last` (the optimizer step the row was last brought to); a row is brought current
// (the skipped zero-gradient steps replayed, adam.h adam_replay_zero) before it is read, and rs_sparse_flush brings every
// row to step t (before state_dict / checkpoint). The replay runs the same fp32 operation
// sequence as the dense kernel (adam.h adam_update) with the same per-step constants
// (consts[s] = {lr/bc1(s), 1/sqrt(bc2(s))}, written once per step by rs_adam_prepare), so lazy and
// dense Adam are bitwise identical. With weight_decay == 0 a row whose exp_avg and exp_avg_sq are
// zero does not move, which is what makes skipping it exact.
#include "common.h"
#include "adam.h"

// no fma contraction: the dense and the lazy (sparse.hip) Adam must round identically
#pragma clang fp contract(off)

namespace rs {
namespace {

// consts[0] (step 0 never runs) holds {cap as int bits, overflow flag as int bits}: every reader
// clamps its step index to cap - 1, so a graph replayed past the capacity reads no memory past the
// table (the constants it then uses are stale: Adam.check_errors raises on the overflow flag)
__global__ void adam_prepare_kernel(int64_t* step, float2* consts, int cap, float lr, float b1,
                                    float b2) {
  const int64_t t = *step + 1;
  *step = t;
  if (t < cap) {
    float2 c;
    adam_step_consts((double)lr, (double)b1, (double)b2, (double)t, &c.x, &c.y);
    consts[t] = c;
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

__global__ void flush_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                             int* __restrict__ last, int64_t V, int D,
                             const int64_t* __restrict__ step, const float2* __restrict__ consts,
                             AdamConst h) {
  const int target = clamp_step(consts, *step);
  const int lane = threadIdx.x & 63;
  for (int64_t row = blockIdx.x * 4 + (threadIdx.x >> 6); row < V; row += (int64_t)gridDim.x * 4) {
    const int2 l2 = reinterpret_cast<const int2*>(last)[row];  // (moments' step, parameters' step)
    if (l2.x >= target) continue;
    for (int c = lane; c < D; c += 64) {
      const int64_t o = row * D + c;
      float pp = p[o], mm = m[o], vv = v[o];
      adam_catch_row<1>(h, consts, l2.x, l2.y, target, &pp, &mm, &vv);
      p[o] = pp; m[o] = mm; v[o] = vv;
    }
    if (lane == 0) reinterpret_cast<int2*>(last)[row] = make_int2(target, target);
  }
}

AdamConst make_hyper(float b1, float b2, float eps, float wd) {
  AdamConst h;
  h.one_m_b1 = 1.f - b1; h.b2 = b2; h.one_m_b2 = 1.f - b2; h.eps = eps; h.wd = wd;
  return h;
}

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
