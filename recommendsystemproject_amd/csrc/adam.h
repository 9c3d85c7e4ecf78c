// One Adam update of one element, shared by the dense optimizer kernel (optim.hip) and the
// lazy-table kernels (sparse.hip flush, lookup.hip catch-up / step), so that lazy and dense Adam
// round identically (bitwise equal; compile every user with fp contract(off)).
//
// torch.optim.Adam, single-tensor path (train_twotower.py:111 -> torch/optim/adam.py):
//   grad += wd * param;  exp_avg.lerp_(grad, 1 - b1);  exp_avg_sq = b2 * exp_avg_sq + (1 - b2) g^2
//   denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps;  param -= (lr / bc1) * exp_avg / denom
// Here 1 / sqrt(bc2) is a per-step constant and the square root and the reciprocal are the
// hardware v_sqrt_f32 / v_rcp_f32 (1 ulp) instead of the correctly rounded sequences: about 10
// VALU operations per element-step instead of ~50, which is what a lazy table's catch-up replays
// once per skipped step. The result differs from torch's by a few ulp per step (well inside the
// 1e-4 parity tolerance) and is identical between the dense and the lazy kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace rs {

struct AdamConst {
  float one_m_b1, b2, one_m_b2, eps, wd;
};

__device__ __forceinline__ void adam_update(const AdamConst& h, float step_size, float inv_bc2_sqrt,
                                            float gs, float& p, float& m, float& v) {
#pragma clang fp contract(off)  // no fma contraction whatever the including file says
  if (h.wd != 0.f) gs = gs + h.wd * p;
  m = m + h.one_m_b1 * (gs - m);
  v = v * h.b2 + h.one_m_b2 * gs * gs;
  const float denom = __builtin_amdgcn_sqrtf(v) * inv_bc2_sqrt + h.eps;
  p = p - step_size * (m * __builtin_amdgcn_rcpf(denom));
}

// Steps from .. to (inclusive) with zero gradient of W <= 4 elements (a lazy table's catch-up),
// bitwise equal to calling adam_update(h, consts[s].x, consts[s].y, 0.f, ...) per element and
// step: with gs = 0 and wd == 0, (1 - b2) * gs * gs is +0 and v * b2 + (+0) == v * b2 exactly
// (v >= 0), so that term is dropped; every other operation is the same IEEE operation in the same
// order. The elements run interleaved (independent chains), two at a time as packed pairs
// (v_pk_mul_f32 / v_pk_add_f32); an element whose moments are zero stays put exactly (m stays 0,
// the update is p - step * (0 * rcp(eps)) = p). wd != 0 takes adam_update itself.
// CF: the step constants' accessor, s -> consts[s] (a global table, or a window of it staged in
// LDS by the caller: the replay's one dependent load per step was the catch-up's latency chain)
template <int W, class CF>
__device__ __forceinline__ void adam_replay_zero(const AdamConst& h, CF cst, int from, int to, float* p, float* m,
                                                 float* v) {
#pragma clang fp contract(off)
  if (from > to) return;
  if (h.wd != 0.f) {
    for (int s = from; s <= to; ++s) {
      const float2 c = cst(s);
#pragma unroll
      for (int j = 0; j < W; ++j) adam_update(h, c.x, c.y, 0.f, p[j], m[j], v[j]);
    }
    return;
  }
  typedef float f2v __attribute__((ext_vector_type(2)));
  constexpr int NP = (W + 1) / 2;
  f2v pp[NP], mm[NP], vv[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    pp[q] = f2v{p[2 * q], 2 * q + 1 < W ? p[2 * q + 1] : 0.f};
    mm[q] = f2v{m[2 * q], 2 * q + 1 < W ? m[2 * q + 1] : 0.f};
    vv[q] = f2v{v[2 * q], 2 * q + 1 < W ? v[2 * q + 1] : 0.f};
  }
  const f2v omb1 = f2v{h.one_m_b1, h.one_m_b1}, b2 = f2v{h.b2, h.b2}, eps = f2v{h.eps, h.eps};
  const f2v zero = f2v{0.f, 0.f};
  for (int s = from; s <= to; ++s) {
    const float2 c = cst(s);
    const f2v ss = f2v{c.x, c.x}, ib = f2v{c.y, c.y};
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      mm[q] = mm[q] + omb1 * (zero - mm[q]);
      vv[q] = vv[q] * b2;
      f2v d = f2v{__builtin_amdgcn_sqrtf(vv[q][0]), __builtin_amdgcn_sqrtf(vv[q][1])};
      d = d * ib + eps;
      const f2v r = f2v{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
      pp[q] = pp[q] - ss * (mm[q] * r);
    }
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    p[2 * q] = pp[q][0]; m[2 * q] = mm[q][0]; v[2 * q] = vv[q][0];
    if (2 * q + 1 < W) { p[2 * q + 1] = pp[q][1]; m[2 * q + 1] = mm[q][1]; v[2 * q + 1] = vv[q][1]; }
  }
}

// The moments alone over zero-gradient steps from .. to (weight_decay == 0 only: then m and v do
// not depend on p): the same m and v bits adam_replay_zero leaves. A lazy table whose forward
// catch-up wrote p alone (its p is current to a later step than its moments, `last` [.., 1] vs
// [.., 0]) brings the moments up to p's step with this before replaying on.
template <int W>
__device__ __forceinline__ void adam_replay_mv(const AdamConst& h, int from, int to, float* m, float* v) {
#pragma clang fp contract(off)
  typedef float f2v __attribute__((ext_vector_type(2)));
  constexpr int NP = (W + 1) / 2;
  f2v mm[NP], vv[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    mm[q] = f2v{m[2 * q], 2 * q + 1 < W ? m[2 * q + 1] : 0.f};
    vv[q] = f2v{v[2 * q], 2 * q + 1 < W ? v[2 * q + 1] : 0.f};
  }
  const f2v omb1 = f2v{h.one_m_b1, h.one_m_b1}, b2 = f2v{h.b2, h.b2}, zero = f2v{0.f, 0.f};
  for (int s = from; s <= to; ++s) {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      mm[q] = mm[q] + omb1 * (zero - mm[q]);
      vv[q] = vv[q] * b2;
    }
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    m[2 * q] = mm[q][0]; v[2 * q] = vv[q][0];
    if (2 * q + 1 < W) { m[2 * q + 1] = mm[q][1]; v[2 * q + 1] = vv[q][1]; }
  }
}

// A lazy row's catch-up from its state -- moments at step lm, parameters at step lp >= lm (equal
// when weight_decay != 0) -- to step `to`: the moments alone to lp, then full zero-gradient steps.
template <int W, class CF>
__device__ __forceinline__ void adam_catch_row_f(const AdamConst& h, CF cst, int lm, int lp, int to, float* p,
                                                 float* m, float* v) {
  if (lp > lm) adam_replay_mv<W>(h, lm + 1, lp < to ? lp : to, m, v);
  adam_replay_zero<W>(h, cst, (lp > lm ? lp : lm) + 1, to, p, m, v);
}

template <int W>
__device__ __forceinline__ void adam_catch_row(const AdamConst& h, const float2* __restrict__ consts, int lm, int lp,
                                               int to, float* p, float* m, float* v) {
  adam_catch_row_f<W>(h, [consts](int s) { return consts[s]; }, lm, lp, to, p, m, v);
}

// The last kConstWin steps' constants staged in LDS by every workgroup of a row kernel (steps
// t - kConstWin + 1 .. t; older steps read the global table): one load round trip per workgroup
// instead of one per replayed step and row
constexpr int kConstWin = 64;
struct ConstWin {
  const float2* g;
  const float2* w;  // LDS window
  int lo;           // step of w[0]
  __device__ __forceinline__ float2 operator()(int s) const { return s >= lo ? w[s - lo] : g[s]; }
};

// per-step constants {lr / bc1(t), 1 / sqrt(bc2(t))}, computed in double then rounded once
__host__ __device__ inline void adam_step_consts(double lr, double b1, double b2, double t,
                                                 float* step_size, float* inv_bc2_sqrt) {
  const double bc1 = 1.0 - pow(b1, t), bc2 = 1.0 - pow(b2, t);
  *step_size = (float)(lr / bc1);
  *inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
}

}  // namespace rs
