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

// per-step constants {lr / bc1(t), 1 / sqrt(bc2(t))}, computed in double then rounded once
__host__ __device__ inline void adam_step_consts(double lr, double b1, double b2, double t,
                                                 float* step_size, float* inv_bc2_sqrt) {
  const double bc1 = 1.0 - pow(b1, t), bc2 = 1.0 - pow(b2, t);
  *step_size = (float)(lr / bc1);
  *inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
}

}  // namespace rs
