// Gradient clipping and Adam over the flat parameter buffer (K18, K19).
// All parameters of a model live in ONE contiguous fp32 buffer (and grads / exp_avg /
// exp_avg_sq in three more), so clip_grad_norm_ is one streaming reduction and the optimizer
// step is one streaming kernel (28 B/param: read p, g, m, v; write p, m, v) regardless of how
// many tensors the model has. The clip coefficient stays on the device: no host sync.
#include "common.h"
#include "adam.h"

// no fma contraction: the dense and the lazy (sparse.hip) Adam must round identically
#pragma clang fp contract(off)

namespace rs {
namespace {

int sq_blocks(int64_t n) {
  int64_t b = (n + 256 * 16 - 1) / (256 * 16);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ g, int64_t n,
                                                     float scale, double* __restrict__ ws) {
  __shared__ double red[4];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t n4 = n / 4;
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == 0;
  if (vec) {
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      const float4 v = g4[i];
      const float a = v.x * scale, b = v.y * scale, c = v.z * scale, d = v.w * scale;
      acc += (double)(a * a) + (double)(b * b) + (double)(c * c) + (double)(d * d);
    }
    for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float a = g[i] * scale;
      acc += (double)(a * a);
    }
  } else {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float a = g[i] * scale;
      acc += (double)(a * a);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// rs_grad_sqnorm_clip_step: sqnorm_kernel's partials, and the last workgroup to finish turns them
// into the clip coefficient exactly as clip_coef_kernel does (its 1,024 threads' strided sums
// emulated as 4 per thread, the same wave trees, the same 16-way order: the same bits) and
// advances the step counter -- one launch instead of two on the optimizer's chain (round 5). The
// hand-off is fence-free (MI355X_MICROARCH.md): each workgroup's partial store is drained
// (vmcnt(0)) before its agent-scope ticket; the last one reads the partials with agent-scope loads
// and re-arms the ticket.
__global__ __launch_bounds__(256) void sqnorm_clip_kernel(const float* __restrict__ g, int64_t n, float scale,
                                                          double* __restrict__ ws, int* __restrict__ ticket,
                                                          float max_norm, float* total_norm, float* coef,
                                                          int64_t* counter) {
  __shared__ double red[16];
  __shared__ int s_last;
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t n4 = n / 4;
  const bool vec = (reinterpret_cast<uintptr_t>(g) & 15) == 0;
  if (vec) {
    const float4* g4 = reinterpret_cast<const float4*>(g);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      const float4 v = g4[i];
      const float a = v.x * scale, b = v.y * scale, c = v.z * scale, d = v.w * scale;
      acc += (double)(a * a) + (double)(b * b) + (double)(c * c) + (double)(d * d);
    }
    for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float a = g[i] * scale;
      acc += (double)(a * a);
    }
  } else {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
      const float a = g[i] * scale;
      acc += (double)(a * a);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(ws + blockIdx.x, red[0] + red[1] + red[2] + red[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  const int nb = gridDim.x;
  double t[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // virtual thread threadIdx.x + 256 q of clip_coef_kernel
    t[q] = 0.0;
    for (int i = threadIdx.x + 256 * q; i < nb; i += 1024)
      t[q] += __hip_atomic_load(ws + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();  // red reused
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double v = wave_sum(t[q]);
    if ((threadIdx.x & 63) == 0) red[4 * q + (threadIdx.x >> 6)] = v;  // virtual wave 4 q + wave
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double tt = 0.0;
  for (int w = 0; w < 16; ++w) tt += red[w];
  const float norm = (float)sqrt(tt);
  if (total_norm) *total_norm = norm;
  float c = max_norm / (norm + 1e-6f);
  *coef = c < 1.f ? c : 1.f;
  if (counter) *counter += 1;
  *ticket = 0;
}

// fixed-order (deterministic) sum of nb partials: strided per-thread sums, then a fixed tree
__global__ __launch_bounds__(1024) void clip_coef_kernel(const double* __restrict__ ws, int nb,
                                                         float max_norm, float* total_norm,
                                                         float* coef, int64_t* counter) {
  __shared__ double red[16];
  double t = 0.0;
  for (int i = threadIdx.x; i < nb; i += 1024) t += ws[i];
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x != 0) return;
  t = 0.0;
  for (int w = 0; w < 16; ++w) t += red[w];
  const float norm = (float)sqrt(t);
  if (total_norm) *total_norm = norm;
  float c = max_norm / (norm + 1e-6f);
  *coef = c < 1.f ? c : 1.f;
  if (counter) *counter += 1;  // the optimizer's step count (rs_clip_coef_step): one launch less
}

// rs_clip_coef_prepare: the clip coefficient and, in the same launch, the lazy tables' Adam step
// constants for the next step (sparse.hip adam_prepare_kernel's body, the same values)
__global__ __launch_bounds__(1024) void clip_coef_prepare_kernel(const double* __restrict__ ws, int nb,
                                                                 float max_norm, float* total_norm, float* coef,
                                                                 int64_t* step, float2* consts, int cap, float lr,
                                                                 float b1, float b2) {
  __shared__ double red[16];
  double t = 0.0;
  for (int i = threadIdx.x; i < nb; i += 1024) t += ws[i];
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x != 0) return;
  t = 0.0;
  for (int w = 0; w < 16; ++w) t += red[w];
  const float norm = (float)sqrt(t);
  if (total_norm) *total_norm = norm;
  float c = max_norm / (norm + 1e-6f);
  *coef = c < 1.f ? c : 1.f;
  const int64_t s = *step + 1;
  *step = s;
  if (s < cap) {
    float2 k;
    adam_step_consts((double)lr, (double)b1, (double)b2, (double)s, &k.x, &k.y);
    consts[s] = k;
    if (s == 1) consts[0] = make_float2(__int_as_float(cap), __int_as_float(0));
  } else {
    consts[0] = make_float2(__int_as_float(cap), __int_as_float(1));
  }
}

__global__ void scale_kernel(float* __restrict__ g, int64_t n, float scale,
                             const float* __restrict__ coef) {
  const float s = scale * (coef ? *coef : 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    g[i] *= s;
}

struct AdamArgs {
  float* p; float* g; float* m; float* v;
  int64_t n;
  float lr, step_size, b1, b2, eps, wd, inv_bc2_sqrt, scale;
  AdamConst h;
  const float* coef;
  const int64_t* step_dev;  // when set, bias corrections come from *step_dev (graph replay)
  int write_grad;
};

__device__ __forceinline__ void adam_elem(const AdamArgs& a, float s, float& p, float& g, float& m,
                                          float& v) {
  const float gs = g * s;
  if (a.write_grad) g = gs;
  adam_update(a.h, a.step_size, a.inv_bc2_sqrt, gs, p, m, v);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const float s = a.scale * (a.coef ? *a.coef : 1.f);
  if (a.step_dev)
    adam_step_consts((double)a.lr, (double)a.b1, (double)a.b2, (double)*a.step_dev, &a.step_size,
                     &a.inv_bc2_sqrt);
  const int64_t stride = (int64_t)gridDim.x * 256;
  const bool vec = ((reinterpret_cast<uintptr_t>(a.p) | reinterpret_cast<uintptr_t>(a.g) |
                     reinterpret_cast<uintptr_t>(a.m) | reinterpret_cast<uintptr_t>(a.v)) & 15) == 0;
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = a.n / 4;
    float4* p4 = reinterpret_cast<float4*>(a.p);
    float4* g4 = reinterpret_cast<float4*>(a.g);
    float4* m4 = reinterpret_cast<float4*>(a.m);
    float4* v4 = reinterpret_cast<float4*>(a.v);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      float4 p = p4[i], g = g4[i], m = m4[i], v = v4[i];
      adam_elem(a, s, p.x, g.x, m.x, v.x);
      adam_elem(a, s, p.y, g.y, m.y, v.y);
      adam_elem(a, s, p.z, g.z, m.z, v.z);
      adam_elem(a, s, p.w, g.w, m.w, v.w);
      p4[i] = p; m4[i] = m; v4[i] = v;
      if (a.write_grad) g4[i] = g;
    }
    done = n4 * 4;
  }
  for (int64_t i = done + blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
    float p = a.p[i], g = a.g[i], m = a.m[i], v = a.v[i];
    adam_elem(a, s, p, g, m, v);
    a.p[i] = p; a.m[i] = m; a.v[i] = v;
    if (a.write_grad) a.g[i] = g;
  }
}

__global__ void counter_add_kernel(int64_t* c, int64_t delta) { *c += delta; }

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int64_t rs_sqnorm_ws_bytes(int64_t n) { return (int64_t)sq_blocks(n) * sizeof(double); }

extern "C" int rs_grad_sqnorm(const float* g, int64_t n, float scale, double* ws, void* stream) {
  RS_CHECK_ARG(g && ws && n >= 0, "rs_grad_sqnorm: bad args");
  sqnorm_kernel<<<sq_blocks(n), 256, 0, as_stream(stream)>>>(g, n, scale, ws);
  RS_CHECK_LAUNCH("rs_grad_sqnorm");
  return 0;
}

extern "C" int rs_sqnorm_parts(int64_t n) { return sq_blocks(n); }

extern "C" int rs_grad_sqnorm_clip_step(const float* g, int64_t n, float scale, double* ws, int* ticket,
                                        float max_norm, float* total_norm, float* coef, int64_t* counter,
                                        void* stream) {
  RS_CHECK_ARG(g && ws && ticket && coef && n >= 0, "rs_grad_sqnorm_clip_step: bad args");
  sqnorm_clip_kernel<<<sq_blocks(n), 256, 0, as_stream(stream)>>>(g, n, scale, ws, ticket, max_norm, total_norm,
                                                                  coef, counter);
  RS_CHECK_LAUNCH("rs_grad_sqnorm_clip_step");
  return 0;
}

extern "C" int rs_clip_coef(const double* ws, int nparts, float max_norm, float* total_norm,
                            float* coef, void* stream) {
  RS_CHECK_ARG(ws && coef && nparts >= 1, "rs_clip_coef: bad args");
  clip_coef_kernel<<<1, 1024, 0, as_stream(stream)>>>(ws, nparts, max_norm, total_norm, coef, nullptr);
  RS_CHECK_LAUNCH("rs_clip_coef");
  return 0;
}

extern "C" int rs_clip_coef_step(const double* ws, int nparts, float max_norm, float* total_norm,
                                 float* coef, int64_t* counter, void* stream) {
  RS_CHECK_ARG(ws && coef && counter && nparts >= 1, "rs_clip_coef_step: bad args");
  clip_coef_kernel<<<1, 1024, 0, as_stream(stream)>>>(ws, nparts, max_norm, total_norm, coef, counter);
  RS_CHECK_LAUNCH("rs_clip_coef_step");
  return 0;
}

extern "C" int rs_clip_coef_prepare(const double* ws, int nparts, float max_norm, float* total_norm, float* coef,
                                    int64_t* step, float* consts, int cap, float lr, float beta1, float beta2,
                                    void* stream) {
  RS_CHECK_ARG(ws && coef && step && consts && nparts >= 1 && cap >= 2, "rs_clip_coef_prepare: bad args");
  clip_coef_prepare_kernel<<<1, 1024, 0, as_stream(stream)>>>(ws, nparts, max_norm, total_norm, coef, step,
                                                              reinterpret_cast<float2*>(consts), cap, lr, beta1,
                                                              beta2);
  RS_CHECK_LAUNCH("rs_clip_coef_prepare");
  return 0;
}

extern "C" int rs_scale_inplace(float* g, int64_t n, float scale, const float* coef, void* stream) {
  RS_CHECK_ARG(g && n >= 0, "rs_scale_inplace: bad args");
  if (n == 0) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  scale_kernel<<<(int)blocks, 256, 0, as_stream(stream)>>>(g, n, scale, coef);
  RS_CHECK_LAUNCH("rs_scale_inplace");
  return 0;
}

__global__ void prof_marker_kernel(int tag) {
  // empty on purpose: only its dispatch record matters (bench.py --pmc-bracket)
  if (tag == -0x7fffffff) __builtin_trap();
}

extern "C" int rs_prof_marker(int tag, void* stream) {
  prof_marker_kernel<<<1, 1, 0, as_stream(stream)>>>(tag);
  RS_CHECK_LAUNCH("rs_prof_marker");
  return 0;
}

extern "C" int rs_counter_add(int64_t* counter, int64_t delta, void* stream) {
  RS_CHECK_ARG(counter, "rs_counter_add: null pointer");
  counter_add_kernel<<<1, 1, 0, as_stream(stream)>>>(counter, delta);
  RS_CHECK_LAUNCH("rs_counter_add");
  return 0;
}

extern "C" int rs_adam_step(float* p, float* g, float* m, float* v, int64_t n, float lr,
                            float beta1, float beta2, float eps, float weight_decay, int step,
                            const int64_t* step_dev, float scale, const float* coef, int write_grad,
                            void* stream) {
  RS_CHECK_ARG(p && g && m && v && n >= 0 && (step >= 1 || step_dev), "rs_adam_step: bad args");
  if (n == 0) return 0;
  AdamArgs a;
  a.p = p; a.g = g; a.m = m; a.v = v; a.n = n;
  const double t = step >= 1 ? (double)step : 1.0;
  a.lr = lr;
  a.step_dev = step_dev;
  adam_step_consts((double)lr, (double)beta1, (double)beta2, t, &a.step_size, &a.inv_bc2_sqrt);
  a.b1 = beta1; a.b2 = beta2;
  a.h.one_m_b1 = 1.f - beta1; a.h.b2 = beta2; a.h.one_m_b2 = 1.f - beta2; a.h.eps = eps;
  a.h.wd = weight_decay;
  a.eps = eps; a.wd = weight_decay; a.scale = scale; a.coef = coef; a.write_grad = write_grad;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  adam_kernel<<<(int)blocks, 256, 0, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_adam_step");
  return 0;
}
