// Shared device/host helpers for librsys_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/rsys_hip.h"

namespace rs {

void set_error(const char* fmt, ...);

// Argument check: sets the thread-local message and returns -1 from the entry point.
#define RS_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      ::rs::set_error(__VA_ARGS__);    \
      return -1;                       \
    }                                  \
  } while (0)

// Launch-status check after a kernel launch.
#define RS_CHECK_LAUNCH(name)                                                       \
  do {                                                                              \
    hipError_t e__ = hipGetLastError();                                             \
    if (e__ != hipSuccess) {                                                        \
      ::rs::set_error("%s: launch failed: %s", name, hipGetErrorString(e__));       \
      return (int)e__;                                                              \
    }                                                                               \
  } while (0)

#define RS_RET_IF(x)        \
  do {                      \
    int r__ = (x);          \
    if (r__ != 0) return r__; \
  } while (0)

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// out[n] = beta*out[n] + scale * sum_{p<P} ws[p*N + n], fixed order (reduce.hip)
int partials_reduce(const float* ws, int P, int N, float scale, float beta, float* out,
                    hipStream_t st);
// the same with columns [0, split) -> out0 and [split, N) -> out1
int partials_reduce2(const float* ws, int P, int N, int split, float scale, float beta, float* out0,
                     float* out1, hipStream_t st);
// deferred reductions (reduce.hip): while deferring, reduce_defer_job queues a job for
// rs_reduce_flush instead of a launch; partials_reduce_any is partials_reduce(2) or a queued job
bool reduce_deferring();
void reduce_defer_job(const float* ws, int P, int N, int nr, float* const* outs, const int* begins,
                      const float* alphas, const float* betas);
int partials_reduce_any(const float* ws, int P, int N, int split, float scale, float beta, float* out0,
                        float* out1, hipStream_t st);
// two partials_reduce2 jobs of one shape (ws0 -> a0 | a1, ws1 -> b0 | b1) in one launch
int partials_reduce2x2(const float* ws0, const float* ws1, int P, int N, int split, float scale, float beta,
                       float* a0, float* a1, float* b0, float* b1, hipStream_t st);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
// debug / A-B switches read at launch time (host only): set and not "0"
inline bool getenv_flag(const char* name) {
  const char* v = getenv(name);
  return v && v[0] && !(v[0] == '0' && v[1] == 0);
}

// the same for a switch that defaults on: true iff set to exactly "0"
inline bool getenv_flag0(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '0' && v[1] == 0;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace rs
