// Deterministic column / full reductions (bias gradients, positional-embedding gradients,
// LayerNorm gamma/beta gradients, mean loss). Two passes with a fixed summation order so that
// repeated runs are bitwise identical (no float atomics).
#include <algorithm>
#include <vector>

#include "common.h"

namespace rs {

// Partial-sum geometry: a chunk of rows per workgroup; 64 columns x 4 row lanes per workgroup.
int colsum_chunks(int M) {
  int s = cdiv(M, 128);
  if (s > 1024) s = 1024;
  if (s < 1) s = 1;
  return s;
}

// out[n] = beta*out[n] + scale * sum_p ws[p*N + n] — 64 columns x 16 lanes per workgroup, each
// lane sums every 16th partial with 8 loads in flight, then a fixed-order LDS tree: bitwise
// reproducible and not latency-bound for thousands of partials.
__global__ __launch_bounds__(1024) void partials_reduce_kernel(const float* __restrict__ ws, int P,
                                                               int N, float scale, float beta,
                                                               float* __restrict__ out,
                                                               float* __restrict__ out1 = nullptr,
                                                               int split = 1 << 30) {
  __shared__ float red[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int l = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < N) {
    int p = l;
    for (; p + 16 * 7 < P; p += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws[(int64_t)(p + 16 * u) * N + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; p < P; p += 16) acc += ws[(int64_t)p * N + c];
  }
  red[l][threadIdx.x & 63] = acc;
  __syncthreads();
  if (l == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
    float* o = c < split ? out + c : out1 + (c - split);
    *o = (beta != 0.f ? beta * *o : 0.f) + scale * t;
  }
}

// Two independent partials_reduce2 jobs in one launch (blockIdx.y picks the job): the fused FFN
// backward's LayerNorm 1 and LayerNorm 2 gamma / beta gradients (round 5: one launch less on the
// C2 backward's critical path, ~4.7 us each)
struct ReduceJob {
  const float* ws;
  int P, N, split;
  float scale, beta;
  float* out0;
  float* out1;
};

__global__ __launch_bounds__(1024) void partials_reduce_jobs_kernel(ReduceJob j0, ReduceJob j1) {
  const ReduceJob& j = blockIdx.y == 0 ? j0 : j1;
  __shared__ float red[16][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if ((int)blockIdx.x * 64 >= j.N) return;  // whole workgroup
  const int l = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < j.N) {
    int p = l;
    for (; p + 16 * 7 < j.P; p += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = j.ws[(int64_t)(p + 16 * u) * j.N + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; p < j.P; p += 16) acc += j.ws[(int64_t)p * j.N + c];
  }
  red[l][threadIdx.x & 63] = acc;
  __syncthreads();
  if (l == 0 && c < j.N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
    float* o = c < j.split ? j.out0 + c : j.out1 + (c - j.split);
    *o = (j.beta != 0.f ? j.beta * *o : 0.f) + j.scale * t;
  }
}

int partials_reduce_any(const float* ws, int P, int N, int split, float scale, float beta, float* out0,
                        float* out1, hipStream_t st);

int partials_reduce2x2(const float* ws0, const float* ws1, int P, int N, int split, float scale, float beta,
                       float* a0, float* a1, float* b0, float* b1, hipStream_t st) {
  if (reduce_deferring()) {
    partials_reduce_any(ws0, P, N, split, scale, beta, a0, a1, st);
    return partials_reduce_any(ws1, P, N, split, scale, beta, b0, b1, st);
  }
  const ReduceJob j0{ws0, P, N, split, scale, beta, a0, a1}, j1{ws1, P, N, split, scale, beta, b0, b1};
  partials_reduce_jobs_kernel<<<dim3(cdiv(N, 64), 2), 1024, 0, st>>>(j0, j1);
  RS_CHECK_LAUNCH("partials_reduce2x2");
  return 0;
}

int partials_reduce(const float* ws, int P, int N, float scale, float beta, float* out,
                    hipStream_t st) {
  partials_reduce_kernel<<<cdiv(N, 64), 1024, 0, st>>>(ws, P, N, scale, beta, out);
  RS_CHECK_LAUNCH("partials_reduce");
  return 0;
}

// columns [0, split) -> out0, [split, N) -> out1 (two parameter gradients, one launch)
int partials_reduce2(const float* ws, int P, int N, int split, float scale, float beta, float* out0,
                     float* out1, hipStream_t st) {
  partials_reduce_kernel<<<cdiv(N, 64), 1024, 0, st>>>(ws, P, N, scale, beta, out0, out1, split);
  RS_CHECK_LAUNCH("partials_reduce2");
  return 0;
}

// ---------------------------------------------------------------- deferred reductions (round 5)
// A backward's parameter-gradient reductions (the weight gradients' split partials, the fused FFN
// weight gradient's, the LayerNorm gamma / beta and positional-embedding partials) are only read
// by the optimizer. Between rs_reduce_defer(1) and rs_reduce_flush the library queues them as jobs
// instead of launching one small reduce kernel each (~4.5 us of launch floor apiece, nine of them
// on the C2 backward's critical path), and the flush runs every queued job in ONE launch. Each job
// sums its partials exactly as partials_reduce_kernel does (16 strided lanes with 8 loads in
// flight, then the fixed 16-way LDS order) and writes out = beta * out + alpha * sum per column
// range, so the deferred and the immediate paths give the same bits. The caller keeps every
// partials buffer alive until the flush is queued (ops.deferred_reduce).
namespace {

constexpr int kJobRanges = 4;
constexpr int kMaxJobs = 24;

struct JobRange {
  float* out;
  int begin;  // first column of this range (ranges ascending, the first at 0)
  float alpha, beta;
};

struct RedJob {
  const float* ws;  // [P][N]
  int P, N, nr, blk0;
  JobRange r[kJobRanges];
};

struct RedJobs {
  RedJob j[kMaxJobs];
  int n;
};

// per job: columns in blocks of 256 (64 lanes x 4 columns, 16-byte loads) when N % 4 == 0, else
// 64 scalar columns; wave w of the 16 sums partials w, w + 16, ... of its lane's columns with 8
// loads in flight, then lanes' sums meet in the fixed 16-way LDS order -- per column exactly the
// operations of partials_reduce_kernel (whose lane group w sums the same partials in the same order)
__host__ __device__ __forceinline__ bool job_vec(const RedJob& j) {
  return (j.N & 3) == 0 && (reinterpret_cast<uintptr_t>(j.ws) & 15) == 0;
}
__device__ __forceinline__ int job_cols(const RedJob& j) { return job_vec(j) ? 256 : 64; }

__device__ __forceinline__ void job_out(const RedJob& j, int c, float t) {
  int q = 0;
  while (q + 1 < j.nr && c >= j.r[q + 1].begin) ++q;
  float* o = j.r[q].out + (c - j.r[q].begin);
  // beta * out + alpha * sum (the partials_reduce / ffn_wgrad_reduce form), alpha * sum when
  // beta == 0 (wgrad_reduce's: no read, and a -0 stays -0)
  *o = j.r[q].beta != 0.f ? j.r[q].beta * *o + j.r[q].alpha * t : j.r[q].alpha * t;
}

__global__ __launch_bounds__(1024) void reduce_jobs_kernel(RedJobs js) {
  int k = 0;
  while (k + 1 < js.n && (int)blockIdx.x >= js.j[k + 1].blk0) ++k;
  const RedJob& j = js.j[k];
  __shared__ float4 red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (job_cols(j) == 256) {
    const int c4 = ((int)blockIdx.x - j.blk0) * 64 + lane;  // float4 column index
    const int n4 = j.N / 4;
    const float4* src = reinterpret_cast<const float4*>(j.ws);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < n4) {
      int p = w;
      for (; p + 16 * 7 < j.P; p += 16 * 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(p + 16 * u) * n4 + c4];
#pragma unroll
        for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
      }
      for (; p < j.P; p += 16) {
        const float4 v = src[(int64_t)p * n4 + c4];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0 && c4 < n4) {
      float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < 16; ++i) { const float4 r = red[i][lane]; t.x += r.x; t.y += r.y; t.z += r.z; t.w += r.w; }
      job_out(j, 4 * c4, t.x);
      job_out(j, 4 * c4 + 1, t.y);
      job_out(j, 4 * c4 + 2, t.z);
      job_out(j, 4 * c4 + 3, t.w);
    }
    return;
  }
  const int c = ((int)blockIdx.x - j.blk0) * 64 + lane;
  float acc = 0.f;
  if (c < j.N) {
    int p = w;
    for (; p + 16 * 7 < j.P; p += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = j.ws[(int64_t)(p + 16 * u) * j.N + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; p < j.P; p += 16) acc += j.ws[(int64_t)p * j.N + c];
  }
  reinterpret_cast<float*>(&red[w][0])[lane] = acc;
  __syncthreads();
  if (w == 0 && c < j.N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += reinterpret_cast<const float*>(&red[i][0])[lane];
    job_out(j, c, t);
  }
}

// Per host thread: a deferred_reduce scope (ops.py) is opened and flushed on the thread that runs
// the encoder's backward (an autograd device thread), and only that thread's reductions queue
// into it; a call from any other thread (another device's autograd worker) launches as usual.
thread_local bool g_defer = false;
thread_local std::vector<RedJob> g_jobs;

int launch_jobs(const RedJob* jobs, int n, hipStream_t st) {
  for (int a = 0; a < n; a += kMaxJobs) {
    RedJobs js{};
    js.n = std::min(kMaxJobs, n - a);
    int blk = 0;
    for (int i = 0; i < js.n; ++i) {
      js.j[i] = jobs[a + i];
      js.j[i].blk0 = blk;
      blk += cdiv(js.j[i].N, job_vec(js.j[i]) ? 256 : 64);
    }
    if (blk == 0) continue;
    reduce_jobs_kernel<<<blk, 1024, 0, st>>>(js);
    RS_CHECK_LAUNCH("rs_reduce_flush");
  }
  return 0;
}

}  // namespace

bool reduce_deferring() { return g_defer; }

// queue a job (deferring) -- the caller launches its own kernel otherwise; outs: up to 4 column
// ranges {out, begin, alpha, beta}
void reduce_defer_job(const float* ws, int P, int N, int nr, float* const* outs, const int* begins,
                      const float* alphas, const float* betas) {
  RedJob j{};
  j.ws = ws; j.P = P; j.N = N; j.nr = nr;
  for (int i = 0; i < nr; ++i) j.r[i] = JobRange{outs[i], begins[i], alphas[i], betas[i]};
  g_jobs.push_back(j);
}

}  // namespace rs

extern "C" int rs_reduce_defer(int on) {
  rs::g_defer = on != 0;
  return 0;
}

extern "C" int rs_reduce_flush(void* stream) {
  std::vector<rs::RedJob> jobs;
  jobs.swap(rs::g_jobs);
  if (jobs.empty()) return 0;
  // the long jobs' workgroups (most partials each) dispatched first, the short ones fill the tail
  // (each job's sums are independent of where it sits in the grid)
  std::stable_sort(jobs.begin(), jobs.end(), [](const rs::RedJob& x, const rs::RedJob& y) { return x.P > y.P; });
  return rs::launch_jobs(jobs.data(), (int)jobs.size(), rs::as_stream(stream));
}

namespace rs {

int partials_reduce_any(const float* ws, int P, int N, int split, float scale, float beta, float* out0,
                        float* out1, hipStream_t st) {
  if (g_defer) {
    float* outs[2] = {out0, out1};
    const int begins[2] = {0, split};
    const float al[2] = {scale, scale}, be[2] = {beta, beta};
    reduce_defer_job(ws, P, N, out1 && split < N ? 2 : 1, outs, begins, al, be);
    return 0;
  }
  return out1 && split < N ? partials_reduce2(ws, P, N, split, scale, beta, out0, out1, st)
                           : partials_reduce(ws, P, N, scale, beta, out0, st);
}

namespace {

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ X, int M,
                                                             int N, int ldx, int rows_per_chunk,
                                                             float* __restrict__ ws) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int r0 = s * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  float acc = 0.f;
  if (c < N) {
    int m = r0 + rl;
    for (; m + 4 * 7 < r1; m += 4 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = X[(int64_t)(m + 4 * u) * ldx + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; m < r1; m += 4) acc += X[(int64_t)m * ldx + c];
  }
  red[rl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rl == 0 && c < N)
    ws[(int64_t)s * N + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                             red[3][threadIdx.x];
}

__global__ __launch_bounds__(1024) void sum_kernel(const float* __restrict__ x, int n, float scale,
                                                   float* __restrict__ out) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += red[i];
    *out = (float)(t * (double)scale);
  }
}

}  // namespace

int colsum_launch(const float* X, int M, int N, int ldx, float scale, float beta, float* out,
                  float* ws, hipStream_t st) {
  const int S = colsum_chunks(M);
  const int rpc = cdiv(M, S);
  colsum_partial_kernel<<<dim3(cdiv(N, 64), S), 256, 0, st>>>(X, M, N, ldx, rpc, ws);
  RS_CHECK_LAUNCH("colsum partial");
  return partials_reduce(ws, S, N, scale, beta, out, st);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_colsum_ws_bytes(int M, int N) {
  return (int64_t)colsum_chunks(M) * N * (int64_t)sizeof(float);
}

extern "C" int rs_colsum(const float* X, int M, int N, int ldx, float scale, float beta,
                         float* out, float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && N >= 0 && ldx >= N, "rs_colsum: bad shape M=%d N=%d ldx=%d", M, N, ldx);
  if (N == 0) return 0;
  RS_CHECK_ARG(X && out && ws, "rs_colsum: null pointer");
  if (M == 0) M = 0;
  return colsum_launch(X, M, N, ldx, scale, beta, out, ws, as_stream(stream));
}

extern "C" int rs_sum(const float* x, int n, float scale, float* out, void* stream) {
  RS_CHECK_ARG(n >= 0 && x && out, "rs_sum: bad args");
  sum_kernel<<<1, 1024, 0, as_stream(stream)>>>(x, n, scale, out);
  RS_CHECK_LAUNCH("rs_sum");
  return 0;
}

// NaN guard of the loss inputs (TwoTowerModel.py:88-91 raises on NaN user/item/hard-negative
// embeddings): flag |= bit when x[0..n) holds a NaN. No sync: the host reads the flag at its
// existing log-point sync (training_utils.train_one_epoch) and raises there.
namespace rs {
namespace {
__global__ __launch_bounds__(256) void nan_check_kernel(const float* __restrict__ x, int64_t n,
                                                        int* __restrict__ flag, int bit) {
  bool bad = false;
  const int64_t n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = x4[i];
    bad |= (v.x != v.x) | (v.y != v.y) | (v.z != v.z) | (v.w != v.w);
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    bad |= x[i] != x[i];
  if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(flag, bit);
}

// up to 4 tensors in one launch (the loss's U, I, H): workgroup b checks tensor i of block range
// [first[i], first[i + 1])
struct NanList {
  const float* x[4];
  int64_t n[4];
  int bit[4];
  int first[5];
  int k;
};

__global__ __launch_bounds__(256) void nan_check_many_kernel(NanList l, int* __restrict__ flag) {
  int i = 0;
  while (i + 1 < l.k && (int)blockIdx.x >= l.first[i + 1]) ++i;
  const int b = blockIdx.x - l.first[i], nb = l.first[i + 1] - l.first[i];
  const float* x = l.x[i];
  const int64_t n = l.n[i];
  bool bad = false;
  const int64_t n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (int64_t j = (int64_t)b * 256 + threadIdx.x; j < n4; j += (int64_t)nb * 256) {
    const float4 v = x4[j];
    bad |= (v.x != v.x) | (v.y != v.y) | (v.z != v.z) | (v.w != v.w);
  }
  for (int64_t j = n4 * 4 + (int64_t)b * 256 + threadIdx.x; j < n; j += (int64_t)nb * 256) bad |= x[j] != x[j];
  if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(flag, l.bit[i]);
}
}  // namespace
}  // namespace rs

extern "C" int rs_nan_check_many(int k, const float* const* x, const int64_t* n, const int* bits, int* flag,
                                 void* stream) {
  RS_CHECK_ARG(k >= 1 && k <= 4 && x && n && bits && flag, "rs_nan_check_many: bad args (k=%d)", k);
  rs::NanList l{};
  l.k = k;
  int wg = 0;
  for (int i = 0; i < k; ++i) {
    RS_CHECK_ARG(x[i] && n[i] >= 0 && rs::aligned16(x[i]), "rs_nan_check_many: tensor %d: bad args", i);
    l.x[i] = x[i];
    l.n[i] = n[i];
    l.bit[i] = bits[i];
    l.first[i] = wg;
    int blocks = rs::cdiv(n[i] / 4 + 1, 256);
    wg += blocks > 512 ? 512 : blocks;
  }
  l.first[k] = wg;
  rs::nan_check_many_kernel<<<wg, 256, 0, rs::as_stream(stream)>>>(l, flag);
  RS_CHECK_LAUNCH("rs_nan_check_many");
  return 0;
}

extern "C" int rs_nan_check(const float* x, int64_t n, int* flag, int bit, void* stream) {
  RS_CHECK_ARG(x && flag && n >= 0 && rs::aligned16(x), "rs_nan_check: bad args");
  if (n == 0) return 0;
  int blocks = rs::cdiv(n / 4 + 1, 256);
  if (blocks > 1024) blocks = 1024;
  rs::nan_check_kernel<<<blocks, 256, 0, rs::as_stream(stream)>>>(x, n, flag, bit);
  RS_CHECK_LAUNCH("rs_nan_check");
  return 0;
}
