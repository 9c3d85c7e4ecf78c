// Normalisation kernels of the training step.
//  * add + LayerNorm (post-LN residual of nn.TransformerEncoderLayer, K8): one wave per row,
//    the row lives in registers (d = 64 -> one float per lane), wave-shuffle reductions.
//  * BatchNorm1d in training mode (feature_bn and the MLP BNs, K12/K13): batch statistics
//    need the whole column, so the forward is partial column sums (fp64) -> per-column finalise
//    (mean, rstd, running-stat update in group order) -> normalise (+ fused ReLU). G row groups
//    keep independent statistics (one item-tower pass per hard-negative slot, trap T13).
//  * row L2 normalisation (F.normalize, K14).
#include "common.h"
#include "rng.h"

namespace rs {
namespace {

// ------------------------------------------------------------------------------ LayerNorm
template <int NPL, bool DROP>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(float* __restrict__ a,
                                                         const float* __restrict__ b,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         float* __restrict__ y,
                                                         float* __restrict__ mean,
                                                         float* __restrict__ rstd, int M, int N,
                                                         float eps, float pdrop,
                                                         const int64_t* __restrict__ key,
                                                         int site) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  float h[NPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    h[i] = 0.f;
    if (c < N) {
      const int64_t o = (int64_t)row * N + c;
      const float av = DROP ? a[o] * keep_mult(dk, (uint64_t)o) : a[o];  // x + dropout(sublayer)
      h[i] = av + b[o];
      a[o] = h[i];
    }
    s += h[i];
  }
  const float mu = wave_sum(s) / (float)N;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    const float t = c < N ? h[i] - mu : 0.f;
    v += t * t;
  }
  const float var = wave_sum(v) / (float)N;
  const float rs_ = 1.f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    if (c < N) y[(int64_t)row * N + c] = (h[i] - mu) * rs_ * gamma[c] + beta[c];
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs_; }
}

// LN backward: each wave owns groups of R = 4 rows (4x the loads in flight of a row-per-wave
// loop), a grid-strided sweep over the rows, per-lane dgamma/dbeta partials in registers, one
// fixed-order partial per workgroup -> partials_reduce (deterministic).
template <int NPL, bool DROP>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ h,
                                                     const float* dy,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, float* dh,
                                                     int M, int N, float* __restrict__ ws,
                                                     float* __restrict__ da, float pdrop,
                                                     const int64_t* __restrict__ key, int site) {
  constexpr int R = 4;
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  __shared__ float red[2][4][NPL * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gm[NPL], pg[NPL], pb[NPL];
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    gm[i] = c < N ? gamma[c] : 0.f;
    pg[i] = 0.f;
    pb[i] = 0.f;
  }
  const int waves = gridDim.x * 4;
  for (int base = (blockIdx.x * 4 + wave) * R; base < M; base += waves * R) {
    float xh[R][NPL], g[R][NPL], s1[R], s2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = base + r;
      const bool ok = row < M;
      const float mu = ok ? mean[row] : 0.f, rr = ok ? rstd[row] : 0.f;
      s1[r] = 0.f;
      s2[r] = 0.f;
#pragma unroll
      for (int i = 0; i < NPL; ++i) {
        const int c = lane + i * 64;
        float hv = 0.f, d = 0.f;
        if (ok && c < N) {
          const int64_t o = (int64_t)row * N + c;
          hv = h[o];
          d = dy[o];
        }
        xh[r][i] = (hv - mu) * rr;
        pg[i] += d * xh[r][i];
        pb[i] += d;
        g[r][i] = d * gm[i];
        s1[r] += g[r][i];
        s2[r] += g[r][i] * xh[r][i];
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      s1[r] = wave_sum(s1[r]) / (float)N;
      s2[r] = wave_sum(s2[r]) / (float)N;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = base + r;
      if (row >= M) break;
      const float rr = rstd[row];
#pragma unroll
      for (int i = 0; i < NPL; ++i) {
        const int c = lane + i * 64;
        if (c < N) {
          const int64_t o = (int64_t)row * N + c;
          const float v = rr * (g[r][i] - s1[r] - xh[r][i] * s2[r]);
          dh[o] = v;
          if (da) da[o] = DROP ? v * keep_mult(dk, (uint64_t)o) : v;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    red[0][wave][lane + i * 64] = pg[i];
    red[1][wave][lane + i * 64] = pb[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += 256) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { sg += red[0][w][c]; sb += red[1][w][c]; }
    ws[(int64_t)blockIdx.x * N + c] = sg;                          // dgamma partials [nb][N]
    ws[(int64_t)gridDim.x * N + (int64_t)blockIdx.x * N + c] = sb; // dbeta partials  [nb][N]
  }
}

// LN backward for the encoder width N = 64: lane (r, q) of a wave owns columns 16q .. 16q+15 of
// row r of a 16-row group (16-byte loads and stores, a row = 4 lanes x 64 contiguous bytes), the
// row sums are two xor-shuffles instead of a 64-lane reduction per row, and the sublayer's
// dropout draws two masks per hash. dgamma/dbeta partials: [nb][128] (gamma | beta).
template <bool DROP>
__global__ __launch_bounds__(256) void ln_bwd64_kernel(const float* __restrict__ h,
                                                       const float* dy,  // may alias dh
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       float* dh, int M,
                                                       float* __restrict__ ws,
                                                       float* __restrict__ da, float pdrop,
                                                       const int64_t* __restrict__ key, int site) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  __shared__ float red[4][64][17];
  DropKey dk{};
  if (DROP) dk = make_key(key, site, pdrop);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  float gm[16], pg[16], pb[16];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f4 v = *reinterpret_cast<const f4*>(gamma + 16 * q + 4 * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) gm[4 * u + e] = v[e];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) pg[i] = pb[i] = 0.f;
  const int groups = (M + 15) / 16;
  for (int gi = blockIdx.x * 4 + wave; gi < groups; gi += gridDim.x * 4) {
    const int row = gi * 16 + r;
    const bool ok = row < M;
    const int64_t o = (int64_t)(ok ? row : 0) * 64 + 16 * q;
    float hv[16], dv[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f4 a = *reinterpret_cast<const f4*>(h + o + 4 * u);
      const f4 b = *reinterpret_cast<const f4*>(dy + o + 4 * u);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hv[4 * u + e] = a[e];
        dv[4 * u + e] = ok ? b[e] : 0.f;
      }
    }
    const float mu = mean[ok ? row : 0], rr = rstd[ok ? row : 0];
    float xh[16], g[16], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      xh[i] = (hv[i] - mu) * rr;
      pg[i] += dv[i] * xh[i];
      pb[i] += dv[i];
      g[i] = dv[i] * gm[i];
      s1 += g[i];
      s2 += g[i] * xh[i];
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    s1 /= 64.f;
    s2 /= 64.f;
    if (ok) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        f4 v, w;
        float mk[4] = {1.f, 1.f, 1.f, 1.f};
        if (DROP) keep4(dk, (uint64_t)(o + 4 * u), mk);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * u + e;
          v[e] = rr * (g[i] - s1 - xh[i] * s2);
          w[e] = DROP ? v[e] * mk[e] : v[e];
        }
        *reinterpret_cast<f4*>(dh + o + 4 * u) = v;
        if (da) *reinterpret_cast<f4*>(da + o + 4 * u) = w;
      }
    }
  }
  // column partials: lanes with the same q hold the same 16 columns; fixed-order sum over the
  // 16 rows r and the 4 waves
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[wave][lane][i] = pass == 0 ? pg[i] : pb[i];
    __syncthreads();
    if (threadIdx.x < 64) {
      const int c = threadIdx.x, qq = c >> 4, i = c & 15;
      float t = 0.f;
      for (int w = 0; w < 4; ++w)
        for (int rr2 = 0; rr2 < 16; ++rr2) t += red[w][16 * qq + rr2][i];
      ws[(int64_t)blockIdx.x * 128 + pass * 64 + c] = t;
    }
    __syncthreads();
  }
}

int ln_blocks(int M) {
  constexpr int cap = 2048;  // 512 / 1,024 / 2,048 / 3,200 measured equal within noise at C2
  int nb = cdiv(M, 4 * 4 * 4);  // >= 4 row groups per wave
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  return nb;
}

// ------------------------------------------------------------------------------ BatchNorm
constexpr int kBnU = 16; // independent loads in flight per thread in the BatchNorm row loops

int bn_chunks(int Bg) {
  // 64-row chunks (32 / 128 / 256 measured slower at C2): 16 rows per thread in
  // the partial kernel
  constexpr int rows = 64;
  int s = cdiv(Bg, rows);
  if (s > 512) s = 512;
  if (s < 1) s = 1;
  return s;
}

// partial (sum a, sum b) per column over a row chunk of one group.
// MODE 0: a = x, b = x*x.   MODE 1: a = dy', b = dy' * xhat  (dy' = relu-masked dy)
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ y,
                                                         const float* __restrict__ dy,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, int Bg,
                                                         int C, int S, int relu,
                                                         float drop_scale,
                                                         double* __restrict__ ws) {
  __shared__ double red[2][256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int g = blockIdx.y, s = blockIdx.z;
  const int rpc = (Bg + S - 1) / S;
  const int r0 = s * rpc, r1 = min(Bg, r0 + rpc);
  double sa = 0.0, sb = 0.0;
  if (c < C) {
    float mu = 0.f, r = 0.f;
    if (MODE == 1) { mu = mean[g * C + c]; r = rstd[g * C + c]; }
    // kBnU rows per thread loaded before any is summed (rows past the chunk re-read its last
    // row and are masked); the summation order is unchanged: i, i + 4, i + 8, ...
    for (int i0 = r0 + rl; i0 < r1; i0 += 4 * kBnU) {
      float xv[kBnU], dv[kBnU], yv[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        const int i = min(i0 + 4 * u, r1 - 1);
        const int64_t o = ((int64_t)g * Bg + i) * C + c;
        xv[u] = x[o];
        if (MODE == 1) {
          dv[u] = dy[o];
          yv[u] = relu ? y[o] : 1.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (i0 + 4 * u >= r1) break;
        if (MODE == 0) {
          sa += (double)xv[u];
          sb += (double)xv[u] * (double)xv[u];
        } else {
          float d = dv[u];
          if (relu) d = yv[u] > 0.f ? d * drop_scale : 0.f;
          const float xh = (xv[u] - mu) * r;
          sa += (double)d;
          sb += (double)d * (double)xh;
        }
      }
    }
  }
  red[0][threadIdx.x] = sa;
  red[1][threadIdx.x] = sb;
  __syncthreads();
  if (rl == 0 && c < C) {
    double ta = 0.0, tb = 0.0;
#pragma unroll
    for (int w = 0; w < 4; ++w) { ta += red[0][w * 64 + threadIdx.x]; tb += red[1][w * 64 + threadIdx.x]; }
    const int64_t base = ((int64_t)g * S + s) * 2 * C;
    ws[base + c] = ta;
    ws[base + C + c] = tb;
  }
}

// column statistics of group g from the S chunk partials, summed in a fixed order (4 row lanes
// strided over the chunks, then lane 0..3): every block of the column group gets the same bits
__device__ __forceinline__ void bn_col_sums(const double* __restrict__ ws, int g, int S, int C,
                                            int c, int rl, double (*red)[2][64], double& A,
                                            double& Bv) {
  const int cl = threadIdx.x & 63;
  double sa = 0.0, sb = 0.0;
  if (c < C)
    for (int s0 = rl; s0 < S; s0 += 4 * kBnU) {
      double pa[kBnU], pb[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        const int64_t base = ((int64_t)g * S + min(s0 + 4 * u, S - 1)) * 2 * C;
        pa[u] = ws[base + c];
        pb[u] = ws[base + C + c];
      }
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (s0 + 4 * u >= S) break;
        sa += pa[u];
        sb += pb[u];
      }
    }
  red[rl][0][cl] = sa;
  red[rl][1][cl] = sb;
  __syncthreads();
  A = red[0][0][cl] + red[1][0][cl] + red[2][0][cl] + red[3][0][cl];
  Bv = red[0][1][cl] + red[1][1][cl] + red[2][1][cl] + red[3][1][cl];
  __syncthreads();
}

// training forward, second kernel: stats from the partials + normalise this block's row chunk.
// Block (column group, g, chunk); chunk-0 blocks publish mean/rstd, block (cg, 0, 0) updates the
// running statistics for g = 0..G-1 in order.
__global__ __launch_bounds__(256) void bn_fwd_norm_kernel(
    const double* __restrict__ ws, const float* __restrict__ x, float* __restrict__ y,
    const float* __restrict__ w, const float* __restrict__ b, float* running_mean,
    float* running_var, int64_t* num_batches, float* __restrict__ mean, float* __restrict__ rstd,
    int G, int Bg, int C, int S, float momentum, float eps, int relu, float drop_p,
    const int64_t* __restrict__ key, int site) {
  __shared__ double red[4][2][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int g = blockIdx.y, s = blockIdx.z;
  const double n = (double)Bg;
  double A, Bv;
  // this block's first kBnU rows are loaded before the statistics are reduced from the partials:
  // the two global latencies overlap (one row batch per thread at the usual 64-row chunks)
  const int rpc = (Bg + S - 1) / S;
  const int r1 = min(Bg, (s + 1) * rpc);
  const int i_first = s * rpc + rl;
  const int cc = min(c, C - 1);
  float xv[kBnU];
#pragma unroll
  for (int u = 0; u < kBnU; ++u) xv[u] = x[((int64_t)g * Bg + min(i_first + 4 * u, r1 - 1)) * C + cc];
  if (g == 0 && s == 0 && running_mean) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && num_batches) *num_batches += G;
    for (int gg = 0; gg < G; ++gg) {
      bn_col_sums(ws, gg, S, C, c, rl, red, A, Bv);
      if (rl == 0 && c < C) {
        const double mu = A / n;
        double var = Bv / n - mu * mu;
        if (var < 0.0) var = 0.0;
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mu;
        const double unb = Bg > 1 ? var * n / (n - 1.0) : var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
      }
    }
  } else if (blockIdx.x == 0 && g == 0 && s == 0 && threadIdx.x == 0 && num_batches) {
    *num_batches += G;
  }
  bn_col_sums(ws, g, S, C, c, rl, red, A, Bv);
  if (c >= C) return;
  const double mu = A / n;
  double var = Bv / n - mu * mu;
  if (var < 0.0) var = 0.0;
  const float muf = (float)mu, r = (float)(1.0 / sqrt(var + (double)eps));
  if (s == 0 && rl == 0) {
    mean[g * C + c] = muf;
    rstd[g * C + c] = r;
  }
  const float wc = w[c], bc = b[c];
  DropKey dk{};
  const bool drop = drop_p > 0.f;
  if (drop) dk = make_key(key, site, drop_p);
  for (int i0 = i_first; i0 < r1; i0 += 4 * kBnU) {
    if (i0 != i_first) {
#pragma unroll
      for (int u = 0; u < kBnU; ++u) xv[u] = x[((int64_t)g * Bg + min(i0 + 4 * u, r1 - 1)) * C + c];
    }
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      if (i0 + 4 * u >= r1) break;
      const int64_t o = ((int64_t)g * Bg + i0 + 4 * u) * C + c;
      float v = (xv[u] - muf) * r * wc + bc;
      if (relu) v = fmaxf(v, 0.f);
      if (drop) v *= keep_mult(dk, (uint64_t)o);  // the block's nn.Dropout (rs_dropout_fwd draw)
      y[o] = v;
    }
  }
}

// backward, second kernel: mean(dy'), mean(dy' * xhat) from the partials + dx for this block's
// row chunk; block (cg, 0, 0) accumulates dW = sum dy' xhat and dB = sum dy' over all groups.
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(
    const double* __restrict__ ws, const float* __restrict__ x, const float* __restrict__ y,
    const float* __restrict__ dy, const float* __restrict__ w, const float* __restrict__ mean,
    const float* __restrict__ rstd, float* __restrict__ dx, float* dw, float* db, int G, int Bg,
    int C, int S, int relu, float drop_scale) {
  __shared__ double red[4][2][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int g = blockIdx.y, s = blockIdx.z;
  double A, Bv;
  // first row batch loaded before the statistics (see bn_fwd_norm_kernel)
  const int rpc = (Bg + S - 1) / S;
  const int r1 = min(Bg, (s + 1) * rpc);
  const int i_first = s * rpc + rl;
  const int cc = min(c, C - 1);
  float xv[kBnU], dv[kBnU], yv[kBnU];
#pragma unroll
  for (int u = 0; u < kBnU; ++u) {
    const int64_t o = ((int64_t)g * Bg + min(i_first + 4 * u, r1 - 1)) * C + cc;
    xv[u] = x[o];
    dv[u] = dy[o];
    yv[u] = relu ? y[o] : 1.f;
  }
  if (g == 0 && s == 0) {
    double tw = 0.0, tb = 0.0;
    for (int gg = 0; gg < G; ++gg) {
      bn_col_sums(ws, gg, S, C, c, rl, red, A, Bv);
      tb += A;
      tw += Bv;
    }
    if (rl == 0 && c < C) {
      dw[c] += (float)tw;
      db[c] += (float)tb;
    }
  }
  bn_col_sums(ws, g, S, C, c, rl, red, A, Bv);
  if (c >= C) return;
  const float mdy = (float)(A / Bg), mdyx = (float)(Bv / Bg);
  const float mu = mean[g * C + c], r = rstd[g * C + c], wr = w[c] * r;
  for (int i0 = i_first; i0 < r1; i0 += 4 * kBnU) {
    if (i0 != i_first) {
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        const int64_t o = ((int64_t)g * Bg + min(i0 + 4 * u, r1 - 1)) * C + c;
        xv[u] = x[o];
        dv[u] = dy[o];
        yv[u] = relu ? y[o] : 1.f;
      }
    }
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      if (i0 + 4 * u >= r1) break;
      float d = dv[u];
      if (relu) d = yv[u] > 0.f ? d * drop_scale : 0.f;
      const float xh = (xv[u] - mu) * r;
      dx[((int64_t)g * Bg + i0 + 4 * u) * C + c] = wr * (d - mdy - xh * mdyx);
    }
  }
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv,
                                     int G, int C, float eps, float* __restrict__ mean,
                                     float* __restrict__ rstd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * C) return;
  const int c = i % C;
  mean[i] = rm[c];
  rstd[i] = 1.f / sqrtf(rv[c] + eps);
}

__global__ void bn_norm_kernel(const float* __restrict__ x, float* __restrict__ y,
                               const float* __restrict__ w, const float* __restrict__ b,
                               const float* __restrict__ mean, const float* __restrict__ rstd,
                               int Bg, int C, int64_t total, int relu) {
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const int g = (int)(idx / ((int64_t)Bg * C));
    float v = (x[idx] - mean[g * C + c]) * rstd[g * C + c] * w[c] + b[c];
    if (relu) v = fmaxf(v, 0.f);
    y[idx] = v;
  }
}

// ------------------------------------------------------------------------------ L2 norm
template <int NPL>
__global__ __launch_bounds__(256) void l2_fwd_kernel(const float* __restrict__ x,
                                                     float* __restrict__ y,
                                                     float* __restrict__ norm, int M, int N,
                                                     float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NPL], s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    v[i] = c < N ? x[(int64_t)row * N + c] : 0.f;
    s += v[i] * v[i];
  }
  const float n = sqrtf(wave_sum(s));
  const float den = fmaxf(n, eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    if (c < N) y[(int64_t)row * N + c] = v[i] / den;
  }
  if (lane == 0) norm[row] = n;
}

template <int NPL>
__global__ __launch_bounds__(256) void l2_bwd_kernel(const float* __restrict__ y,
                                                     const float* __restrict__ norm,
                                                     const float* __restrict__ dy,
                                                     float* __restrict__ dx, int M, int N,
                                                     float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float yv[NPL], g[NPL], s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    yv[i] = 0.f; g[i] = 0.f;
    if (c < N) { yv[i] = y[(int64_t)row * N + c]; g[i] = dy[(int64_t)row * N + c]; }
    s += yv[i] * g[i];
  }
  const float dot = wave_sum(s);
  const float n = norm[row];
  const bool clamped = !(n > eps);
  const float den = fmaxf(n, eps);
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = lane + i * 64;
    if (c < N) dx[(int64_t)row * N + c] = clamped ? g[i] / den : (g[i] - yv[i] * dot) / den;
  }
}

int npl_for(int N) {
  int k = cdiv(N, 64);
  if (k <= 1) return 1;
  if (k <= 2) return 2;
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 16) return 16;
  return -1;
}

}  // namespace
}  // namespace rs

using namespace rs;

#define RS_NPL_DISPATCH(NPLV, KERNEL, GRID, ...)                               \
  switch (NPLV) {                                                              \
    case 1: KERNEL<1><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    case 2: KERNEL<2><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    case 4: KERNEL<4><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    case 8: KERNEL<8><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    default: KERNEL<16><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;             \
  }

#define RS_NPL_DROP_DISPATCH(NPLV, DROPV, KERNEL, GRID, ...)                              \
  if (DROPV) {                                                                            \
    switch (NPLV) {                                                                       \
      case 1: KERNEL<1, true><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                  \
      case 2: KERNEL<2, true><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                  \
      case 4: KERNEL<4, true><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                  \
      case 8: KERNEL<8, true><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                  \
      default: KERNEL<16, true><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                \
    }                                                                                     \
  } else {                                                                                \
    switch (NPLV) {                                                                       \
      case 1: KERNEL<1, false><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
      case 2: KERNEL<2, false><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
      case 4: KERNEL<4, false><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
      case 8: KERNEL<8, false><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;                 \
      default: KERNEL<16, false><<<GRID, 256, 0, st>>>(__VA_ARGS__); break;               \
    }                                                                                     \
  }

extern "C" int rs_add_layernorm_fwd(float* a, const float* b, const float* gamma,
                                    const float* beta, float* y, float* mean, float* rstd, int M,
                                    int N, float eps, float p, const int64_t* key, int site,
                                    void* stream) {
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_add_layernorm_fwd: bad dropout p");
  RS_CHECK_ARG(a && b && gamma && beta && y && mean && rstd, "rs_add_layernorm_fwd: null pointer");
  const int npl = npl_for(N);
  RS_CHECK_ARG(M >= 0 && N >= 1 && npl > 0, "rs_add_layernorm_fwd: bad shape M=%d N=%d", M, N);
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  RS_NPL_DROP_DISPATCH(npl, p > 0.f, add_ln_fwd_kernel, cdiv(M, 4), a, b, gamma, beta, y, mean, rstd,
                       M, N, eps, p, key, site);
  RS_CHECK_LAUNCH("rs_add_layernorm_fwd");
  return 0;
}

extern "C" int64_t rs_layernorm_ws_bytes(int M, int N) {
  return (int64_t)ln_blocks(M) * 2 * N * (int64_t)sizeof(float);
}

extern "C" int rs_layernorm_bwd(const float* h, const float* dy, const float* gamma,
                                const float* mean, const float* rstd, float* dh, float* dgamma,
                                float* dbeta, int M, int N, float* da, float p, const int64_t* key,
                                int site, float* ws, void* stream) {
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || (key && da)), "rs_layernorm_bwd: bad dropout p");
  RS_CHECK_ARG(h && dy && gamma && mean && rstd && dh && dgamma && dbeta && ws,
               "rs_layernorm_bwd: null pointer");
  const int npl = npl_for(N);
  RS_CHECK_ARG(M >= 0 && N >= 1 && npl > 0, "rs_layernorm_bwd: bad shape");
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int nb = ln_blocks(M);
  if (N == 64 && aligned16(h) && aligned16(dy) && aligned16(dh) && aligned16(gamma) &&
      (!da || aligned16(da))) {
    if (p > 0.f) ln_bwd64_kernel<true><<<nb, 256, 0, st>>>(h, dy, gamma, mean, rstd, dh, M, ws, da, p, key, site);
    else ln_bwd64_kernel<false><<<nb, 256, 0, st>>>(h, dy, gamma, mean, rstd, dh, M, ws, da, p, key, site);
    RS_CHECK_LAUNCH("rs_layernorm_bwd n64");
    return partials_reduce2(ws, nb, 128, 64, 1.f, 1.f, dgamma, dbeta, st);
  }
  RS_NPL_DROP_DISPATCH(npl, p > 0.f, ln_bwd_kernel, nb, h, dy, gamma, mean, rstd, dh, M, N, ws, da, p,
                       key, site);
  RS_CHECK_LAUNCH("rs_layernorm_bwd");
  RS_RET_IF(partials_reduce(ws, nb, N, 1.f, 1.f, dgamma, st));
  return partials_reduce(ws + (int64_t)nb * N, nb, N, 1.f, 1.f, dbeta, st);
}

extern "C" int64_t rs_batchnorm_ws_bytes(int G, int Bg, int C) {
  const int S = bn_chunks(Bg);
  return (int64_t)G * S * 2 * C * (int64_t)sizeof(double) + (int64_t)G * 2 * C * sizeof(float);
}

extern "C" int rs_batchnorm_fwd(const float* x, float* y, const float* w, const float* b,
                                float* running_mean, float* running_var, int64_t* num_batches,
                                float* mean, float* rstd, int G, int Bg, int C, float momentum,
                                float eps, int relu, int training, float drop_p,
                                const int64_t* key, int site, float* ws, void* stream) {
  RS_CHECK_ARG(x && y && w && b && mean && rstd && ws, "rs_batchnorm_fwd: null pointer");
  RS_CHECK_ARG(drop_p == 0.f || (relu && training && key && drop_p > 0.f && drop_p < 1.f),
               "rs_batchnorm_fwd: dropout needs relu, training, a key and 0 < p < 1");
  RS_CHECK_ARG(G >= 1 && Bg >= 1 && C >= 1, "rs_batchnorm_fwd: bad shape G=%d Bg=%d C=%d", G, Bg, C);
  RS_CHECK_ARG(!running_mean == !running_var, "rs_batchnorm_fwd: running stats must come together");
  hipStream_t st = as_stream(stream);
  const int S = bn_chunks(Bg);
  double* wsd = reinterpret_cast<double*>(ws);
  const int64_t total = (int64_t)G * Bg * C;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  if (!training) {
    RS_CHECK_ARG(running_mean, "rs_batchnorm_fwd: eval mode needs running stats");
    bn_eval_stats_kernel<<<cdiv((int64_t)G * C, 256), 256, 0, st>>>(running_mean, running_var, G, C,
                                                                     eps, mean, rstd);
    RS_CHECK_LAUNCH("rs_batchnorm_fwd eval stats");
    bn_norm_kernel<<<blocks, 256, 0, st>>>(x, y, w, b, mean, rstd, Bg, C, total, relu);
    RS_CHECK_LAUNCH("rs_batchnorm_fwd norm");
    return 0;
  }
  bn_partial_kernel<0><<<dim3(cdiv(C, 64), G, S), 256, 0, st>>>(x, nullptr, nullptr, nullptr,
                                                                 nullptr, Bg, C, S, 0, 1.f, wsd);
  RS_CHECK_LAUNCH("rs_batchnorm_fwd partial");
  bn_fwd_norm_kernel<<<dim3(cdiv(C, 64), G, S), 256, 0, st>>>(wsd, x, y, w, b, running_mean,
                                                              running_var, num_batches, mean, rstd,
                                                              G, Bg, C, S, momentum, eps, relu,
                                                              drop_p, key, site);
  RS_CHECK_LAUNCH("rs_batchnorm_fwd norm");
  return 0;
}

extern "C" int rs_batchnorm_bwd(const float* x, const float* y, const float* dy, const float* w,
                                const float* mean, const float* rstd, float* dx, float* dw,
                                float* db, int G, int Bg, int C, int relu, float drop_scale,
                                float* ws, void* stream) {
  RS_CHECK_ARG(x && dy && w && mean && rstd && dx && dw && db && ws,
               "rs_batchnorm_bwd: null pointer");
  RS_CHECK_ARG(!relu || y, "rs_batchnorm_bwd: relu needs y");
  RS_CHECK_ARG(G >= 1 && Bg >= 1 && C >= 1, "rs_batchnorm_bwd: bad shape");
  hipStream_t st = as_stream(stream);
  const int S = bn_chunks(Bg);
  double* wsd = reinterpret_cast<double*>(ws);
  bn_partial_kernel<1><<<dim3(cdiv(C, 64), G, S), 256, 0, st>>>(x, y, dy, mean, rstd, Bg, C, S,
                                                                 relu, drop_scale, wsd);
  RS_CHECK_LAUNCH("rs_batchnorm_bwd partial");
  bn_bwd_dx_kernel<<<dim3(cdiv(C, 64), G, S), 256, 0, st>>>(wsd, x, y, dy, w, mean, rstd, dx, dw,
                                                            db, G, Bg, C, S, relu, drop_scale);
  RS_CHECK_LAUNCH("rs_batchnorm_bwd dx");
  return 0;
}

extern "C" int rs_l2norm_fwd(const float* x, float* y, float* norm, int M, int N, float eps,
                             void* stream) {
  RS_CHECK_ARG(x && y && norm, "rs_l2norm_fwd: null pointer");
  const int npl = npl_for(N);
  RS_CHECK_ARG(M >= 0 && N >= 1 && npl > 0, "rs_l2norm_fwd: bad shape");
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  RS_NPL_DISPATCH(npl, l2_fwd_kernel, cdiv(M, 4), x, y, norm, M, N, eps);
  RS_CHECK_LAUNCH("rs_l2norm_fwd");
  return 0;
}

extern "C" int rs_l2norm_bwd(const float* y, const float* norm, const float* dy, float* dx, int M,
                             int N, float eps, void* stream) {
  RS_CHECK_ARG(y && norm && dy && dx, "rs_l2norm_bwd: null pointer");
  const int npl = npl_for(N);
  RS_CHECK_ARG(M >= 0 && N >= 1 && npl > 0, "rs_l2norm_bwd: bad shape");
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  RS_NPL_DISPATCH(npl, l2_bwd_kernel, cdiv(M, 4), y, norm, dy, dx, M, N, eps);
  RS_CHECK_LAUNCH("rs_l2norm_bwd");
  return 0;
}
