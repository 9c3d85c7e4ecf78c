// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, one
// rounding per fma, 64 FLOP/clk/SIMD = the f32 vector peak; there is no xf32 on gfx950).
//
// Used for every dense contraction of the training step (nn.Linear forward/backward in the
// towers and the encoder, U @ I^T of the in-batch loss). Shapes on the hot path are skinny
// (K, N <= 256, M up to B*L = 204800) so the kernel is built for streaming A: 256-thread
// workgroups, 2x2 waves, each wave a (BM/2)x(BN/2) block of 32x32 MFMA tiles, BK = 16,
// global->register prefetch of tile t+1 under the MFMAs of tile t, double-buffered LDS (one
// barrier per k-tile). Transposed operands are written k-major into LDS so every MFMA operand
// read is a conflict-free ds_read_b32 across 32 consecutive lanes.
// Split-K (reductions over M = B*L for weight gradients) writes f32 partial slabs that a second
// kernel sums in a fixed order (bitwise reproducible) and finishes with the epilogue.
#include "common.h"
#include "gemm_stream.h"
#include "rng.h"

namespace rs {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BK = 16;
constexpr int PAD = 4;

struct GemmArgs {
  int M, N, K;
  float alpha, beta;
  const float* A;
  int lda;
  const float* B;
  int ldb;
  float* C;
  int ldc;
  int epi;
  const float* bias;
  const float* aux;
  int ld_aux, aux_mod;
  int split_k, kchunk;
  float* ws;
  float* rowsum;  // rowsum[m] += alpha * sum_k op(A)[m, k]
  int vecA, vecB;
  float drop_p;
  const int64_t* drop_key;
  int site_a, site_b;
};

template <class Args>
__device__ __forceinline__ float epilogue(const Args& a, int m, int n, float v, const DropKey& ka,
                                          const DropKey& kb) {
  if (a.epi & RS_EPI_BIAS) v += a.bias[n];
  if (a.epi & RS_EPI_AUX_MASK) v = a.aux[(int64_t)m * a.ld_aux + n] > 0.f ? v : 0.f;
  if (a.epi & RS_EPI_RELU) v = fmaxf(v, 0.f);
  if (a.epi & (RS_EPI_DROP_A | RS_EPI_DROP_B)) {
    const uint64_t e = (uint64_t)m * a.N + n;
    if (a.epi & RS_EPI_DROP_A) v *= keep_mult(ka, e);
    if (a.epi & RS_EPI_AUX_ADD) v += a.aux[(int64_t)(m % a.aux_mod) * a.ld_aux + n];
    if (a.epi & RS_EPI_DROP_B) v *= keep_mult(kb, e);
  } else if (a.epi & RS_EPI_AUX_ADD) {
    v += a.aux[(int64_t)(m % a.aux_mod) * a.ld_aux + n];
  }
  if (a.beta != 0.f) v += a.beta * a.C[(int64_t)m * a.ldc + n];
  return v;
}

// Loads of one operand tile (ROWS = M or N extent of the tile) into registers.
// T == false: element (r, k) at P[r*ld + k] (contiguous in k) -> slots of 4 consecutive k.
// T == true : element (r, k) at P[k*ld + r] (contiguous in r) -> slots of 4 consecutive r.
template <int ROWS, bool T>
struct TileLoader {
  static constexpr int kSlots = ROWS * BK / 4;           // float4 slots per tile
  static constexpr int kPer = (kSlots + 255) / 256;      // slots per thread
  float4 reg[kPer];

  __device__ __forceinline__ void load(const float* __restrict__ P, int ld, int r0, int rmax,
                                       int k0, int kend, bool vec, int tid) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      int s = tid + i * 256;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < kSlots) {
        int r, k;
        if (!T) { r = s / (BK / 4); k = (s % (BK / 4)) * 4; }
        else    { k = s / (ROWS / 4); r = (s % (ROWS / 4)) * 4; }
        int gr = r0 + r, gk = k0 + k;
        if (!T) {
          if (gr < rmax) {
            const float* p = P + (int64_t)gr * ld + gk;
            if (vec && gk + 3 < kend) v = *reinterpret_cast<const float4*>(p);
            else {
              if (gk + 0 < kend) v.x = p[0];
              if (gk + 1 < kend) v.y = p[1];
              if (gk + 2 < kend) v.z = p[2];
              if (gk + 3 < kend) v.w = p[3];
            }
          }
        } else {
          if (gk < kend) {
            const float* p = P + (int64_t)gk * ld + gr;
            if (vec && gr + 3 < rmax) v = *reinterpret_cast<const float4*>(p);
            else {
              if (gr + 0 < rmax) v.x = p[0];
              if (gr + 1 < rmax) v.y = p[1];
              if (gr + 2 < rmax) v.z = p[2];
              if (gr + 3 < rmax) v.w = p[3];
            }
          }
        }
      }
      reg[i] = v;
    }
  }

  // LDS image is k-major: S[k][r], pitch ROWS + PAD.
  __device__ __forceinline__ void store(float* S, int tid) const {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      int s = tid + i * 256;
      if (s >= kSlots) break;
      if (!T) {
        int r = s / (BK / 4), k = (s % (BK / 4)) * 4;
        S[(k + 0) * (ROWS + PAD) + r] = reg[i].x;
        S[(k + 1) * (ROWS + PAD) + r] = reg[i].y;
        S[(k + 2) * (ROWS + PAD) + r] = reg[i].z;
        S[(k + 3) * (ROWS + PAD) + r] = reg[i].w;
      } else {
        int k = s / (ROWS / 4), r = (s % (ROWS / 4)) * 4;
        *reinterpret_cast<float4*>(&S[k * (ROWS + PAD) + r]) = reg[i];
      }
    }
  }
};

template <int BM, int BN, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs a) {
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 tiles per wave in m / n
  __shared__ __attribute__((aligned(16))) float As[2][BK * (BM + PAD)];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * (BN + PAD)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int z = blockIdx.z;
  const int kbeg = z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // fused row sums of op(A) (bias gradient of a weight-gradient GEMM): one n-tile column of
  // workgroups, thread t < BM owns row m0 + t and reads its k-column of the staged A tile
  const bool do_rowsum = a.rowsum != nullptr && blockIdx.y == 0 && tid < BM;
  float rsum = 0.f;

  TileLoader<BM, TA> la;
  TileLoader<BN, !TB> lb;  // B(k, n): !TB is contiguous in n  ->  "T" layout of the loader
  const bool vecA = a.vecA, vecB = a.vecB;

  int buf = 0;
  if (kbeg < kend) {
    la.load(a.A, a.lda, m0, a.M, kbeg, kend, vecA, tid);
    lb.load(a.B, a.ldb, n0, a.N, kbeg, kend, vecB, tid);
    la.store(As[0], tid);
    lb.store(Bs[0], tid);
  }
  __syncthreads();

  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) {
      la.load(a.A, a.lda, m0, a.M, k0 + BK, kend, vecA, tid);
      lb.load(a.B, a.ldb, n0, a.N, k0 + BK, kend, vecB, tid);
    }
    const float* Asb = As[buf];
    const float* Bsb = Bs[buf];
    if (do_rowsum) {
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) rsum += Asb[kk * (BM + PAD) + tid];
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int kr = kk + (lane >> 5);
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = Asb[kr * (BM + PAD) + wm + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bsb[kr * (BN + PAD) + wn + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.store(As[buf ^ 1], tid);
      lb.store(Bs[buf ^ 1], tid);
    }
    __syncthreads();
    buf ^= 1;
  }

  if (do_rowsum && m0 + tid < a.M) {
    if (a.split_k > 1) a.ws[(int64_t)a.split_k * a.M * a.N + (int64_t)z * a.M + m0 + tid] = a.alpha * rsum;
    else a.rowsum[m0 + tid] += a.alpha * rsum;
  }
  DropKey ka{}, kb{};
  if (a.epi & RS_EPI_DROP_A) ka = make_key(a.drop_key, a.site_a, a.drop_p);
  if (a.epi & RS_EPI_DROP_B) kb = make_key(a.drop_key, a.site_b, a.drop_p);
  // epilogue: C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn + j * 32 + (lane & 31);
      if (n >= a.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= a.M) continue;
        float v = a.alpha * acc[i][j][r];
        if (a.split_k > 1) {
          a.ws[((int64_t)z * a.M + m) * a.N + n] = v;
        } else {
          a.C[(int64_t)m * a.ldc + n] = epilogue(a, m, n, v, ka, kb);
        }
      }
    }
}

__global__ void splitk_reduce_kernel(GemmArgs a) {
  const int64_t total = (int64_t)a.M * a.N;
  DropKey ka{}, kb{};
  if (a.epi & RS_EPI_DROP_A) ka = make_key(a.drop_key, a.site_a, a.drop_p);
  if (a.epi & RS_EPI_DROP_B) kb = make_key(a.drop_key, a.site_b, a.drop_p);
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float v[16];
    int z = 0;
    float acc = 0.f;
    // fixed order, 16 independent loads in flight
    for (; z + 16 <= a.split_k; z += 16) {
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = a.ws[(int64_t)(z + u) * total + idx];
#pragma unroll
      for (int u = 0; u < 16; ++u) acc += v[u];
    }
    for (; z < a.split_k; ++z) acc += a.ws[(int64_t)z * total + idx];
    const int m = (int)(idx / a.N), n = (int)(idx % a.N);
    a.C[(int64_t)m * a.ldc + n] = epilogue(a, m, n, acc, ka, kb);
    if (a.rowsum && idx < a.M) {
      const float* rs = a.ws + (int64_t)a.split_k * total;
      float r = 0.f;
      for (int zz = 0; zz < a.split_k; ++zz) r += rs[(int64_t)zz * a.M + idx];
      a.rowsum[idx] += r;
    }
  }
}

template <int BM, int BN>
void launch_tile(const GemmArgs& g, int ta, int tb, hipStream_t st) {
  dim3 grid(cdiv(g.M, BM), cdiv(g.N, BN), g.split_k);
  if (!ta && !tb) gemm_f32_kernel<BM, BN, false, false><<<grid, 256, 0, st>>>(g);
  else if (!ta && tb) gemm_f32_kernel<BM, BN, false, true><<<grid, 256, 0, st>>>(g);
  else if (ta && !tb) gemm_f32_kernel<BM, BN, true, false><<<grid, 256, 0, st>>>(g);
  else gemm_f32_kernel<BM, BN, true, true><<<grid, 256, 0, st>>>(g);
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_gemm_auto_split(int M, int N, int K) {
  // Fill the chip (>= ~512 workgroups) when the output is small and K is long.
  const int BMt = M >= 2048 ? 128 : 64, BNt = N > 64 ? 128 : 64;
  int64_t tiles = (int64_t)cdiv(M, BMt) * cdiv(N, BNt);
  if (tiles >= 256 || K < 1024) return 1;
  // weight-gradient streaming kernel (gemm_stream.hip): needs a workspace only
  if (K >= 2048 && (int64_t)M * N <= 16384 && wgrad_instance(M, N)) return 2;
  int s = (int)((512 + tiles - 1) / tiles);
  // each split keeps >= 256 rows of K: the fixed-order reduce then sums <= K/256 partials per
  // output (a 64-way split of a K = 4096 weight gradient took 22 us to compute and 20 us to
  // reduce; 16-way: one batch of loads in the reduce)
  int maxs = K / 256;
  if (s > maxs) s = maxs;
  if (s > 64) s = 64;
  return s < 1 ? 1 : s;
}

extern "C" int64_t rs_gemm_ws_bytes(int M, int N, int K, int split_k) {
  int64_t b = split_k > 1 ? (int64_t)split_k * ((int64_t)M * N + M) * (int64_t)sizeof(float) : 0;
  if (K >= 2048) {  // the weight-gradient streaming kernel may be chosen (gemm_stream.hip)
    const int64_t w = wgrad_ws_bytes(M, N, K);
    if (w > b) b = w;
  }
  return b;
}

extern "C" int rs_gemm_f32(int transA, int transB, int M, int N, int K, float alpha,
                           const float* A, int lda, const float* B, int ldb, float beta, float* C,
                           int ldc, int epilogue, const float* bias, const float* aux, int ld_aux,
                           int aux_mod, float drop_p, const int64_t* drop_key, int site_a,
                           int site_b, float* rowsum, int split_k, float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "rs_gemm_f32: negative size M=%d N=%d K=%d", M, N, K);
  if (M == 0 || N == 0) return 0;
  const int mode = epilogue & RS_GEMM_BF16;  // a compute-mode flag, not an epilogue stage
  const int io = epilogue & (RS_GEMM_A_BF16 | RS_GEMM_C_BF16);  // bf16 storage of A / C
  epilogue &= ~(RS_GEMM_BF16 | RS_GEMM_A_BF16 | RS_GEMM_C_BF16);
  RS_CHECK_ARG(!io || (mode && !transA && !rowsum && split_k <= 1),
               "rs_gemm_f32: bf16 A/C storage needs RS_GEMM_BF16, transA = 0, no rowsum/split-K");
  RS_CHECK_ARG(A && B && C, "rs_gemm_f32: null operand");
  RS_CHECK_ARG(ldc >= N, "rs_gemm_f32: ldc %d < N %d", ldc, N);
  RS_CHECK_ARG(transA ? lda >= M : lda >= K, "rs_gemm_f32: bad lda %d", lda);
  RS_CHECK_ARG(transB ? ldb >= K : ldb >= N, "rs_gemm_f32: bad ldb %d", ldb);
  RS_CHECK_ARG(!(epilogue & RS_EPI_BIAS) || bias, "rs_gemm_f32: bias epilogue without bias");
  RS_CHECK_ARG(!(epilogue & (RS_EPI_AUX_ADD | RS_EPI_AUX_MASK)) || (aux && ld_aux > 0),
               "rs_gemm_f32: aux epilogue without aux");
  RS_CHECK_ARG(!((epilogue & RS_EPI_AUX_ADD) && (epilogue & RS_EPI_AUX_MASK)),
               "rs_gemm_f32: AUX_ADD and AUX_MASK are exclusive");
  RS_CHECK_ARG(!(epilogue & (RS_EPI_DROP_A | RS_EPI_DROP_B)) ||
                   (drop_key && drop_p >= 0.f && drop_p < 1.f),
               "rs_gemm_f32: dropout epilogue needs a key and 0 <= p < 1");
  if (split_k < 1) split_k = 1;
  RS_CHECK_ARG(split_k == 1 || ws, "rs_gemm_f32: split_k %d needs a workspace", split_k);
  GemmArgs g;
  g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
  g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc;
  g.epi = epilogue; g.bias = bias; g.aux = aux; g.ld_aux = ld_aux;
  g.aux_mod = (epilogue & RS_EPI_AUX_ADD) ? (aux_mod > 0 ? aux_mod : M) : 1;
  int kt = cdiv(K, BK);
  int per = cdiv(kt, split_k);
  g.kchunk = per * BK;
  g.split_k = cdiv(K, g.kchunk);
  if (K == 0) { g.split_k = 1; g.kchunk = BK; }
  g.ws = ws;
  g.rowsum = rowsum;
  g.drop_p = drop_p; g.drop_key = drop_key; g.site_a = site_a; g.site_b = site_b;
  g.vecA = (lda % 4 == 0) && aligned16(A);
  g.vecB = (ldb % 4 == 0) && aligned16(B);
  hipStream_t st = as_stream(stream);
  {
    StreamArgs sa{};
    sa.M = M; sa.N = N; sa.K = K; sa.alpha = alpha; sa.beta = beta; sa.A = A; sa.lda = lda;
    sa.B = B; sa.ldb = ldb; sa.C = C; sa.ldc = ldc; sa.epi = epilogue | mode | io; sa.bias = bias;
    sa.aux = aux; sa.ld_aux = ld_aux; sa.aux_mod = g.aux_mod; sa.rowsum = rowsum; sa.ws = ws;
    sa.transB = transB;
    sa.drop_p = drop_p; sa.drop_key = drop_key; sa.site_a = site_a; sa.site_b = site_b;
    if (!rowsum && rowgemm_supported(transA, M, N, K, A, lda)) return rowgemm_launch(sa, st);
    RS_CHECK_ARG(!io, "rs_gemm_f32: no streaming instance for bf16 A/C storage (M=%d N=%d K=%d)", M, N, K);
    if (ws && wgrad_supported(transA, transB, M, N, K, A, lda, B, ldb, ldc, epilogue))
      return wgrad_launch(sa, st);
  }
  // 128-wide tiles only when they still give >= 256 workgroups
  const bool bigM = M >= 2048 && (int64_t)cdiv(M, 128) * cdiv(N, N > 64 ? 128 : 64) * g.split_k >= 256;
  const bool wideN = N > 64 && (int64_t)cdiv(M, bigM ? 128 : 64) * cdiv(N, 128) * g.split_k >= 256;
  if (bigM && wideN) launch_tile<128, 128>(g, transA, transB, st);
  else if (bigM) launch_tile<128, 64>(g, transA, transB, st);
  else if (wideN) launch_tile<64, 128>(g, transA, transB, st);
  else launch_tile<64, 64>(g, transA, transB, st);
  RS_CHECK_LAUNCH("rs_gemm_f32");
  if (g.split_k > 1) {
    int64_t total = (int64_t)M * N;
    if (total < M) total = M;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    splitk_reduce_kernel<<<blocks, 256, 0, st>>>(g);
    RS_CHECK_LAUNCH("rs_gemm_f32 splitk");
  }
  return 0;
}

// h = dropout(A W^T + bias) + resid; y = LayerNorm(h) (TransformerEncoderLayer's
// norm(x + dropout(sublayer(x))) with the sublayer's last Linear). One streaming kernel for the
// encoder shape (N = d_model = 64); otherwise the GEMM followed by rs_add_layernorm_fwd.
// rs_gemm_add_layernorm with the residual read in place: row m's residual is resid row
// m * resid_bag + resid_rows[m] (round 5: the pruned last encoder layer's x[b, last[b]], no gathered
// copy). bf16 mode, M % 16 == 0, N == 64, K % 64 == 0 only; -1 (rs_last_error) otherwise, and the
// caller gathers and takes rs_gemm_add_layernorm.
extern "C" int rs_gemm_add_layernorm_rows(int M, int N, int K, const float* A, int lda, const float* W, int ldw,
                                          const float* bias, const float* resid, const int64_t* resid_rows,
                                          int resid_bag, float* h, float* y, const float* gamma, const float* beta,
                                          float* mean, float* rstd, float eps, float p, const int64_t* key, int site,
                                          int flags, void* stream) {
  RS_CHECK_ARG(A && W && resid && resid_rows && h && y && gamma && beta && mean && rstd && resid_bag >= 1,
               "rs_gemm_add_layernorm_rows: null pointer / bad bag");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_gemm_add_layernorm_rows: bad dropout p");
  RS_CHECK_ARG((flags & RS_GEMM_BF16) && M >= 16 && M % 16 == 0 && N == 64 && K % 64 == 0 && lda % 4 == 0 &&
                   ldw % 4 == 0 && aligned16(A) && aligned16(W) && (K == 64 || K == 256),
               "rs_gemm_add_layernorm_rows: bf16 mode, M %% 16 == 0, N == 64, K in {64, 256} only");
  if (M == 0) return 0;
  StreamArgs sa{};
  sa.M = M; sa.N = N; sa.K = K; sa.alpha = 1.f; sa.beta = 0.f; sa.A = A; sa.lda = lda;
  sa.B = W; sa.ldb = ldw; sa.transB = 1; sa.C = h; sa.ldc = N;
  sa.epi = RS_EPI_AUX_ADD | (bias ? RS_EPI_BIAS : 0) | (p > 0.f ? RS_EPI_DROP_A : 0) | RS_GEMM_BF16;
  sa.bias = bias; sa.aux = resid; sa.ld_aux = N; sa.aux_mod = M;
  sa.aux_rows = resid_rows; sa.aux_bag = resid_bag;
  sa.drop_p = p; sa.drop_key = key; sa.site_a = site;
  sa.ln_gamma = gamma; sa.ln_beta = beta; sa.ln_y = y; sa.ln_mean = mean; sa.ln_rstd = rstd;
  sa.ln_eps = eps;
  return rowgemm_ln_launch(sa, as_stream(stream));
}

extern "C" int rs_gemm_add_layernorm(int M, int N, int K, const float* A, int lda, const float* W,
                                     int ldw, const float* bias, const float* resid, float* h,
                                     float* y, const float* gamma, const float* beta, float* mean,
                                     float* rstd, float eps, float p, const int64_t* key, int site,
                                     int flags, void* stream) {
  RS_CHECK_ARG(M >= 0 && N >= 1 && K >= 1, "rs_gemm_add_layernorm: bad shape");
  RS_CHECK_ARG(A && W && resid && h && y && gamma && beta && mean && rstd,
               "rs_gemm_add_layernorm: null pointer");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_gemm_add_layernorm: bad dropout p");
  if (M == 0) return 0;
  hipStream_t st = as_stream(stream);
  // bf16 mode, B-row calls (the pruned last encoder layer, M = 4,096): the fused bf16 kernel takes
  // them too (round 5: one launch instead of the small-M fp32 GEMM + rs_add_layernorm_fwd)
  // K in {64, 256}: the bf16 instances' kc = K / 64 in {1, 4} (other FFN widths take the GEMM +
  // rs_add_layernorm_fwd below)
  const bool small_bf16 = (flags & RS_GEMM_BF16) && M >= 16 && M % 16 == 0 && N == 64 &&
                          (K == 64 || K == 256) && lda % 4 == 0 && ldw % 4 == 0 && aligned16(A) && aligned16(W);
  if ((rowgemm_ln_supported(M, N, K, A, lda) || small_bf16) && !getenv_flag("RSYS_UNFUSED_LN")) {
    StreamArgs sa{};
    sa.M = M; sa.N = N; sa.K = K; sa.alpha = 1.f; sa.beta = 0.f; sa.A = A; sa.lda = lda;
    sa.B = W; sa.ldb = ldw; sa.transB = 1; sa.C = h; sa.ldc = N;
    sa.epi = RS_EPI_AUX_ADD | (bias ? RS_EPI_BIAS : 0) | (p > 0.f ? RS_EPI_DROP_A : 0) |
             (flags & RS_GEMM_BF16);
    sa.bias = bias; sa.aux = resid; sa.ld_aux = N; sa.aux_mod = M;
    sa.drop_p = p; sa.drop_key = key; sa.site_a = site;
    sa.ln_gamma = gamma; sa.ln_beta = beta; sa.ln_y = y; sa.ln_mean = mean; sa.ln_rstd = rstd;
    sa.ln_eps = eps;
    return rowgemm_ln_launch(sa, st);
  }
  RS_RET_IF(rs_gemm_f32(0, 1, M, N, K, 1.f, A, lda, W, ldw, 0.f, h, N,
                        (bias ? RS_EPI_BIAS : 0) | (flags & RS_GEMM_BF16), bias,
                        nullptr, 0, 0, 0.f, nullptr, 0, 0, nullptr, 1, nullptr, stream));
  return rs_add_layernorm_fwd(h, resid, gamma, beta, y, mean, rstd, M, N, eps, p, key, site, stream);
}
