// Streaming fp32 GEMMs for the encoder's big-M shapes (M = B*L = 204,800 tokens, K, N <= 256),
// selected automatically by rs_gemm_f32.
//
// rowgemm: C[M,N] = A[M,K] @ op(B)  (A row-major; B = W[N][K] (nn.Linear forward) or W[K][N]
//   (input gradient)). The whole op(B) (<= 256 x 256 fp32) is staged ONCE per persistent
//   workgroup into LDS as Bs[n][k]; each wave streams 16-row groups of A straight from HBM into
//   registers with 16-byte loads and keeps all N columns of its 16 rows in accumulators.
//   v_mfma_f32_16x16x4_f32 with a permuted k order: lane (r = l&15, q = l>>4) loads
//   A[r][16t+4q .. +3] as one float4 and feeds element s to the s-th MFMA of chunk t, whose k slot
//   q then stands for k = 16t + 4q + s; the B fragment for the same lane is the float4
//   Bs[n][16t+4q .. +3] (one ds_read_b128). Sums over k are order-free, so every A byte is read
//   once, coalesced, with no LDS round trip; the next row group is prefetched under the MFMAs.
// wgrad: dW[Mo,No] = dY^T X over a long M (weight gradients). One workgroup owns the whole dW
//   tile (Mo*No <= 16K floats in accumulators) for a chunk of rows; dY and X chunks are staged
//   k-major exactly as they lie in memory (no transposition), partial tiles are summed by a
//   fixed-order reduce (deterministic), and the bias gradient colsum(dY) is fused.
#include "common.h"
#include "gemm_stream.h"
#include "rng.h"
#include "stage.h"

namespace rs {



namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// same epilogue order as gemm.hip (see rsys_hip.h)
__device__ __forceinline__ float epi_apply(const StreamArgs& a, int m, int n, float v,
                                           const DropKey& ka, const DropKey& kb) {
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

// four consecutive columns n0..n0+3 of row m (same order of operations as epi_apply)
// aux row element of (m, n0..n0+3) for AUX_MASK (row m) / AUX_ADD (row m % aux_mod)
__device__ __forceinline__ const float* aux_ptr(const StreamArgs& a, int m, int n0) {
  const int row = (a.epi & RS_EPI_AUX_ADD) ? m % a.aux_mod : m;
  return a.aux + (int64_t)row * a.ld_aux + n0;
}

// auxv: the prefetched aux values of (m, n0..n0+3) when the epilogue has AUX_MASK / AUX_ADD
__device__ __forceinline__ floatx4 epi_apply4(const StreamArgs& a, int m, int n0, floatx4 v,
                                              const DropKey& ka, const DropKey& kb,
                                              const floatx4& auxv) {
  if (a.epi & RS_EPI_BIAS) v += *reinterpret_cast<const floatx4*>(a.bias + n0);
  if (a.epi & RS_EPI_AUX_MASK) {
    const floatx4 mk = auxv;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = mk[i] > 0.f ? v[i] : 0.f;
  }
  if (a.epi & RS_EPI_RELU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
  }
  const uint64_t e0 = (uint64_t)m * a.N + n0;
  if (a.epi & RS_EPI_DROP_A) {
    float mk[4];
    keep4(ka, e0, mk);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= mk[i];
  }
  if (a.epi & RS_EPI_AUX_ADD) v += auxv;
  if (a.epi & RS_EPI_DROP_B) {
    float mk[4];
    keep4(kb, e0, mk);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= mk[i];
  }
  if (a.beta != 0.f) v += a.beta * *reinterpret_cast<const floatx4*>(a.C + (int64_t)m * a.ldc + n0);
  return v;
}

// residual + LayerNorm over a full row of N = NT*16 columns. Lane (r, q) holds, for row m, the
// columns t*16 + 4q + e (t < NT, e < 4); the row's other columns are in the lanes q' != q with
// the same r: two xor shuffles (16, 32) complete the row sums. Same operation order per element
// as the unfused pair (GEMM epilogue: alpha*acc + bias; add_ln: drop(.) + resid, mean, centred
// variance, 1/sqrtf).
template <int NT, int EPI>
__device__ __forceinline__ void ln_epilogue(const StreamArgs& a, int m, int q, const floatx4* acc,
                                            const floatx4* resv, const DropKey& ka,
                                            const float* sbias, const float* sgamma,
                                            const float* sbeta) {
  constexpr bool kBias = EPI >= 0 ? (EPI & RS_EPI_BIAS) != 0 : false;
  constexpr bool kDrop = EPI >= 0 ? (EPI & RS_EPI_DROP_A) != 0 : false;
  constexpr int N = NT * 16;
  float hv[NT][4];
  float s = 0.f;
  const bool ok = EPI >= 0 || m < a.M;  // specialised instances: M % 16 == 0
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n0 = t * 16 + 4 * q;
    floatx4 v = acc[t] * a.alpha;
    if (EPI >= 0 ? kBias : (a.epi & RS_EPI_BIAS) != 0) v += *reinterpret_cast<const floatx4*>(sbias + n0);
    const floatx4 res = resv[t];
    float mk[4] = {1.f, 1.f, 1.f, 1.f};
    if (EPI >= 0 ? kDrop : (a.epi & RS_EPI_DROP_A) != 0) keep4(ka, (uint64_t)m * N + n0, mk);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (EPI >= 0 ? kDrop : (a.epi & RS_EPI_DROP_A) != 0) x *= mk[e];
      hv[t][e] = x + res[e];
      s += hv[t][e];
    }
  }
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mu = s / (float)N;
  float vs = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = hv[t][e] - mu;
      vs += d * d;
    }
  vs += __shfl_xor(vs, 16, 64);
  vs += __shfl_xor(vs, 32, 64);
  const float rs = 1.f / sqrtf(vs / (float)N + a.ln_eps);
  if (!ok) return;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n0 = t * 16 + 4 * q;
    const floatx4 gm = *reinterpret_cast<const floatx4*>(sgamma + n0);
    const floatx4 bt = *reinterpret_cast<const floatx4*>(sbeta + n0);
    floatx4 h4, y4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      h4[e] = hv[t][e];
      y4[e] = (hv[t][e] - mu) * rs * gm[e] + bt[e];
    }
    *reinterpret_cast<floatx4*>(a.C + (int64_t)m * a.ldc + n0) = h4;
    *reinterpret_cast<floatx4*>(a.ln_y + (int64_t)m * N + n0) = y4;
  }
  if (q == 0) {
    a.ln_mean[m] = mu;
    a.ln_rstd[m] = rs;
  }
}

// compile-time epilogue (EPI = RS_EPI_* bits | kEpiBeta): no uniform branches in the store
// loop, so the compiler can count outstanding stores exactly instead of draining vmcnt(0) (which
// also waited for the next row group's prefetched A) after every epilogue load. bias and the
// AUX_ADD table (aux_mod rows: the positional embedding) come from LDS.
constexpr int kEpiBeta = 64;
template <int EPI>
__device__ __forceinline__ floatx4 epi4_ct(const StreamArgs& a, int m, int n0, floatx4 v,
                                           const DropKey& ka, const DropKey& kb,
                                           const floatx4& biasv, const floatx4& auxv,
                                           const floatx4& cv) {
  if constexpr ((EPI & RS_EPI_BIAS) != 0) v += biasv;
  if constexpr ((EPI & RS_EPI_AUX_MASK) != 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = auxv[i] > 0.f ? v[i] : 0.f;
  }
  if constexpr ((EPI & RS_EPI_RELU) != 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
  }
  const uint64_t e0 = (uint64_t)m * a.N + n0;
  if constexpr ((EPI & RS_EPI_DROP_A) != 0) {
    float mk[4];
    keep4(ka, e0, mk);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= mk[i];
  }
  if constexpr ((EPI & RS_EPI_AUX_ADD) != 0) v += auxv;
  if constexpr ((EPI & RS_EPI_DROP_B) != 0) {
    float mk[4];
    keep4(kb, e0, mk);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= mk[i];
  }
  if constexpr ((EPI & kEpiBeta) != 0) v += a.beta * cv;
  return v;
}

// ---------------------------------------------------------------------------------- rowgemm
// RG row groups of 16 per wave step: every B fragment read from LDS feeds RG MFMA chains (the
// LDS reads, not the MFMAs, bounded the one-group loop at K = 64: 45 % MFMA-busy measured).
template <int NT, int KT, bool LN = false, int RG = 1, int EPI = -1>
__global__ __launch_bounds__(512) void rowgemm_kernel(StreamArgs a) {
  constexpr int KP = KT * 16 + 4;  // LDS pitch (floats): conflict-free ds_read_b128 per 16 lanes
  // specialised instances are lean enough (~100 VGPRs) to prefetch K = 256 rows too
  constexpr bool PREFETCH = KT * RG <= 8 || (EPI >= 0 && RG == 1 && KT <= 16);
  extern __shared__ __attribute__((aligned(16))) float Bs[];  // [NT*16][KP]
  const int tid = threadIdx.x;
  const int nb0 = blockIdx.y * NT * 16;  // this workgroup's column slice (small-M N split)
  // the first row group's A loads are issued before the weight staging: the two global
  // latencies overlap instead of adding up (small-M grids run one or two row groups per wave)
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int groups = (a.M + 16 * RG - 1) / (16 * RG);
  DropKey ka{}, kb{};
  if (a.epi & RS_EPI_DROP_A) ka = make_key(a.drop_key, a.site_a, a.drop_p);
  if (a.epi & RS_EPI_DROP_B) kb = make_key(a.drop_key, a.site_b, a.drop_p);
  const int stride = gridDim.x * 8;
  int g = blockIdx.x * 8 + wave;
  floatx4 areg[RG][KT];
  // FULL (specialised instances): M % 16 == 0 and K % 4 == 0, so no row / k guards and no
  // uniform branches in the loop body -- the waitcnt pass can then count the outstanding
  // stores exactly instead of draining vmcnt(0) (which also waited for the prefetch). When K is
  // not a multiple of 16 (the sequence projection, K = 40) the last k tile's out-of-range float4s
  // re-read the row's last float4 (clamped address): the staged weight is zero for k >= K, so
  // they contribute exact zeros.
  constexpr bool FULL = EPI >= 0;
  auto load_group = [&](int gg, floatx4 (*dst)[KT]) {
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      const int m = (gg * RG + rg) * 16 + r;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int k = 16 * t + 4 * q;
        const int kc = (FULL && t == KT - 1) ? min(k, a.K - 4) : k;
        floatx4 v = {0.f, 0.f, 0.f, 0.f};
        // explicit global address space: a flat load would also count against lgkmcnt
        if (FULL || (m < a.M && k < a.K))
          v = *(const __attribute__((address_space(1))) floatx4*)(a.A + (int64_t)m * a.lda + kc);
        dst[rg][t] = v;
      }
    }
  };
  if (g < groups) load_group(g, areg);
  // stage op(B)[:, nb0 : nb0 + NT*16] as Bs[n][k], zero padded to NT*16 x KT*16
  // batched 16-byte loads (dispatch: K % 4 == 0; [K][N] weights also need N % 4 == 0)
  if (a.ldb % 4 == 0 && ((uintptr_t)a.B & 15) == 0 && (a.transB || a.N % 4 == 0)) {
    if (a.transB) {
      stage_batched<NT * 16, KT * 16, 512>(
          a.B + (int64_t)nb0 * a.ldb, a.ldb,
          [&](int n, int k, const floatx4& v) { *reinterpret_cast<floatx4*>(Bs + n * KP + k) = v; },
          [&](int n, int k) { return nb0 + n < a.N && k < a.K; });
    } else {
      stage_batched<KT * 16, NT * 16, 512>(
          a.B + nb0, a.ldb,
          [&](int k, int n, const floatx4& v) {
#pragma unroll
            for (int e = 0; e < 4; ++e) Bs[(n + e) * KP + k] = v[e];
          },
          [&](int k, int n) { return k < a.K && nb0 + n < a.N; });
    }
  } else if (a.transB) {  // B[n*ldb + k]: consecutive threads -> consecutive k
    for (int idx = tid; idx < NT * 16 * KT * 16; idx += 512) {
      const int n = idx / (KT * 16), k = idx % (KT * 16);
      Bs[n * KP + k] = (nb0 + n < a.N && k < a.K) ? a.B[(int64_t)(nb0 + n) * a.ldb + k] : 0.f;
    }
  } else {  // B[k*ldb + n]: consecutive threads -> consecutive n
    for (int idx = tid; idx < NT * 16 * KT * 16; idx += 512) {
      const int k = idx / (NT * 16), n = idx % (NT * 16);
      Bs[n * KP + k] = (nb0 + n < a.N && k < a.K) ? a.B[(int64_t)k * a.ldb + nb0 + n] : 0.f;
    }
  }
  // specialised epilogues: bias [NT*16] and the AUX_ADD table [aux_mod][NT*16] in LDS
  constexpr int NTN = NT * 16;
  float* sbias = Bs + NTN * KP;
  float* saux = sbias + NTN;
  if constexpr ((EPI >= 0 && (EPI & RS_EPI_BIAS) != 0) || LN) {
    if (EPI >= 0 ? (EPI & RS_EPI_BIAS) != 0 : (a.epi & RS_EPI_BIAS) != 0)
      for (int n = tid; n < NTN; n += 512) sbias[n] = a.bias[nb0 + n];
  }
  float* sgamma = saux;  // LN: gamma, beta after the bias (LN kernels have no AUX table in LDS)
  float* sbeta = saux + NTN;
  if constexpr (LN) {
    for (int n = tid; n < NTN; n += 512) {
      sgamma[n] = a.ln_gamma[n];
      sbeta[n] = a.ln_beta[n];
    }
  }
  if constexpr (!LN && EPI >= 0 && (EPI & RS_EPI_AUX_ADD) != 0) {
    for (int idx = tid; idx < a.aux_mod * NTN; idx += 512) {
      const int rr = idx / NTN, n = idx % NTN;
      saux[idx] = a.aux[(int64_t)rr * a.ld_aux + nb0 + n];
    }
  }
  __syncthreads();

  floatx4 lnacc[LN ? RG : 1][LN ? NT : 1];
  for (; g < groups; g += stride) {
    floatx4 lnres[LN ? RG : 1][LN ? NT : 1];
    if constexpr (LN) {  // residual rows, issued BEFORE the next group's A prefetch (vmcnt is in order)
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int m = (g * RG + rg) * 16 + r;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const floatx4 z = {0.f, 0.f, 0.f, 0.f};
          lnres[rg][t] = (FULL || m < a.M) ? *reinterpret_cast<const floatx4*>(a.aux + (int64_t)m * a.ld_aux + t * 16 + 4 * q) : z;
        }
      }
    }
    // specialised epilogues' global operands (AUX_MASK rows / C for beta), also issued before
    // the A prefetch so that waiting for them does not wait for the prefetch
    constexpr bool EPRE = EPI >= 0 && (EPI & (RS_EPI_AUX_MASK | kEpiBeta)) != 0;
    static_assert(EPI < 0 || (EPI & RS_EPI_AUX_MASK) == 0 || (EPI & kEpiBeta) == 0,
                  "AUX_MASK and beta cannot both be preloaded");
    floatx4 epre[EPRE ? RG : 1][EPRE ? NT : 1];
    if constexpr (EPRE) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        const int m = (g * RG + rg) * 16 + r;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n0 = nb0 + t * 16 + 4 * q;
          if constexpr ((EPI & RS_EPI_AUX_MASK) != 0)
            epre[rg][t] = *reinterpret_cast<const floatx4*>(a.aux + (int64_t)m * a.ld_aux + n0);
          else
            epre[rg][t] = *reinterpret_cast<const floatx4*>(a.C + (int64_t)m * a.ldc + n0);
        }
      }
    }
    floatx4 anext[RG][KT];  // dead (eliminated) without PREFETCH
    if constexpr (PREFETCH) {
      if constexpr (FULL) load_group(g + stride < groups ? g + stride : g, anext);  // no branch
      else if (g + stride < groups) load_group(g + stride, anext);
    }
    // N tiles in groups of TG: TG independent accumulator chains hide the 40-cycle dependent
    // MFMA latency; each group is stored right away so only 4*TG*RG accumulators are live.
    // Specialised instances use TG = 4 (more MFMAs between the B-fragment LDS reads).
    constexpr int TG = (EPI >= 0 && NT % 4 == 0 && RG == 1) ? 4 : 2;
#pragma unroll
    for (int j0 = 0; j0 < NT; j0 += TG) {
      // keep the scheduler from hoisting every group's B reads / accumulators (register spills)
      __builtin_amdgcn_sched_barrier(0);
      floatx4 acc[RG][TG];
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int h = 0; h < TG; ++h) acc[rg][h] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        floatx4 b[TG];
#pragma unroll
        for (int h = 0; h < TG; ++h)
          b[h] = (j0 + h < NT) ? *reinterpret_cast<const floatx4*>(&Bs[((j0 + h) * 16 + r) * KP + 16 * t + 4 * q])
                               : b[0];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          // W rows on the MFMA row side, the 16 A rows on the column side: each lane ends up
          // holding 4 consecutive output columns of one row (float4 epilogue loads / stores)
#pragma unroll
          for (int rg = 0; rg < RG; ++rg)
#pragma unroll
            for (int h = 0; h < TG; ++h)
              if (j0 + h < NT)
                acc[rg][h] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[h][s4], areg[rg][t][s4], acc[rg][h], 0, 0, 0);
        }
      }
      // C/D map of 16x16: col = lane&15 -> row m of A, row = 4*(lane>>4) + i -> column n of C
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        if constexpr (LN) {
#pragma unroll
          for (int h = 0; h < TG; ++h)
            if (j0 + h < NT) lnacc[rg][j0 + h] = acc[rg][h];
          continue;
        }
        const int m = (g * RG + rg) * 16 + r;
        if constexpr (EPI >= 0) {  // N % (NT*16) == 0 and 16-byte rows guaranteed by the dispatch
#pragma unroll
          for (int h = 0; h < TG; ++h) {
            if (j0 + h >= NT) break;
            const int nl = (j0 + h) * 16 + 4 * q, n0 = nb0 + nl;
            {  // FULL: every row valid
              const floatx4 z = {0.f, 0.f, 0.f, 0.f};
              floatx4 biasv = z, auxv = z, cv = z;
              if constexpr ((EPI & RS_EPI_BIAS) != 0) biasv = *reinterpret_cast<const floatx4*>(sbias + nl);
              if constexpr ((EPI & RS_EPI_AUX_ADD) != 0)
                auxv = *reinterpret_cast<const floatx4*>(saux + (m % a.aux_mod) * NTN + nl);
              if constexpr ((EPI & RS_EPI_AUX_MASK) != 0) auxv = epre[rg][j0 + h];
              if constexpr ((EPI & kEpiBeta) != 0) cv = epre[rg][j0 + h];
              *reinterpret_cast<floatx4*>(a.C + (int64_t)m * a.ldc + n0) =
                  epi4_ct<EPI>(a, m, n0, acc[rg][h] * a.alpha, ka, kb, biasv, auxv, cv);
            }
          }
          continue;
        }
#pragma unroll
        for (int h = 0; h < TG; ++h) {
          if (j0 + h >= NT) break;
          const int n0 = nb0 + (j0 + h) * 16 + 4 * q;
          if (m >= a.M || n0 >= a.N) continue;
          const floatx4 v = acc[rg][h] * a.alpha;
          float* crow = a.C + (int64_t)m * a.ldc;
          if (a.vec_epi && n0 + 3 < a.N) {
            floatx4 auxv = {0.f, 0.f, 0.f, 0.f};
            if (a.epi & (RS_EPI_AUX_ADD | RS_EPI_AUX_MASK))
              auxv = *reinterpret_cast<const floatx4*>(aux_ptr(a, m, n0));
            *reinterpret_cast<floatx4*>(crow + n0) = epi_apply4(a, m, n0, v, ka, kb, auxv);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + i < a.N) crow[n0 + i] = epi_apply(a, m, n0 + i, v[i], ka, kb);
          }
        }
      }
    }
    if constexpr (LN) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
        ln_epilogue<NT, EPI>(a, (g * RG + rg) * 16 + r, q, lnacc[rg], lnres[rg], ka, sbias, sgamma, sbeta);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PREFETCH) {
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
#pragma unroll
        for (int t = 0; t < KT; ++t) areg[rg][t] = anext[rg][t];
    } else if (g + stride < groups) {
      load_group(g + stride, areg);
    }
  }
}

// ---------------------------------------------------------------------------------- wgrad
constexpr int WG_BK = 16;

// op(A) = A^T with A = dY [Kr rows][lda] (GEMM M = Mo = dY columns), B = X [Kr][ldb] (N = No)
template <int MO_PAD, int NO_PAD>
__global__ __launch_bounds__(256) void wgrad_kernel(StreamArgs a, int rows_per_block) {
  constexpr int mo_pad = MO_PAD, no_pad = NO_PAD;
  constexpr int TPW = ((MO_PAD / 32) * (NO_PAD / 32) + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ys = sm;                                // [2][WG_BK][mo_pad]
  float* Xs = Ys + 2 * WG_BK * mo_pad;           // [2][WG_BK][no_pad]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Mo = a.M, No = a.N;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(a.K, r0 + rows_per_block);
  constexpr int tiles_n = no_pad / 32;
  constexpr int ntiles = (mo_pad / 32) * tiles_n;
  // register staging of one chunk: WG_BK rows x (mo_pad + no_pad) floats, float4 per slot
  constexpr int ysl = WG_BK * mo_pad / 4, xsl = WG_BK * no_pad / 4;
  constexpr int MAXS = (ysl + xsl + 255) / 256;
  floatx4 st[MAXS];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int i = 0; i < MAXS; ++i) {
      const int s = tid + i * 256;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if (s < ysl) {
        const int kk = s / (mo_pad / 4), c = (s % (mo_pad / 4)) * 4, m = c0 + kk;
        if (m < r1 && c < Mo) v = *reinterpret_cast<const floatx4*>(a.A + (int64_t)m * a.lda + c);
      } else if (s < ysl + xsl) {
        const int s2 = s - ysl;
        const int kk = s2 / (no_pad / 4), c = (s2 % (no_pad / 4)) * 4, m = c0 + kk;
        if (m < r1 && c < No) v = *reinterpret_cast<const floatx4*>(a.B + (int64_t)m * a.ldb + c);
      }
      st[i] = v;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < MAXS; ++i) {
      const int s = tid + i * 256;
      if (s < ysl) {
        *reinterpret_cast<floatx4*>(&Ys[buf * WG_BK * mo_pad + s * 4]) = st[i];
      } else if (s < ysl + xsl) {
        *reinterpret_cast<floatx4*>(&Xs[buf * WG_BK * no_pad + (s - ysl) * 4]) = st[i];
      }
    }
  };
  floatx16 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  float rsum = 0.f;
  const bool do_rs = a.rowsum != nullptr && tid < Mo;

  int buf = 0;
  if (r0 < r1) {
    load_chunk(r0);
    store_chunk(0);
  }
  __syncthreads();
  for (int c0 = r0; c0 < r1; c0 += WG_BK) {
    const bool more = c0 + WG_BK < r1;
    if (more) load_chunk(c0 + WG_BK);
    const float* Y = Ys + buf * WG_BK * mo_pad;
    const float* X = Xs + buf * WG_BK * no_pad;
    if (do_rs) {
#pragma unroll
      for (int kk = 0; kk < WG_BK; ++kk) rsum += Y[kk * mo_pad + tid];
    }
#pragma unroll
    for (int kk = 0; kk < WG_BK; kk += 2) {
      const int kr = kk + (lane >> 5);
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int tile = wave + 4 * t;
        if (tile < ntiles) {
          const int ti = tile / tiles_n, tj = tile % tiles_n;
          const float av = Y[kr * mo_pad + ti * 32 + (lane & 31)];
          const float bv = X[kr * no_pad + tj * 32 + (lane & 31)];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
        }
      }
    }
    if (more) store_chunk(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // partial tile -> ws[block][Mo][No] (fixed-order reduce later); rowsum partial after the tiles
  float* out = a.ws + (int64_t)blockIdx.x * Mo * No;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = wave + 4 * t;
    if (tile >= ntiles) continue;
    const int ti = tile / tiles_n, tj = tile % tiles_n;
    const int n = tj * 32 + (lane & 31);
    if (n >= No) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = ti * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      if (m < Mo) out[(int64_t)m * No + n] = acc[t][e];
    }
  }
  if (do_rs) a.ws[(int64_t)gridDim.x * Mo * No + (int64_t)blockIdx.x * Mo + tid] = rsum;
}

// C[m][n] = beta*C + alpha*sum_p ws[p][m*No+n];  rowsum[m] += alpha*sum_p wsr[p][m]
__global__ __launch_bounds__(1024) void wgrad_reduce_kernel(StreamArgs a, int P) {
  __shared__ float red[16][64];
  const int total = a.M * a.N;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int l = threadIdx.x >> 6;
  const bool is_rs = e >= total;
  const int rs_idx = e - total;
  float acc = 0.f;
  if (!is_rs || (a.rowsum && rs_idx < a.M)) {
    const float* base = is_rs ? a.ws + (int64_t)P * total + rs_idx : a.ws + e;
    const int64_t stride = is_rs ? a.M : total;
    int p = l;
    for (; p + 16 * 7 < P; p += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = base[(int64_t)(p + 16 * u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; p < P; p += 16) acc += base[(int64_t)p * stride];
  }
  red[l][threadIdx.x & 63] = acc;
  __syncthreads();
  if (l != 0) return;
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
  if (!is_rs) {
    if (e < total) {
      const int m = e / a.N, n = e % a.N;
      float v = a.alpha * t;
      if (a.beta != 0.f) v += a.beta * a.C[(int64_t)m * a.ldc + n];
      a.C[(int64_t)m * a.ldc + n] = v;
    }
  } else if (a.rowsum && rs_idx < a.M) {
    a.rowsum[rs_idx] += a.alpha * t;
  }
}

// --------------------------------------------------------------------- wgrad, bf16 MFMA
// bf16 compute mode: the same dW = dY^T X over a long row range on v_mfma_f32_32x32x16_bf16
// (16x the f32 MFMA rate, so the kernel is HBM-bound on the fp32 operands it streams). Rows are
// staged 32 at a time through registers (fp32, 16-byte loads) into a row-major bf16 LDS image;
// the MFMA operands want 8 consecutive ROWS of one column per lane, which ds_read_b64_tr_b16
// delivers from the row-major image (two transposed reads per fragment). The bias gradient
// colsum(dY) is taken from the fp32 registers before rounding (per-thread partials, then a
// fixed-order sum over the chunk's rows): it is exact fp32 as in the fp32 kernel.
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4w __attribute__((ext_vector_type(4)));
constexpr int WB_BK = 32;

// LDS row pitch (bf16 elements) for a pad-wide image: the 4 rows of one transposed read must
// fall in distinct 64-byte windows of the 256-byte bank space -> pitch*2 mod 256 in {64, 192}
constexpr int wb_pitch(int pad) { return (pad % 128 == 32 || pad % 128 == 96) ? pad : pad + 32; }

// wave grid over the (MO/32) x (NO/32) tiles: the split of 4 waves with the fewest fragments
constexpr int wb_gm(int tm, int tn) {
  int best = 1, cost = 1 << 30;
  for (int gm = 1; gm <= 4; gm *= 2) {
    const int gn = 4 / gm;
    const int c = (tm + gm - 1) / gm + (tn + gn - 1) / gn + 64 * ((tm < gm) + (tn < gn));
    if (c < cost) { cost = c; best = gm; }
  }
  return best;
}

__device__ __forceinline__ bf16x8w tr_frag(const __bf16* lds_lo, const __bf16* lds_hi) {
  typedef __attribute__((address_space(3))) shortx4* lptr;
  const shortx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds_lo));
  const shortx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds_hi));
  const shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8w, v);
}

// YB / XB: the operand is stored as bf16 in HBM (16-byte loads carry 8 elements and go to LDS
// as they are); otherwise fp32 (4 elements per load, rounded to bf16 on the way to LDS)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int MO_PAD, int NO_PAD, bool YB, bool XB>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(StreamArgs a, int rows_per_block) {
  constexpr int PY = wb_pitch(MO_PAD), PX = wb_pitch(NO_PAD);
  constexpr int TMT = MO_PAD / 32, TNT = NO_PAD / 32;
  constexpr int GM = wb_gm(TMT, TNT), GN = 4 / GM;
  constexpr int TM = (TMT + GM - 1) / GM, TN = (TNT + GN - 1) / GN;
  constexpr int VY = YB ? 8 : 4, VX = XB ? 8 : 4;  // elements per 16-byte slot
  constexpr int ysl = WB_BK * MO_PAD / VY, xsl = WB_BK * NO_PAD / VX;
  constexpr int MAXS = (ysl + xsl + 255) / 256;
  constexpr int NYS = (ysl + 255) / 256;  // slots that can hold dY (column partials)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __bf16* Ys = reinterpret_cast<__bf16*>(smem_raw);  // [2][WB_BK][PY]
  __bf16* Xs = Ys + 2 * WB_BK * PY;                    // [2][WB_BK][PX]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Mo = a.M, No = a.N;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(a.K, r0 + rows_per_block);
  const int wm = wave / GN, wn = wave % GN;
  const unsigned char* Ag = reinterpret_cast<const unsigned char*>(a.A);
  const unsigned char* Bg = reinterpret_cast<const unsigned char*>(a.B);
  constexpr int EY = YB ? 2 : 4, EX = XB ? 2 : 4;  // bytes per element in HBM
  u32x4 st[MAXS];
  float ysum[NYS][VY];
#pragma unroll
  for (int i = 0; i < NYS; ++i)
#pragma unroll
    for (int e = 0; e < VY; ++e) ysum[i][e] = 0.f;
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int i = 0; i < MAXS; ++i) {
      const int s = tid + i * 256;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (s < ysl) {
        const int kk = s / (MO_PAD / VY), c = (s % (MO_PAD / VY)) * VY, m = c0 + kk;
        if (m < r1 && c < Mo) v = *reinterpret_cast<const u32x4*>(Ag + ((int64_t)m * a.lda + c) * EY);
      } else if (s < ysl + xsl) {
        const int s2 = s - ysl;
        const int kk = s2 / (NO_PAD / VX), c = (s2 % (NO_PAD / VX)) * VX, m = c0 + kk;
        if (m < r1 && c < No) v = *reinterpret_cast<const u32x4*>(Bg + ((int64_t)m * a.ldb + c) * EX);
      }
      st[i] = v;
    }
  };
  auto put = [&](__bf16* dst, const u32x4& v, bool is_bf16) {
    if (is_bf16) {
      *reinterpret_cast<u32x4*>(dst) = v;
    } else {
      const floatx4 f = __builtin_bit_cast(floatx4, v);
      bf16x4w h;
      h[0] = (__bf16)f[0]; h[1] = (__bf16)f[1]; h[2] = (__bf16)f[2]; h[3] = (__bf16)f[3];
      *reinterpret_cast<bf16x4w*>(dst) = h;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < MAXS; ++i) {
      const int s = tid + i * 256;
      if (s < ysl) {
        if constexpr (YB) {
          const bf16x8w hv = __builtin_bit_cast(bf16x8w, st[i]);
#pragma unroll
          for (int e = 0; e < 8; ++e) ysum[i < NYS ? i : 0][e] += (float)hv[e];
        } else {
          const floatx4 f = __builtin_bit_cast(floatx4, st[i]);
#pragma unroll
          for (int e = 0; e < 4; ++e) ysum[i < NYS ? i : 0][e] += f[e];
        }
        const int kk = s / (MO_PAD / VY), c = (s % (MO_PAD / VY)) * VY;
        put(&Ys[(buf * WB_BK + kk) * PY + c], st[i], YB);
      } else if (s < ysl + xsl) {
        const int s2 = s - ysl;
        const int kk = s2 / (NO_PAD / VX), c = (s2 % (NO_PAD / VX)) * VX;
        put(&Xs[(buf * WB_BK + kk) * PX + c], st[i], XB);
      }
    }
  };
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // transposed-read addresses: lane 4q+p of 16-lane group g reads row q (+4 for the second
  // half of the fragment) of the block, columns 4p..4p+3 of the 16-column half (g & 1);
  // rows 8h.. with h = g >> 1
  const int g = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;
  const int trow = 8 * (g >> 1) + lq, tcol = 16 * (g & 1) + 4 * lp;

  int buf = 0;
  if (r0 < r1) {
    load_chunk(r0);
    store_chunk(0);
  }
  __syncthreads();
  for (int c0 = r0; c0 < r1; c0 += WB_BK) {
    const bool more = c0 + WB_BK < r1;
    if (more) load_chunk(c0 + WB_BK);
    const __bf16* Y = Ys + buf * WB_BK * PY;
    const __bf16* X = Xs + buf * WB_BK * PX;
#pragma unroll
    for (int ks = 0; ks < WB_BK / 16; ++ks) {
      bf16x8w af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ti = wm * TM + i;
        const __bf16* p = Y + (16 * ks + trow) * PY + 32 * (ti < TMT ? ti : 0) + tcol;
        af[i] = tr_frag(p, p + 4 * PY);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int tj = wn * TN + j;
        const __bf16* p = X + (16 * ks + trow) * PX + 32 * (tj < TNT ? tj : 0) + tcol;
        bfr[j] = tr_frag(p, p + 4 * PX);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_chunk(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // partial tile -> ws[block][Mo][No] (fixed-order reduce later)
  float* out = a.ws + (int64_t)blockIdx.x * Mo * No;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ti = wm * TM + i;
    if (ti >= TMT) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int tj = wn * TN + j;
      if (tj >= TNT) continue;
      const int n = tj * 32 + (lane & 31);
      if (n >= No) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = ti * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (m < Mo) out[(int64_t)m * No + n] = acc[i][j][e];
      }
    }
  }
  if (a.rowsum != nullptr) {
    // per-thread column partials -> R[kk][c] (reusing the staging LDS), then rows summed in order
    float* R = reinterpret_cast<float*>(smem_raw);
#pragma unroll
    for (int i = 0; i < NYS; ++i) {
      const int s = tid + i * 256;
      if (s < ysl)
#pragma unroll
        for (int e = 0; e < VY; ++e) R[s * VY + e] = ysum[i][e];
    }
    __syncthreads();
    if (tid < Mo) {
      float rsum = 0.f;
#pragma unroll 8
      for (int kk = 0; kk < WB_BK; ++kk) rsum += R[kk * MO_PAD + tid];
      a.ws[(int64_t)gridDim.x * Mo * No + (int64_t)blockIdx.x * Mo + tid] = rsum;
    }
  }
}

int wgrad_blocks(int Kr) {
  // row splits: 512 measured best at C2 (256 -> 0.101, 384 -> 0.091, 512 -> 0.083, 768 -> 0.082,
  // 1024 -> 0.099 ms per step of rs_wgrad_bf16)
  constexpr int cap = 512;
  int nb = Kr / 64;  // >= 64 rows per workgroup; short K (the MLP's B = 4096) still fills 64 CUs
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  return nb;
}


// ------------------------------------------------------------------------ rowgemm, bf16 MFMA
// Same streaming structure as rowgemm (persistent waves, op(B) staged once in LDS, one 16-row
// group of A per wave step, float4 epilogue via the swapped operand order), computing on
// v_mfma_f32_16x16x32_bf16: op(B) is rounded to bf16 once while staging, A rows are rounded in
// registers; products are exact in fp32 and accumulate in fp32. 16x the f32 MFMA rate, so these
// shapes (K <= 256) become purely HBM-bound. Used when the caller sets RS_GEMM_BF16 (bf16
// compute mode; SURVEY §8d: C2 is quoted in bf16 with fp32 master weights).
// k map of a 64-wide chunk c: lane (r, q) holds k = 64c + 16q + (0..15); MFMA 2c uses its first
// 8, MFMA 2c+1 the next 8 -- the same permutation for both operands, so the sum is unchanged.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 cvt8(const floatx4& lo, const floatx4& hi) {
  bf16x8 r;
  r[0] = (__bf16)lo[0]; r[1] = (__bf16)lo[1]; r[2] = (__bf16)lo[2]; r[3] = (__bf16)lo[3];
  r[4] = (__bf16)hi[0]; r[5] = (__bf16)hi[1]; r[6] = (__bf16)hi[2]; r[7] = (__bf16)hi[3];
  return r;
}

// IO bit 0: A is bf16 storage (RS_GEMM_A_BF16; loaded as bf16x8, no conversion); bit 1: C is
// written as bf16 (RS_GEMM_C_BF16; 8-byte stores). Either leaves every product unchanged.
template <int NT, int KC, bool LN, int EPI, int IO = 0>
__global__ __launch_bounds__(512) void rowgemm_bf16_kernel(StreamArgs a) {
  constexpr bool ABF = (IO & 1) != 0, CBF = (IO & 2) != 0;
  static_assert(!(CBF && (LN || (EPI & (RS_EPI_AUX_MASK | kEpiBeta)) != 0)),
                "bf16 C: no epilogue that reads C or aux rows");
  constexpr int KK = KC * 64;
  constexpr int KPH = KK + 8;  // LDS pitch in bf16 (16-byte pad: conflict-free b128 reads)
  constexpr int NTN = NT * 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __bf16* Bs = reinterpret_cast<__bf16*>(smem_raw);
  float* sbias = reinterpret_cast<float*>(smem_raw + (size_t)NTN * KPH * 2);
  float* saux = sbias + NTN;  // AUX_ADD table, or LN gamma / beta
  const int tid = threadIdx.x;
  // K tail (K < KK, K % 4 == 0, fp32 A only): op(B) columns k >= K are staged as zeros and the A
  // float4s at k >= K are not loaded (zeros), so the padded k slots add exact zeros
  const int K = a.K;
  // N tail (N < NTN, N % 4 == 0, no LN): op(B) rows n >= N are zeros and columns n >= N are
  // neither loaded (epilogue operands) nor stored
  const int N = a.N;
  if (a.transB) {  // B = W[N][K]: rows n (dispatch: ldb % 4 == 0, 16-byte aligned)
    stage_batched<NTN, KK, 512>(a.B, a.ldb, [&](int n, int k, const floatx4& v) {
      bf16x4w h;
      h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
      *reinterpret_cast<bf16x4w*>(Bs + n * KPH + k) = h;
    }, [&](int n, int k) { return k < K && n < N; });
  } else {  // B = W[K][N]: rows k
    stage_batched<KK, NTN, 512>(a.B, a.ldb, [&](int k, int n, const floatx4& v) {
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[(n + e) * KPH + k] = (__bf16)v[e];
    }, [&](int k, int n) { return k < K && n < N; });
  }
  if constexpr ((EPI & RS_EPI_BIAS) != 0)
    for (int n = tid; n < NTN; n += 512) sbias[n] = n < N ? a.bias[n] : 0.f;
  if constexpr (LN) {
    for (int n = tid; n < NTN; n += 512) {
      saux[n] = a.ln_gamma[n];
      saux[NTN + n] = a.ln_beta[n];
    }
  } else if constexpr ((EPI & RS_EPI_AUX_ADD) != 0) {
    for (int idx = tid; idx < a.aux_mod * NTN; idx += 512) {
      const int rr = idx / NTN, n = idx % NTN;
      saux[idx] = n < N ? a.aux[(int64_t)rr * a.ld_aux + n] : 0.f;
    }
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int groups = a.M / 16;  // dispatch: M % 16 == 0
  DropKey ka{}, kb{};
  if constexpr ((EPI & RS_EPI_DROP_A) != 0) ka = make_key(a.drop_key, a.site_a, a.drop_p);
  if constexpr ((EPI & RS_EPI_DROP_B) != 0) kb = make_key(a.drop_key, a.site_b, a.drop_p);
  const int stride = gridDim.x * 8;
  int g = blockIdx.x * 8 + wave;
  typedef const __attribute__((address_space(1))) floatx4* gptr4;
  typedef const __attribute__((address_space(1))) bf16x8* gptrb8;
  floatx4 araw[ABF ? 1 : KC][4];
  bf16x8 abraw[ABF ? KC : 1][2];
  auto load_raw = [&](int gg, floatx4 (*dst)[4]) {
    if constexpr (ABF) {
      const __bf16* row = reinterpret_cast<const __bf16*>(a.A) + (int64_t)(gg * 16 + r) * a.lda + 16 * q;
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        abraw[c][0] = *(gptrb8)(row + 64 * c);
        abraw[c][1] = *(gptrb8)(row + 64 * c + 8);
      }
    } else {
      const float* row = a.A + (int64_t)(gg * 16 + r) * a.lda + 16 * q;
#pragma unroll
      for (int c = 0; c < KC; ++c)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          dst[c][u] = (c + 1) * 64 <= K || 64 * c + 16 * q + 4 * u < K ? *(gptr4)(row + 64 * c + 4 * u)
                                                                      : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (g < groups) load_raw(g, araw);
  constexpr bool EPRE = !LN && (EPI & (RS_EPI_AUX_MASK | kEpiBeta)) != 0;
  for (; g < groups; g += stride) {
    const int m = g * 16 + r;
    floatx4 lnres[LN ? NT : 1];
    floatx4 epre[EPRE ? NT : 1];
    if constexpr (LN) {
      const int64_t rr = a.aux_rows ? (int64_t)m * a.aux_bag + a.aux_rows[m] : (int64_t)m;
#pragma unroll
      for (int t = 0; t < NT; ++t) lnres[t] = *(gptr4)(a.aux + rr * a.ld_aux + t * 16 + 4 * q);
    }
    if constexpr (EPRE) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n0 = t * 16 + 4 * q;
        if (n0 >= N) epre[t] = floatx4{0.f, 0.f, 0.f, 0.f};
        else if constexpr ((EPI & RS_EPI_AUX_MASK) != 0) epre[t] = *(gptr4)(a.aux + (int64_t)m * a.ld_aux + n0);
        else epre[t] = *(gptr4)(a.C + (int64_t)m * a.ldc + n0);
      }
    }
    bf16x8 af[KC][2];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      if constexpr (ABF) {
        af[c][0] = abraw[c][0];
        af[c][1] = abraw[c][1];
      } else {
        af[c][0] = cvt8(araw[c][0], araw[c][1]);
        af[c][1] = cvt8(araw[c][2], araw[c][3]);
      }
    }
    load_raw(g + stride < groups ? g + stride : g, araw);  // next group, no branch
    floatx4 lnacc[LN ? NT : 1];
    constexpr int TG = NT % 4 == 0 ? 4 : (NT % 2 == 0 ? 2 : 1);
#pragma unroll
    for (int j0 = 0; j0 < NT; j0 += TG) {
      __builtin_amdgcn_sched_barrier(0);
      floatx4 acc[TG];
#pragma unroll
      for (int h = 0; h < TG; ++h) acc[h] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KC; ++c) {
        bf16x8 b[TG][2];
#pragma unroll
        for (int h = 0; h < TG; ++h) {
          const __bf16* bp = Bs + ((j0 + h) * 16 + r) * KPH + 64 * c + 16 * q;
          b[h][0] = *reinterpret_cast<const bf16x8*>(bp);
          b[h][1] = *reinterpret_cast<const bf16x8*>(bp + 8);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int h = 0; h < TG; ++h)
            acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[h][u], af[c][u], acc[h], 0, 0, 0);
      }
#pragma unroll
      for (int h = 0; h < TG; ++h) {
        if constexpr (LN) {
          lnacc[j0 + h] = acc[h];
        } else {
          const int nl = (j0 + h) * 16 + 4 * q;
          const floatx4 z = {0.f, 0.f, 0.f, 0.f};
          floatx4 biasv = z, auxv = z, cv = z;
          if constexpr ((EPI & RS_EPI_BIAS) != 0) biasv = *reinterpret_cast<const floatx4*>(sbias + nl);
          if constexpr ((EPI & RS_EPI_AUX_ADD) != 0)
            auxv = *reinterpret_cast<const floatx4*>(saux + (m % a.aux_mod) * NTN + nl);
          if constexpr ((EPI & RS_EPI_AUX_MASK) != 0) auxv = epre[j0 + h];
          if constexpr ((EPI & kEpiBeta) != 0) cv = epre[j0 + h];
          if (nl >= N) continue;  // N tail
          const floatx4 v = epi4_ct<EPI>(a, m, nl, acc[h] * a.alpha, ka, kb, biasv, auxv, cv);
          if constexpr (CBF) {
            bf16x4w o;
            o[0] = (__bf16)v[0]; o[1] = (__bf16)v[1]; o[2] = (__bf16)v[2]; o[3] = (__bf16)v[3];
            *reinterpret_cast<bf16x4w*>(reinterpret_cast<__bf16*>(a.C) + (int64_t)m * a.ldc + nl) = o;
          } else {
            *reinterpret_cast<floatx4*>(a.C + (int64_t)m * a.ldc + nl) = v;
          }
        }
      }
    }
    if constexpr (LN) ln_epilogue<NT, EPI>(a, m, q, lnacc, lnres, ka, sbias, saux, saux + NTN);
  }
}

}  // namespace

// ------------------------------------------------------------------------------ dispatch
// Small M: split N over workgroups (NT = 4 column tiles each) so the grid still fills the chip.
constexpr int kSmallM = 32768;
constexpr int kSmallNT = 2;  // small M (the MLP at B = 4096): 32 columns per workgroup

// Grid of the big-M streaming GEMMs (persistent workgroups of 8 waves; each stages the whole
// weight once, so fewer, longer-lived workgroups re-read less of it). The grid is a whole number
// of workgroups per CU: the row groups are dealt round-robin, so every workgroup gets the same
// share and the kernel's time is that of the busiest CU. A fixed 32 groups per workgroup gave 400
// workgroups at C2 (12,800 groups): 144 CUs ran two, 112 one. Measured at C2 (token GEMMs per
// step): 32 per workgroup 0.280 ms, 25 (512 workgroups) 0.270, 50 (256) 0.264.
int stream_grid(int groups, int per_cu, int min_per_wg = 40) {
  int bx;
  if (groups <= 256 * 8) {
    bx = cdiv(groups, 8);  // one row group per wave
  } else {
    int k = groups / (256 * min_per_wg);  // >= min_per_wg groups per workgroup
    if (k < 1) k = 1;
    if (k > per_cu) k = per_cu;
    bx = 256 * k;
  }
  return bx < 1 ? 1 : bx;
}

bool rowgemm_supported(int transA, int M, int N, int K, const float* A, int lda) {
  if (transA || M < 1024 || K < 4 || K > 256 || N < 1 || N > 256) return false;
  if (K % 4 != 0 || lda % 4 != 0 || !aligned16(A)) return false;
  const int nt = M < kSmallM ? kSmallNT : (N + 15) / 16, kt = (K + 15) / 16;
  // instantiated (NT, KT) pairs: the encoder/projection shapes and the small-M MLP shapes
  switch (nt * 100 + kt) {
    case 403: case 404: case 412: case 416: case 1204: case 1604: case 304: case 1216:
    case 204: case 804: case 408: case 808: case 1608:
    case 405: case 504:  // C5's sequence projection (K = 72) and its input gradient (N = 72)
    case 203: case 208: case 211: case 212: case 216: return true;
    default: return false;
  }
}

int rowgemm_launch(const StreamArgs& s_in, hipStream_t st) {
  StreamArgs s = s_in;
  s.vec_epi = s.N % 4 == 0 && s.ldc % 4 == 0 && aligned16(s.C) &&
              (!(s.epi & RS_EPI_BIAS) || aligned16(s.bias)) &&
              (!(s.epi & (RS_EPI_AUX_ADD | RS_EPI_AUX_MASK)) || (s.ld_aux % 4 == 0 && aligned16(s.aux)));
  const bool small = s.M < kSmallM;
  const int nt = small ? kSmallNT : (s.N + 15) / 16, kt = (s.K + 15) / 16;
  const int nsplit = small ? cdiv(s.N, kSmallNT * 16) : 1;
  const size_t lds = (size_t)nt * 16 * (kt * 16 + 4) * sizeof(float);
  // one 16-row group per wave step (measured and removed: two groups per step sharing the B
  // fragments, 10-25 % slower on every K = 64 shape: more VGPRs, fewer resident waves)
  const int groups = (s.M + 15) / 16;
  int bx = cdiv(groups, small ? 8 : 8 * 2);  // small M: one row group per wave
  const int per_cu = lds > 80 * 1024 ? 1 : (lds > 53 * 1024 ? 2 : (lds > 40 * 1024 ? 3 : 4));
  if (bx > 256 * per_cu) bx = 256 * per_cu;
  if (bx < 1) bx = 1;
  const dim3 blocks(bx, nsplit);
  // bf16 compute mode: the bf16-MFMA instances (fp32 kernels below for anything else)
  const int io = ((s.epi & RS_GEMM_A_BF16) ? 1 : 0) | ((s.epi & RS_GEMM_C_BF16) ? 2 : 0);
  const int ekey = (s.epi & ~(RS_GEMM_BF16 | RS_GEMM_A_BF16 | RS_GEMM_C_BF16)) | (s.beta != 0.f ? kEpiBeta : 0);
  // K: a multiple of 64, or (fp32 A) of 4 with the tail zero-padded in the kernel
  if ((s.epi & RS_GEMM_BF16) && !small && s.vec_epi && s.M % 16 == 0 &&
      (s.K % 64 == 0 || (s.K % 4 == 0 && !(io & 1))) &&
      s.ldb % 4 == 0 && aligned16(s.B) &&
      (s.N == nt * 16 || (s.N % 4 == 0 && io == 0)) && s.lda % ((io & 1) ? 8 : 4) == 0 && (!(io & 1) || aligned16(s.A)) &&
      (!(s.epi & RS_EPI_AUX_ADD) || (int64_t)s.aux_mod * nt * 16 * 4 <= 48 * 1024)) {
    const int kc = (s.K + 63) / 64;
    const size_t ldsb = (size_t)nt * 16 * (kc * 64 + 8) * 2 + (size_t)(nt * 16 + ((s.epi & RS_EPI_AUX_ADD) ? s.aux_mod * nt * 16 : 0)) * 4;
    const int per_cub = ldsb > 80 * 1024 ? 1 : (ldsb > 53 * 1024 ? 2 : (ldsb > 40 * 1024 ? 3 : 4));
    const int bxb = stream_grid(s.M / 16, per_cub);
#define RS_RGB(NTV, KCV, EV, IOV)                                                                 \
    if (nt == NTV && kc == KCV && ekey == EV && io == IOV) {                                      \
      rowgemm_bf16_kernel<NTV, KCV, false, EV, IOV><<<bxb, 512, ldsb, st>>>(s);                   \
      RS_CHECK_LAUNCH("rowgemm bf16");                                                            \
      return 0;                                                                                   \
    }
    RS_RGB(16, 1, 19, 0) RS_RGB(16, 1, 3, 0) RS_RGB(16, 1, 8, 0) RS_RGB(16, 1, 0, 0) RS_RGB(12, 1, 1, 0)
    RS_RGB(4, 3, 64, 0) RS_RGB(4, 4, 64, 0) RS_RGB(4, 1, 0, 0) RS_RGB(4, 1, 64, 0) RS_RGB(4, 4, 0, 0)
    RS_RGB(4, 3, 0, 0) RS_RGB(3, 1, 0, 0) RS_RGB(3, 1, 64, 0)
    // the sequence projection (K = 48 at C2, 72 at C5: zero-padded k tail) and its input gradient
    RS_RGB(4, 1, 53, 0) RS_RGB(4, 1, 5, 0) RS_RGB(4, 2, 53, 0) RS_RGB(4, 2, 5, 0)
    // bf16 storage: the qkv projection's output (C) and its input gradient's dqkv operand (A)
    RS_RGB(12, 1, 1, 2) RS_RGB(12, 1, 0, 2) RS_RGB(4, 3, 64, 1) RS_RGB(4, 3, 0, 1)
#undef RS_RGB
  }
  if (io != 0) {
    set_error("rowgemm: no bf16-storage instance for M=%d N=%d K=%d epi=%d", s.M, s.N, s.K, s.epi);
    return -1;
  }
  // specialised (compile-time epilogue) instances for the encoder's GEMMs
  // the AUX_ADD table (positional rows) in LDS: up to 64 KB covers C5's L = 200 x 64 (51 KB; two
  // workgroups per CU then)
  const bool aux_small = !(s.epi & RS_EPI_AUX_ADD) || (int64_t)s.aux_mod * nt * 16 * 4 <= 64 * 1024;
  if (!small && s.vec_epi && s.N % (nt * 16) == 0 && aux_small && s.M % 16 == 0 &&
      s.K % 4 == 0 && !getenv_flag("RSYS_ROWGEMM_GENERIC")) {
    const size_t lds2 = lds + (size_t)(nt * 16 + ((s.epi & RS_EPI_AUX_ADD) ? s.aux_mod * nt * 16 : 0)) * sizeof(float);
    const int per_cu2 = lds2 > 80 * 1024 ? 1 : (lds2 > 53 * 1024 ? 2 : (lds2 > 40 * 1024 ? 3 : 4));
    const int bx2 = stream_grid(groups, per_cu2);
#define RS_RGE(NTV, KTV, EV)                                                                     \
    if (nt == NTV && kt == KTV && ekey == EV) {                                                  \
      rowgemm_kernel<NTV, KTV, false, 1, EV><<<dim3(bx2, 1), 512, lds2, st>>>(s);               \
      RS_CHECK_LAUNCH("rowgemm (specialised)");                                                  \
      return 0;                                                                                  \
    }
    RS_RGE(16, 4, 19) RS_RGE(16, 4, 3) RS_RGE(16, 4, 8) RS_RGE(16, 4, 0) RS_RGE(12, 4, 1)
    RS_RGE(4, 12, 64) RS_RGE(4, 16, 64) RS_RGE(4, 4, 0) RS_RGE(4, 4, 64) RS_RGE(4, 3, 53)
    RS_RGE(4, 3, 5) RS_RGE(4, 16, 0) RS_RGE(4, 12, 0) RS_RGE(4, 5, 53) RS_RGE(4, 5, 5)
#undef RS_RGE
  }
#define RS_RG(NTV, KTV)                                                            \
  case NTV * 100 + KTV:                                                            \
    rowgemm_kernel<NTV, KTV><<<blocks, 512, lds, st>>>(s);                          \
    break;
  switch (nt * 100 + kt) {
    RS_RG(4, 3) RS_RG(4, 4) RS_RG(4, 12) RS_RG(4, 16) RS_RG(12, 4) RS_RG(16, 4) RS_RG(3, 4)
    RS_RG(12, 16) RS_RG(2, 4) RS_RG(8, 4) RS_RG(4, 8) RS_RG(8, 8) RS_RG(16, 8)
    RS_RG(2, 3) RS_RG(2, 8) RS_RG(2, 11) RS_RG(2, 12) RS_RG(2, 16) RS_RG(4, 5) RS_RG(5, 4)
    default: set_error("rowgemm: no instance for N=%d K=%d", s.N, s.K); return -1;
  }
#undef RS_RG
  RS_CHECK_LAUNCH("rowgemm");
  return 0;
}

bool rowgemm_ln_supported(int M, int N, int K, const float* A, int lda) {
  if (N != 64 || M < kSmallM || K % 4 != 0 || lda % 4 != 0 || !aligned16(A)) return false;
  const int kt = (K + 15) / 16;
  return kt == 4 || kt == 16;
}

int rowgemm_ln_launch(const StreamArgs& s, hipStream_t st) {
  const int kt = (s.K + 15) / 16;
  RS_CHECK_ARG(s.ldc % 4 == 0 && s.ld_aux % 4 == 0 && aligned16(s.C) && aligned16(s.aux) &&
                   aligned16(s.ln_y) && aligned16(s.ln_gamma) && aligned16(s.ln_beta) &&
                   (!(s.epi & RS_EPI_BIAS) || aligned16(s.bias)),
               "rowgemm_ln: operands must be 16-byte aligned");
  const size_t lds = (size_t)4 * 16 * (kt * 16 + 4 + 3) * sizeof(float);  // + bias, gamma, beta
  const int groups = (s.M + 15) / 16;
  int bx = cdiv(groups, 16);
  const int per_cu = lds > 80 * 1024 ? 1 : (lds > 53 * 1024 ? 2 : (lds > 40 * 1024 ? 3 : 4));
  if (bx > 256 * per_cu) bx = 256 * per_cu;
  const int ekey = s.epi & (RS_EPI_BIAS | RS_EPI_DROP_A);
  if ((s.epi & RS_GEMM_BF16) && s.M % 16 == 0 && s.K % 64 == 0 && s.lda % 4 == 0 && s.ldb % 4 == 0 &&
      aligned16(s.B)) {
    const int kc = s.K / 64;
    const size_t ldsb = (size_t)64 * (s.K + 8) * 2 + (size_t)3 * 64 * 4;
    const int per_cub = ldsb > 80 * 1024 ? 1 : (ldsb > 53 * 1024 ? 2 : (ldsb > 40 * 1024 ? 3 : 4));
    // the LayerNorm-epilogue instances measured best at 2 workgroups per CU (25 groups each at
    // C2: 0.060 ms per step against 0.062 at one and 0.065 at the old 400 workgroups)
    const int bxb = stream_grid(s.M / 16, per_cub, 20);
#define RS_LNB(KCV, EV) \
  if (kc == KCV && ekey == EV) { rowgemm_bf16_kernel<4, KCV, true, EV><<<bxb, 512, ldsb, st>>>(s); RS_CHECK_LAUNCH("rowgemm_ln bf16"); return 0; }
    RS_LNB(1, 0) RS_LNB(1, 1) RS_LNB(1, 16) RS_LNB(1, 17) RS_LNB(4, 0) RS_LNB(4, 1) RS_LNB(4, 16) RS_LNB(4, 17)
#undef RS_LNB
  }
  // no instance: an error, never a silent return with h / y unwritten (round-6 advisor finding)
  RS_CHECK_ARG(kt == 4 || kt == 16, "rowgemm_ln: no instance for N=%d K=%d (K/16 must be 4 or 16)", s.N, s.K);
  if (s.M % 16 != 0 || s.K != kt * 16) {  // guarded generic instances
    if (kt == 4) rowgemm_kernel<4, 4, true><<<bx, 512, lds, st>>>(s);
    else rowgemm_kernel<4, 16, true><<<bx, 512, lds, st>>>(s);
  } else {
#define RS_LN(KTV, EV) \
  if (kt == KTV && ekey == EV) rowgemm_kernel<4, KTV, true, 1, EV><<<bx, 512, lds, st>>>(s);
    RS_LN(4, 0) else RS_LN(4, 1) else RS_LN(4, 16) else RS_LN(4, 17)
    else RS_LN(16, 0) else RS_LN(16, 1) else RS_LN(16, 16) else RS_LN(16, 17)
    else { set_error("rowgemm_ln: no instance for K=%d epilogue %d", s.K, ekey); return -1; }
#undef RS_LN
  }
  RS_CHECK_LAUNCH("rowgemm_ln");
  return 0;
}

bool wgrad_instance(int M, int N) {
  const int mo_pad = (M + 31) / 32 * 32, no_pad = (N + 31) / 32 * 32;
  switch (mo_pad * 1000 + no_pad) {
    case 64064: case 64256: case 256064: case 192064: case 64192: case 128128: case 128064:
    case 64128: case 32064: case 64032: case 128256: case 256128: case 64096: case 96064:
    case 256192:  // the user tower's first Linear (172 inputs): generic split-K GEMM + reduce was 32 us
      return true;
    default: return false;
  }
}

bool wgrad_supported(int transA, int transB, int M, int N, int K, const float* A, int lda,
                     const float* B, int ldb, int ldc, int epi) {
  if (!transA || transB || epi != 0 || K < 2048) return false;
  if (!wgrad_instance(M, N)) return false;
  if (M % 4 != 0 || N % 4 != 0 || lda % 4 != 0 || ldb % 4 != 0 || !aligned16(A) || !aligned16(B))
    return false;
  (void)ldc;
  return true;
}

int64_t wgrad_ws_bytes(int M, int N, int K) {
  return (int64_t)wgrad_blocks(K) * ((int64_t)M * N + M) * (int64_t)sizeof(float);
}

// wgrad_reduce_kernel's work as deferred jobs (reduce.hip) while the library defers reductions:
// C = alpha * sum + beta * C over the M x N partials (a contiguous C only), rowsum += alpha * sum
bool wgrad_reduce_deferred(const StreamArgs& s, int P) {
  if (!reduce_deferring() || s.ldc != s.N) return false;
  const int total = s.M * s.N;
  float* oc[1] = {s.C};
  const int b0[1] = {0};
  const float al[1] = {s.alpha}, bc[1] = {s.beta}, br[1] = {1.f};
  reduce_defer_job(s.ws, P, total, 1, oc, b0, al, bc);
  if (s.rowsum) {
    float* orow[1] = {s.rowsum};
    reduce_defer_job(s.ws + (int64_t)P * total, P, s.M, 1, orow, b0, al, br);
  }
  return true;
}

int wgrad_bf16_launch(const StreamArgs& s, bool y_bf16, bool x_bf16, hipStream_t st) {
  const int mo_pad = (s.M + 31) / 32 * 32, no_pad = (s.N + 31) / 32 * 32;
  const int nb = wgrad_blocks(s.K);
  const int rpb = cdiv(cdiv(s.K, nb), WB_BK) * WB_BK;
  const int nblk = cdiv(s.K, rpb);
  const size_t stage = (size_t)2 * WB_BK * (wb_pitch(mo_pad) + wb_pitch(no_pad)) * 2;
  const size_t red = (size_t)WB_BK * mo_pad * sizeof(float);
  const size_t lds = stage > red ? stage : red;
  const int key = (mo_pad * 1000 + no_pad) * 4 + (y_bf16 ? 2 : 0) + (x_bf16 ? 1 : 0);
#define RS_WB(MOV, NOV, YB, XB)                                                    \
  case (MOV * 1000 + NOV) * 4 + (YB ? 2 : 0) + (XB ? 1 : 0):                       \
    wgrad_bf16_kernel<MOV, NOV, YB, XB><<<nblk, 256, lds, st>>>(s, rpb);           \
    break;
  switch (key) {
    RS_WB(64, 64, false, false) RS_WB(64, 256, false, false) RS_WB(256, 64, false, false)
    RS_WB(192, 64, false, false) RS_WB(64, 192, false, false) RS_WB(128, 128, false, false)
    RS_WB(128, 64, false, false) RS_WB(64, 128, false, false) RS_WB(32, 64, false, false)
    RS_WB(64, 32, false, false) RS_WB(128, 256, false, false) RS_WB(256, 128, false, false)
    RS_WB(64, 96, false, false) RS_WB(96, 64, false, false) RS_WB(256, 192, false, false)
    RS_WB(64, 256, false, true) RS_WB(256, 64, true, false)  // the fused FFN's weight gradients
    RS_WB(192, 64, true, false)  // in_proj from the bf16 dqkv (RS_ATTN_QKV_BF16)
    default:
      set_error("wgrad bf16: no instance for %dx%d (bf16 operands %d/%d)", s.M, s.N, (int)y_bf16,
                (int)x_bf16);
      return -1;
  }
#undef RS_WB
  RS_CHECK_LAUNCH("wgrad bf16");
  if (wgrad_reduce_deferred(s, nblk)) return 0;
  const int total = s.M * s.N + (s.rowsum ? s.M : 0);
  wgrad_reduce_kernel<<<cdiv(total, 64), 1024, 0, st>>>(s, nblk);
  RS_CHECK_LAUNCH("wgrad reduce");
  return 0;
}

int wgrad_launch(const StreamArgs& s, hipStream_t st) {
  const int mo_pad = (s.M + 31) / 32 * 32, no_pad = (s.N + 31) / 32 * 32;
  const int nb = wgrad_blocks(s.K);
  const int rpb = cdiv(cdiv(s.K, nb), WG_BK) * WG_BK;
  const int nblk = cdiv(s.K, rpb);
  if (s.epi & RS_GEMM_BF16) return wgrad_bf16_launch(s, false, false, st);
  const size_t lds = (size_t)2 * WG_BK * (mo_pad + no_pad) * sizeof(float);
#define RS_WG(MOV, NOV)                                                   \
  case MOV * 1000 + NOV:                                                  \
    wgrad_kernel<MOV, NOV><<<nblk, 256, lds, st>>>(s, rpb);               \
    break;
  switch (mo_pad * 1000 + no_pad) {
    RS_WG(64, 64) RS_WG(64, 256) RS_WG(256, 64) RS_WG(192, 64) RS_WG(64, 192) RS_WG(128, 128)
    RS_WG(128, 64) RS_WG(64, 128) RS_WG(32, 64) RS_WG(64, 32) RS_WG(128, 256) RS_WG(256, 128)
    RS_WG(64, 96) RS_WG(96, 64) RS_WG(256, 192)
    default: set_error("wgrad: no instance for %dx%d", s.M, s.N); return -1;
  }
#undef RS_WG
  RS_CHECK_LAUNCH("wgrad");
  if (wgrad_reduce_deferred(s, nblk)) return 0;
  const int total = s.M * s.N + (s.rowsum ? s.M : 0);
  wgrad_reduce_kernel<<<cdiv(total, 64), 1024, 0, st>>>(s, nblk);
  RS_CHECK_LAUNCH("wgrad reduce");
  return 0;
}

}  // namespace rs
