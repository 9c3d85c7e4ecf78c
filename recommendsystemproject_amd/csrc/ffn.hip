// The Transformer layer's feed-forward block fused per 16-token row group (bf16 compute mode).
//
// Reference: nn.TransformerEncoderLayer(norm_first=False, activation=relu) inside
// SequenceEncoder (SequenceEncoder.py:17-29):
//     x2 = norm2(x1 + dropout2(linear2(dropout(relu(linear1(x1))))))
//
// Unfused, the [tokens, F = 256] inner activation f1 is the largest tensor of the step: written
// by linear1, read by linear2, by linear2's weight gradient and (as the ReLU mask) by its input
// gradient, and the same again for its gradient dPre1. Here it never reaches HBM in the forward:
//
// rs_ffn_fwd_bf16: per wave and 16-row group, f1 = drop(relu(x1 W1^T + b1)) stays in registers as
//   the bf16 operand of linear2 (the 16x16 accumulator tiles of the first product ARE the k-slices
//   of the second product's operand under a fixed k permutation, applied to W2's LDS image too),
//   followed by bias + dropout2 + residual + LayerNorm in the epilogue. Stores h2, x2, mean, rstd
//   and one bit per f1 element (kept by dropout and positive): [M][F/64] uint64 (6.5 MB at C2).
// rs_ffn_bwd_bf16: recomputes x1 W1^T + b1 on the MFMA (exactly the forward's operation order),
//   rebuilds f1 from the bits (no dropout hash in the backward), writes f1 and
//   dPre1 = (dff W2) * mask / (1 - p) as bf16 for the two weight gradients, and accumulates
//   dx1 += dPre1 W1 -- three products per row group, f1 / dPre1 never read back.
// Weight gradients: rs_wgrad_bf16 with the bf16 operands (gemm_stream.hip).
//
// Numerics are those of the bf16 compute mode (operands rounded to bf16, fp32 accumulation,
// fp32 epilogues): identical element values to the unfused bf16 path except for the summation
// order inside linear2 / dx1 (a different k permutation) and db1, which is summed from the bf16
// dPre1 (as under autocast, where the gradient reaching the bias is bf16).
#include "common.h"
#include "gemm_stream.h"
#include "rng.h"
#include "stage.h"

namespace rs {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) floatx4* gptr4;

constexpr int D = 64;      // d_model
constexpr int DP = D + 8;  // LDS pitch (bf16) of [*][D] images: conflict-free 16-byte reads

struct FfnArgs {
  int M;
  const float* x;   // [M, D] FFN input x1 (also the LayerNorm residual)
  const float* W1;  // [F, D]
  const float* b1;  // [F]
  const float* W2;  // [D, F]
  const float* b2;  // [D]
  const float* gamma;
  const float* beta;
  float eps;
  float* h;      // fwd: x1 + dropout2(linear2(.))  [M, D]
  float* y;      // fwd: LayerNorm(h)               [M, D]
  float* mean;   // fwd: [M]
  float* rstd;   // fwd: [M]
  uint64_t* mask;        // fwd: out, bwd: in -- [M][F/64] (f1 > 0 bits)
  const float* dff;      // bwd: gradient of linear2's output after dropout2's backward [M, D]
  const float* dres;     // bwd: [M, D] gradient already reaching x1 (residual path)
  float* dx;             // bwd: out [M, D] = dres + dPre1 W1 (may alias dres)
  __bf16* f1;            // bwd: out [M, F]
  __bf16* dpre;          // bwd: out [M, F]
  float p;
  const int64_t* key;
  int site1, site2;
  // bwd with the next LayerNorm's backward fused (rs_ffn_bwd_ln_bf16): the block's x1 is
  // LN1(h1); dx1 never reaches HBM, the kernel writes dh1 = LN1-backward(dx1) and
  // dsa = dropout-backward(dh1) (site ln_site), and [grid][128] dgamma | dbeta partials
  const float* ln_h;
  const float* ln_gamma;
  const float* ln_mean;
  const float* ln_rstd;
  float* ln_da;  // nullable (p == 0)
  float* ln_ws;
  int ln_site;
  // bwd with norm2's backward fused as the prologue too (rs_ffn_bwd_ln2_bf16): the kernel reads
  // the gradient of the layer output dy2 and norm2's input h2 instead of dff / dres, and writes
  // dff = dropout2-backward(dh2) for the weight gradients; [grid][128] dgamma2 | dbeta2 partials
  const float* ln2_h;
  const float* ln2_dy;
  const float* ln2_gamma;
  const float* ln2_mean;
  const float* ln2_rstd;
  float* ln2_ws;
  float* dff_out;
  int ln2_site;
};

// k permutation of a 32-wide chunk: operand slot 8q + j (lane quad q, element j) holds column
// kp(q, j) of the chunk -- the columns lane quad q owns in the two 16x16 output tiles 2c, 2c+1
__host__ __device__ constexpr int kp(int q, int j) { return j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4); }

__device__ __forceinline__ bf16x8 cvt8(const floatx4& lo, const floatx4& hi) {
  bf16x8 r;
  r[0] = (__bf16)lo[0]; r[1] = (__bf16)lo[1]; r[2] = (__bf16)lo[2]; r[3] = (__bf16)lo[3];
  r[4] = (__bf16)hi[0]; r[5] = (__bf16)hi[1]; r[6] = (__bf16)hi[2]; r[7] = (__bf16)hi[3];
  return r;
}

__device__ __forceinline__ bf16x8 lds8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// column k of a 32-wide chunk -> its slot in the k-permuted image (inverse of kp)
__host__ __device__ constexpr int kslot(int k) {
  const int kk = k & 31, c = k >> 5;
  return 32 * c + (kk < 16 ? 8 * (kk >> 2) + (kk & 3) : 8 * ((kk - 16) >> 2) + 4 + (kk & 3));
}

__device__ __forceinline__ void put4(__bf16* p, const floatx4& v) {
  bf16x4 h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = h;
}

// x [M, D] row m, columns 16q .. 16q+15 (lane quad q) as the k-fragments of a K = 64 product
__device__ __forceinline__ void load_row64(const float* base, int64_t m, int q, floatx4 (&v)[4]) {
  const float* row = base + m * D + 16 * q;
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = *(gptr4)(row + 4 * u);
}

// acc[t] = sum over the K = 64 fragments of W-image rows 16t + r (two MFMAs)
#define RS_MFMA2(ACC, IMG, PITCH, ROW, AF)                                                  \
  do {                                                                                      \
    const __bf16* bp_ = (IMG) + (ROW) * (PITCH) + 16 * q;                                   \
    ACC = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(bp_), (AF)[0], ACC, 0, 0, 0);        \
    ACC = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(bp_ + 8), (AF)[1], ACC, 0, 0, 0);    \
  } while (0)

template <int F, bool DROP>
__global__ __launch_bounds__(512) void ffn_fwd_bf16_kernel(FfnArgs a) {
  constexpr int FP = F + 8;
  constexpr int NH = F / 16, NC = F / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __bf16* W1s = reinterpret_cast<__bf16*>(smem_raw);  // [F][DP]
  __bf16* W2p = W1s + F * DP;                           // [D][FP], k-permuted
  float* sb1 = reinterpret_cast<float*>(W2p + D * FP);  // [F]
  float* sb2 = sb1 + F;                                 // [D]
  float* sg = sb2 + D;
  float* sbt = sg + D;
  // W1 [F][D] as is; W2 [D][F] with each 32-chunk's columns in kslot order (4 consecutive
  // columns stay consecutive)
  stage_batched<F, D, 512>(a.W1, D, [&](int n, int k, const floatx4& v) { put4(W1s + n * DP + k, v); });
  stage_batched<D, F, 512>(a.W2, F, [&](int n, int k, const floatx4& v) { put4(W2p + n * FP + kslot(k), v); });
  for (int i = threadIdx.x; i < F; i += blockDim.x) sb1[i] = a.b1[i];
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    sb2[i] = a.b2[i];
    sg[i] = a.gamma[i];
    sbt[i] = a.beta[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int groups = a.M / 16;  // host: M % 16 == 0
  DropKey k1{}, k2{};
  if constexpr (DROP) {
    k1 = make_key(a.key, a.site1, a.p);
    k2 = make_key(a.key, a.site2, a.p);
  }
  const int stride = gridDim.x * 8;
  int g = blockIdx.x * 8 + wave;
  floatx4 xr[4];
  if (g < groups) load_row64(a.x, (int64_t)g * 16 + r, q, xr);
  for (; g < groups; g += stride) {
    // an opaque zero offset per iteration keeps the W fragment reads inside the loop (hoisted,
    // the 64 fragments alone would take every VGPR and spill)
    int zo = 0;
    asm volatile("" : "+s"(zo));
    const __bf16* W1i = W1s + zo;
    const __bf16* W2i = W2p + zo;
    const int64_t m = (int64_t)g * 16 + r;
    floatx4 res[4];  // LayerNorm residual x1[m][16t + 4q ..]
#pragma unroll
    for (int t = 0; t < 4; ++t) res[t] = *(gptr4)(a.x + m * D + 16 * t + 4 * q);
    bf16x8 af[2] = {cvt8(xr[0], xr[1]), cvt8(xr[2], xr[3])};
    const int gn = g + stride < groups ? g + stride : g;
    load_row64(a.x, (int64_t)gn * 16 + r, q, xr);
    // dropout element indices m*F + n / m*D + n in 32 bits (host: M*F < 2^32)
    const uint32_t base1 = (uint32_t)m * F + 4 * q, base2 = (uint32_t)m * D + 4 * q;
    // linear1 + bias + relu + dropout, 4 tiles at a time, into linear2's operand fragments
    bf16x8 a2[NC];
    uint64_t bits = 0;
#pragma unroll
    for (int h0 = 0; h0 < NH; h0 += 4) {
      floatx4 acc[4];
#pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        acc[hh] = floatx4{0.f, 0.f, 0.f, 0.f};
        RS_MFMA2(acc[hh], W1i, DP, (h0 + hh) * 16 + r, af);
      }
#pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        const int h = h0 + hh, n0 = 16 * h + 4 * q;
        const floatx4 bv = *reinterpret_cast<const floatx4*>(sb1 + n0);
        float mk[4];
        if constexpr (DROP) keep4_32(k1, base1 + 16 * h, mk);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[hh][i] * 1.0f + bv[i];
          v = fmaxf(v, 0.f);
          if constexpr (DROP) v *= mk[i];
          if (v > 0.f) bits |= 1ull << (4 * h + i);
          a2[h >> 1][4 * (h & 1) + i] = (__bf16)v;
        }
      }
    }
    a.mask[m * (F / 64) + q] = bits;  // F == 256: one word per lane quad
    // linear2 over the permuted k slices
    floatx4 acc2[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc2[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc2[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(W2i + (16 * t + r) * FP + 32 * c + 8 * q),
                                                           a2[c], acc2[t], 0, 0, 0);
    // bias + dropout2 + residual + LayerNorm (same per-element order as rs_gemm_add_layernorm)
    float hv[4][4];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n0 = 16 * t + 4 * q;
      const floatx4 bv = *reinterpret_cast<const floatx4*>(sb2 + n0);
      float mk[4];
      if constexpr (DROP) keep4_32(k2, base2 + 16 * t, mk);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc2[t][e] * 1.0f + bv[e];
        if constexpr (DROP) v *= mk[e];
        hv[t][e] = v + res[t][e];
        s += hv[t][e];
      }
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mu = s / (float)D;
    float vs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = hv[t][e] - mu;
        vs += d * d;
      }
    vs += __shfl_xor(vs, 16, 64);
    vs += __shfl_xor(vs, 32, 64);
    const float rs = 1.f / sqrtf(vs / (float)D + a.eps);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n0 = 16 * t + 4 * q;
      const floatx4 gm = *reinterpret_cast<const floatx4*>(sg + n0);
      const floatx4 bt = *reinterpret_cast<const floatx4*>(sbt + n0);
      floatx4 h4, y4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h4[e] = hv[t][e];
        y4[e] = (hv[t][e] - mu) * rs * gm[e] + bt[e];
      }
      *reinterpret_cast<floatx4*>(a.h + m * D + n0) = h4;
      *reinterpret_cast<floatx4*>(a.y + m * D + n0) = y4;
    }
    if (q == 0) {
      a.mean[m] = mu;
      a.rstd[m] = rs;
    }
  }
}

// ACTS: also write f1 and dPre1 (bf16) for rs_wgrad_bf16; without them (the weight gradients
// by rs_ffn_wgrad_bf16) linear1 is not recomputed and its W1 image is not staged.
// LN2 (with LN1, !ACTS): norm2's backward is the prologue. Lane (r, q) holds row r's columns
// 16t + 4q + e (the layout of the residual add after the last product), so dh2 IS the residual
// gradient; dff = drop2(dh2) is stored (fp32, for rs_ffn_wgrad_bf16) and goes through a per-wave
// LDS tile as bf16 to reach the 16q .. 16q+15 layout of the dff W2 product's operand.
template <int F, bool LN1 = false, bool LNDROP = false, bool ACTS = true, bool LN2 = false>
__global__ __launch_bounds__(512) void ffn_bwd_bf16_kernel(FfnArgs a) {
  static_assert(!LN2 || (LN1 && !ACTS), "LN2 prologue needs the LN1 epilogue and no activations");
  constexpr int FP = F + 8;
  constexpr int NH = F / 16, NC = F / 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __bf16* W1s = reinterpret_cast<__bf16*>(smem_raw);  // [F][DP]  (x1 W1^T; ACTS only)
  __bf16* W2t = W1s + (ACTS ? F * DP : 0);              // [F][DP]  W2^T (dff W2)
  __bf16* W1t = W2t + F * DP;                           // [D][FP]  W1^T, k-permuted (dPre1 W1)
  float* sb1 = reinterpret_cast<float*>(W1t + D * FP);  // [F]
  float* sg2 = sb1 + F;                                 // [D] gamma2 (LN2)
  __bf16* dsc = reinterpret_cast<__bf16*>(sg2 + D);     // [8 waves][16][DP] dff tiles (LN2)
  if constexpr (LN2)
    for (int i = threadIdx.x; i < D; i += blockDim.x) sg2[i] = a.ln2_gamma[i];
  stage_batched<F, D, 512>(a.W1, D, [&](int n1, int k, const floatx4& v) {
    if constexpr (ACTS) put4(W1s + n1 * DP + k, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) W1t[(k + e) * FP + kslot(n1)] = (__bf16)v[e];  // W1^T, k-permuted
  });
  stage_batched<D, F, 512>(a.W2, F, [&](int n2, int n1, const floatx4& v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) W2t[(n1 + e) * DP + n2] = (__bf16)v[e];  // W2^T
  });
  for (int i = threadIdx.x; i < F; i += blockDim.x) sb1[i] = a.b1[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int groups = a.M / 16;
  const float scale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  const int stride = gridDim.x * 8;
  int g = blockIdx.x * 8 + wave;
  floatx4 xr[4], dr[4];
  // LN2: the next group's dy2 / h2 rows (t layout) and statistics, loaded one group ahead
  floatx4 pdy[LN2 ? 4 : 1], ph2[LN2 ? 4 : 1], lpg2[LN2 ? 4 : 1], lpb2[LN2 ? 4 : 1];
  float pmu2 = 0.f, prs2 = 0.f;
  DropKey ldk2{};
  if (g < groups) {
    if constexpr (ACTS) load_row64(a.x, (int64_t)g * 16 + r, q, xr);
    if constexpr (LN2) {
      const int64_t m0 = (int64_t)g * 16 + r;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        pdy[t] = *(gptr4)(a.ln2_dy + m0 * D + 16 * t + 4 * q);
        ph2[t] = *(gptr4)(a.ln2_h + m0 * D + 16 * t + 4 * q);
      }
      pmu2 = a.ln2_mean[m0];
      prs2 = a.ln2_rstd[m0];
    } else {
      load_row64(a.dff, (int64_t)g * 16 + r, q, dr);
    }
  }
  if constexpr (LN2) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      lpg2[t] = floatx4{0.f, 0.f, 0.f, 0.f};
      lpb2[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (LNDROP) ldk2 = make_key(a.key, a.ln2_site, a.p);
  }
  if constexpr (!ACTS) {  // x1 only feeds linear1's recompute
#pragma unroll
    for (int u = 0; u < 4; ++u) xr[u] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  // LN1: gamma at this lane's columns 16t + 4q + e, and its dgamma / dbeta partial sums
  floatx4 lgm[LN1 ? 4 : 1], lpg[LN1 ? 4 : 1], lpb[LN1 ? 4 : 1];
  DropKey ldk{};
  if constexpr (LN1) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      lgm[t] = *(gptr4)(a.ln_gamma + 16 * t + 4 * q);
      lpg[t] = floatx4{0.f, 0.f, 0.f, 0.f};
      lpb[t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (LNDROP) ldk = make_key(a.key, a.ln_site, a.p);
  }
  for (; g < groups; g += stride) {
    int zo = 0;
    asm volatile("" : "+s"(zo));
    const __bf16* W1i = W1s + zo;
    const __bf16* W2i = W2t + zo;
    const __bf16* W3i = W1t + zo;
    const int64_t m = (int64_t)g * 16 + r;
    floatx4 res[4];  // dres[m][16t + 4q ..] (accumulated into)
    if constexpr (!LN2) {
#pragma unroll
      for (int t = 0; t < 4; ++t) res[t] = *(gptr4)(a.dres + m * D + 16 * t + 4 * q);
    }
    floatx4 lh[LN1 ? 4 : 1];
    float lmu = 0.f, lrs = 0.f;
    if constexpr (LN1) {  // LN1 operands, issued with the residual rows
#pragma unroll
      for (int t = 0; t < 4; ++t) lh[t] = *(gptr4)(a.ln_h + m * D + 16 * t + 4 * q);
      lmu = a.ln_mean[m];
      lrs = a.ln_rstd[m];
    }
    const uint64_t bits = a.mask[m * (F / 64) + q];
    bf16x8 ax[2] = {cvt8(xr[0], xr[1]), cvt8(xr[2], xr[3])};
    bf16x8 ad[2];
    const int gn = g + stride < groups ? g + stride : g;
    if constexpr (ACTS) load_row64(a.x, (int64_t)gn * 16 + r, q, xr);
    if constexpr (LN2) {
      // norm2 backward of row m (its 64 columns in the 4 lanes r, r+16, r+32, r+48), as
      // ln_bwd64_kernel: dh2 = rstd (g - mean(g) - xhat mean(g xhat)), g = dy2 * gamma2
      floatx4 xh[4], gg[4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const floatx4 gm = *reinterpret_cast<const floatx4*>(sg2 + 16 * t + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[t][e] = (ph2[t][e] - pmu2) * prs2;
          lpg2[t][e] += pdy[t][e] * xh[t][e];
          lpb2[t][e] += pdy[t][e];
          gg[t][e] = pdy[t][e] * gm[e];
          s1 += gg[t][e];
          s2 += gg[t][e] * xh[t][e];
        }
      }
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      s1 /= 64.f;
      s2 /= 64.f;
      const float rs2 = prs2;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) res[t][e] = rs2 * (gg[t][e] - s1 - xh[t][e] * s2);
      // the current dy2 / h2 are dead: the next group's go in flight behind this one's products
      const int64_t mn = (int64_t)gn * 16 + r;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        pdy[t] = *(gptr4)(a.ln2_dy + mn * D + 16 * t + 4 * q);
        ph2[t] = *(gptr4)(a.ln2_h + mn * D + 16 * t + 4 * q);
      }
      pmu2 = a.ln2_mean[mn];
      prs2 = a.ln2_rstd[mn];
      // dff = drop2(dh2): stored for the weight gradients, and as bf16 through this wave's LDS
      // tile into the operand layout (lane quad q: columns 16q .. 16q+15 of row r)
      __bf16* tile = dsc + (wave * 16 + r) * DP;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        floatx4 f = res[t];
        if constexpr (LNDROP) {
          float mk[4];
          keep4(ldk2, (uint64_t)(m * D + 16 * t + 4 * q), mk);  // ln_bwd64_kernel's draw
#pragma unroll
          for (int e = 0; e < 4; ++e) f[e] *= mk[e];
        }
        *reinterpret_cast<floatx4*>(a.dff_out + m * D + 16 * t + 4 * q) = f;
        put4(tile + 16 * t + 4 * q, f);
      }
      // one wave writes and reads its own tile: LDS executes a wave's operations in order
      asm volatile("" ::: "memory");
      ad[0] = lds8(tile + 16 * q);
      ad[1] = lds8(tile + 16 * q + 8);
      asm volatile("" ::: "memory");
    } else {
      ad[0] = cvt8(dr[0], dr[1]);
      ad[1] = cvt8(dr[2], dr[3]);
      load_row64(a.dff, (int64_t)gn * 16 + r, q, dr);
    }
    bf16x8 a3[NC];
#pragma unroll
    for (int h0 = 0; h0 < NH; h0 += 4) {
      floatx4 acc[4], accd[4];
#pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        acc[hh] = floatx4{0.f, 0.f, 0.f, 0.f};
        accd[hh] = floatx4{0.f, 0.f, 0.f, 0.f};
        if constexpr (ACTS) RS_MFMA2(acc[hh], W1i, DP, (h0 + hh) * 16 + r, ax);
        RS_MFMA2(accd[hh], W2i, DP, (h0 + hh) * 16 + r, ad);
      }
#pragma unroll
      for (int hh = 0; hh < 4; ++hh) {
        const int h = h0 + hh, n0 = 16 * h + 4 * q;
        const floatx4 bv = *reinterpret_cast<const floatx4*>(sb1 + n0);
        bf16x4 f4, d4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool keep = (bits >> (4 * h + i)) & 1ull;
          const float pre = acc[hh][i] * 1.0f + bv[i];
          const float f = keep ? pre * scale : 0.f;  // == the forward's drop(relu(pre))
          const float d = keep ? scale * accd[hh][i] : 0.f;
          f4[i] = (__bf16)f;
          d4[i] = (__bf16)d;
          a3[h >> 1][4 * (h & 1) + i] = d4[i];
        }
        if constexpr (ACTS) {
          *reinterpret_cast<bf16x4*>(a.f1 + m * F + n0) = f4;
          *reinterpret_cast<bf16x4*>(a.dpre + m * F + n0) = d4;
        }
      }
    }
    floatx4 acc3[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc3[t] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        acc3[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds8(W3i + (16 * t + r) * FP + 32 * c + 8 * q),
                                                           a3[c], acc3[t], 0, 0, 0);
    if constexpr (!LN1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        floatx4 v = acc3[t] * 1.0f;
        v += 1.0f * res[t];
        *reinterpret_cast<floatx4*>(a.dx + m * D + 16 * t + 4 * q) = v;
      }
    } else {
      // LayerNorm backward of the row (its 64 columns sit in the 4 lanes r, r+16, r+32, r+48):
      // dh = rstd (g - mean(g) - xhat mean(g xhat)), g = dx1 * gamma
      floatx4 v[4], xh[4], gg[4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v[t] = acc3[t] * 1.0f;
        v[t] += 1.0f * res[t];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[t][e] = (lh[t][e] - lmu) * lrs;
          gg[t][e] = v[t][e] * lgm[t][e];
          s1 += gg[t][e];
          s2 += gg[t][e] * xh[t][e];
          lpg[t][e] += v[t][e] * xh[t][e];
          lpb[t][e] += v[t][e];
        }
      }
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      s1 /= 64.f;
      s2 /= 64.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        floatx4 dh;
#pragma unroll
        for (int e = 0; e < 4; ++e) dh[e] = lrs * (gg[t][e] - s1 - xh[t][e] * s2);
        *reinterpret_cast<floatx4*>(a.dx + m * D + 16 * t + 4 * q) = dh;
        if constexpr (LNDROP) {
          float mk[4];
          keep4(ldk, (uint64_t)(m * D + 16 * t + 4 * q), mk);  // rs_dropout_fwd's draw
#pragma unroll
          for (int e = 0; e < 4; ++e) dh[e] *= mk[e];
          *reinterpret_cast<floatx4*>(a.ln_da + m * D + 16 * t + 4 * q) = dh;
        }
      }
    }
  }
  if constexpr (LN1) {
    // dgamma | dbeta partials of this workgroup: fixed-order sum over the 16 rows r of each
    // lane quad and the 8 waves (the weight images are dead: the LDS is reused)
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem_raw);  // [8 waves][64 lanes][32]
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[(wave * 64 + lane) * 32 + 4 * t + e] = lpg[t][e];
        red[(wave * 64 + lane) * 32 + 16 + 4 * t + e] = lpb[t][e];
      }
    __syncthreads();
    if (threadIdx.x < 128) {
      const int st = threadIdx.x >> 6, c = threadIdx.x & 63;  // st 0: dgamma, 1: dbeta
      const int t = c >> 4, qq = (c & 15) >> 2, e = c & 3;
      float acc = 0.f;
      for (int w = 0; w < 8; ++w)
        for (int rr = 0; rr < 16; ++rr) acc += red[(w * 64 + rr + 16 * qq) * 32 + 16 * st + 4 * t + e];
      a.ln_ws[(int64_t)blockIdx.x * 128 + threadIdx.x] = acc;
    }
    if constexpr (LN2) {  // the same for norm2's dgamma2 | dbeta2 (columns in the same t layout)
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[(wave * 64 + lane) * 32 + 4 * t + e] = lpg2[t][e];
          red[(wave * 64 + lane) * 32 + 16 + 4 * t + e] = lpb2[t][e];
        }
      __syncthreads();
      if (threadIdx.x < 128) {
        const int st = threadIdx.x >> 6, c = threadIdx.x & 63;
        const int t = c >> 4, qq = (c & 15) >> 2, e = c & 3;
        float acc = 0.f;
        for (int w = 0; w < 8; ++w)
          for (int rr = 0; rr < 16; ++rr) acc += red[(w * 64 + rr + 16 * qq) * 32 + 16 * st + 4 * t + e];
        a.ln2_ws[(int64_t)blockIdx.x * 128 + threadIdx.x] = acc;
      }
    }
  }
}

// ------------------------------------------------------------------ fused weight gradients
// rs_ffn_wgrad_bf16: dW1 += dPre1^T x1, db1 += colsum(dPre1), dW2 += dff^T f1, db2 += colsum(dff)
// with f1 = drop(relu(x1 W1^T + b1)) and dPre1 = (dff W2) * mask / (1 - p) recomputed on the
// MFMA from x1, dff and the forward's bit mask -- the [M, F] activations never reach HBM (the
// unfused pair wrote them as bf16 in the backward and read them back in two rs_wgrad_bf16
// passes: 3 KB per token against 544 B here).
//
// A workgroup streams a contiguous row range in chunks of 64 rows (x1, dff rounded to bf16 into
// row-major LDS images, the mask words beside them; registers double-buffer the next chunk).
// Wave w owns the F columns n1 in [32w, 32w + 32): its W1 / W2^T fragments live in registers, it
// recomputes linear1 and dff W2 for its columns with x1 / dff as the A operand (the same k split
// as the forward and rs_ffn_bwd_bf16, so f1 and dPre1 are the same bits), which leaves the
// 16 x 16 results in exactly the operand layout of a 16x16x16 MFMA that contracts over the rows:
//   dW2[n2][n1] += dff^T (ds_read_b64_tr_b16 from the dff image) x f1 (registers),
//   dW1[n1][k]  += dPre1 (registers) x x1 (transposed read from the x1 image).
// Per workgroup partials [dW1 | dW2 | db1 | db2] go to ws in fixed order; ffn_wgrad_reduce adds
// them into the gradients (deterministic).
constexpr int WG_ROWS = 64;
constexpr int WXP = 96;  // LDS pitch (bf16) of the [64][64] images: the 4 rows of a transposed
                         // read fall in distinct 64-byte windows (wb_pitch rule)
constexpr int WG_F = 256;
constexpr int WG_OUT = 2 * WG_F * D + WG_F + D;  // dW1 [F][D], dW2 [D][F], db1 [F], db2 [D]

typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ shortx4 tr4(const __bf16* p) {
  typedef __attribute__((address_space(3))) shortx4* lptr;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(p));
}

__device__ __forceinline__ short bf16_bits(float v) { return __builtin_bit_cast(short, (__bf16)v); }

__global__ __launch_bounds__(512) void ffn_wgrad_bf16_kernel(FfnArgs a, float* ws, int rows_per_block) {
  constexpr int F = WG_F;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  __bf16* Xs = reinterpret_cast<__bf16*>(smem_raw);                      // [2][64][WXP]
  __bf16* Ds = Xs + 2 * WG_ROWS * WXP;                                    // [2][64][WXP]
  uint64_t* Ms = reinterpret_cast<uint64_t*>(Ds + 2 * WG_ROWS * WXP);      // [2][64][4]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(a.M, r0 + rows_per_block);
  const float scale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  // this wave's W fragments: column n1 = 32 wave + 16 j + r of W1 (k = 16q + 8h ..) and of W2^T
  bf16x8 w1f[2][2], w2f[2][2];
  float b1v[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n1 = 32 * wave + 16 * j + r;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float* w1 = a.W1 + n1 * D + 16 * q + 8 * h;
      const floatx4 lo = *(gptr4)(w1), hi = *(gptr4)(w1 + 4);
      w1f[j][h] = cvt8(lo, hi);
#pragma unroll
      for (int e = 0; e < 8; ++e) w2f[j][h][e] = (__bf16)a.W2[(16 * q + 8 * h + e) * F + n1];
    }
    b1v[j] = a.b1[n1];
  }
  // staging: thread slots tid, tid + 512 of x1 and of dff (64 rows x 16 float4 each), and for
  // tid < 128 two mask words (64 rows x 4 words)
  floatx4 st[4];
  u32x4 mst = {0u, 0u, 0u, 0u};
  float ysum[4] = {0.f, 0.f, 0.f, 0.f};  // colsum(dff) partials of this thread's 4 columns
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s2 = tid + 512 * (i & 1), row = c0 + s2 / 16, col = (s2 % 16) * 4;
      const float* src = i < 2 ? a.x : a.dff;
      st[i] = row < r1 ? *(gptr4)(src + (int64_t)row * D + col) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (tid < 128) {
      const int row = c0 + tid / 2;
      mst = row < r1 ? *reinterpret_cast<const u32x4*>(a.mask + (int64_t)row * 4 + 2 * (tid & 1))
                     : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s2 = tid + 512 * (i & 1), row = s2 / 16, col = (s2 % 16) * 4;
      if (i >= 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ysum[e] += st[i][e];
      }
      put4((i < 2 ? Xs : Ds) + (buf * WG_ROWS + row) * WXP + col, st[i]);
    }
    if (tid < 128) *reinterpret_cast<u32x4*>(Ms + (buf * WG_ROWS + tid / 2) * 4 + 2 * (tid & 1)) = mst;
  };
  floatx4 acc1[2][4], acc2[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc1[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
      acc2[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  // db1 = colsum(dPre1) as one more 16x16x16 product with a ones operand (every column of the
  // result holds the partial column sums)
  floatx4 accb[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
  const short one = bf16_bits(1.f);
  const shortx4 ones = {one, one, one, one};
  const int lq = (lane & 15) >> 2, lp = lane & 3;  // transposed-read row / column group
  int buf = 0;
  if (r0 < r1) {
    load_chunk(r0);
    store_chunk(0);
  }
  __syncthreads();
  for (int c0 = r0; c0 < r1; c0 += WG_ROWS) {
    const bool more = c0 + WG_ROWS < r1;
    if (more) load_chunk(c0 + WG_ROWS);
    const __bf16* X = Xs + buf * WG_ROWS * WXP;
    const __bf16* DF = Ds + buf * WG_ROWS * WXP;
    const uint64_t* MK = Ms + buf * WG_ROWS * 4;
#pragma unroll
    for (int mt = 0; mt < WG_ROWS / 16; ++mt) {
      // recompute operands: row mt*16 + r, k = 16q .. 16q + 15
      const __bf16* xrow = X + (mt * 16 + r) * WXP + 16 * q;
      const __bf16* drow = DF + (mt * 16 + r) * WXP + 16 * q;
      const bf16x8 xa0 = lds8(xrow), xa1 = lds8(xrow + 8), da0 = lds8(drow), da1 = lds8(drow + 8);
      // contraction operands over the rows: lane -> column 16t + r, rows mt*16 + 4q .. + 3
      shortx4 xt[4], dt[4];
      const int trow = mt * 16 + 4 * q + lq;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xt[t] = tr4(X + trow * WXP + 16 * t + 4 * lp);
        dt[t] = tr4(DF + trow * WXP + 16 * t + 4 * lp);
      }
      // mask words of this lane's rows 4q + e: column n1 = 16 T + r sits in word r >> 2, bit
      // 4 T + (r & 3) (the forward's layout)
      uint64_t mw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) mw[e] = MK[(mt * 16 + 4 * q + e) * 4 + (r >> 2)];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        floatx4 pre = {0.f, 0.f, 0.f, 0.f}, dpr = {0.f, 0.f, 0.f, 0.f};
        pre = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa0, w1f[j][0], pre, 0, 0, 0);
        pre = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa1, w1f[j][1], pre, 0, 0, 0);
        dpr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da0, w2f[j][0], dpr, 0, 0, 0);
        dpr = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da1, w2f[j][1], dpr, 0, 0, 0);
        const int bit = 4 * (2 * wave + j) + (r & 3);
        shortx4 f4, d4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool keep = (mw[e] >> bit) & 1ull;
          const float pv = pre[e] * 1.0f + b1v[j];
          const float f = keep ? pv * scale : 0.f;  // == rs_ffn_bwd_bf16's f1
          const float d = keep ? scale * dpr[e] : 0.f;
          f4[e] = bf16_bits(f);
          d4[e] = bf16_bits(d);
        }
        accb[j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(d4, ones, accb[j], 0, 0, 0);  // db1 (bf16 dPre1)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          acc2[j][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(dt[t], f4, acc2[j][t], 0, 0, 0);
          acc1[j][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(d4, xt[t], acc1[j][t], 0, 0, 0);
        }
      }
    }
    if (more) store_chunk(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // partials of this workgroup -> ws[block]: dW1 [n1][k], dW2 [n2][n1], db1, db2
  float* out = ws + (int64_t)blockIdx.x * WG_OUT;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int T = 2 * wave + j;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        out[(16 * T + 4 * q + e) * D + 16 * t + r] = acc1[j][t][e];
        out[F * D + (16 * t + 4 * q + e) * F + 16 * T + r] = acc2[j][t][e];
      }
  }
  if (r == 0) {  // accb rows n1 = 16 T + 4 q + e (every column alike)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[2 * F * D + 16 * (2 * wave + j) + 4 * q + e] = accb[j][e];
  }
  float* red = reinterpret_cast<float*>(smem_raw);  // the images are dead
#pragma unroll
  for (int e = 0; e < 4; ++e) red[1024 + tid * 4 + e] = ysum[e];
  __syncthreads();
  if (tid >= F && tid < F + D) {  // column c of dff: the threads 16 row + c / 4 (32 rows of slots)
    const int c = tid - F;
    float v = 0.f;
    for (int rw = 0; rw < 32; ++rw) v += red[1024 + (16 * rw + c / 4) * 4 + (c & 3)];
    out[2 * F * D + F + c] = v;
  }
}

// grad[i] += sum over the P workgroup partials of entry i, in partial order
__global__ __launch_bounds__(1024) void ffn_wgrad_reduce_kernel(const float* __restrict__ ws, int P, float* dW1,
                                                                float* dW2, float* db1, float* db2) {
  __shared__ float red[16][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63);
  const int l = threadIdx.x >> 6;
  float acc = 0.f;
  if (e < WG_OUT) {
    int p = l;
    for (; p + 16 * 7 < P; p += 16 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws[(int64_t)(p + 16 * u) * WG_OUT + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; p < P; p += 16) acc += ws[(int64_t)p * WG_OUT + e];
  }
  red[l][threadIdx.x & 63] = acc;
  __syncthreads();
  if (l != 0 || e >= WG_OUT) return;
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
  constexpr int FD = WG_F * D;
  if (e < FD) dW1[e] += t;
  else if (e < 2 * FD) dW2[e - FD] += t;
  else if (e < 2 * FD + WG_F) db1[e - 2 * FD] += t;
  else db2[e - 2 * FD - WG_F] += t;
}

int wgrad_fused_grid(int M) {
  const int chunks = cdiv(M, WG_ROWS);
  int g = cdiv(chunks, 4);  // >= 4 chunks per workgroup: the partials stay well below the reads
  // small batches (the last encoder layer's B rows: 64 chunks at B = 4096) ran 16 workgroups of 4
  // chunks one after another; one chunk per workgroup there, the partials (64 x 130 KB) are cheap
  if (g < 64) g = chunks < 64 ? chunks : 64;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}

size_t wgrad_fused_lds() { return (size_t)2 * 2 * WG_ROWS * WXP * 2 + (size_t)2 * WG_ROWS * 4 * 8; }

#undef RS_MFMA2

size_t fwd_lds(int F) { return (size_t)F * DP * 2 + (size_t)D * (F + 8) * 2 + (size_t)(F + 3 * D) * 4; }
size_t bwd_lds(int F, bool acts = true) {
  return (size_t)(acts ? 2 : 1) * F * DP * 2 + (size_t)D * (F + 8) * 2 + (size_t)F * 4;
}
// + gamma2 and the 8 waves' [16][DP] bf16 dff tiles
size_t bwd_ln2_lds(int F) { return bwd_lds(F, false) + (size_t)D * 4 + (size_t)8 * 16 * DP * 2; }

int grid_for(int M, size_t lds) {
  const int per_cu = lds > 80 * 1024 ? 1 : 2;
  int bx = cdiv(M / 16, 16);
  // small batches (the last encoder layer's B rows): one 16-row group per wave instead of 16 per
  // workgroup, while that stays under one workgroup per CU (B = 4096: 32 workgroups, not 16)
  if (bx < 256) bx = cdiv(M / 16, 8) < 256 ? cdiv(M / 16, 8) : 256;
  if (bx > 256 * per_cu) bx = 256 * per_cu;
  return bx < 1 ? 1 : bx;
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int64_t rs_ffn_mask_words(int M, int F) { return (int64_t)M * (F / 64); }

extern "C" int rs_ffn_fwd_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                               const float* W2, const float* b2, const float* gamma,
                               const float* beta, float eps, float* h, float* y, float* mean,
                               float* rstd, uint64_t* mask, float p, const int64_t* key,
                               int site1, int site2, void* stream) {
  RS_CHECK_ARG(M >= 0 && M % 16 == 0 && F == 256, "rs_ffn_fwd_bf16: need M %% 16 == 0 and F == 256 (M=%d F=%d)", M, F);
  RS_CHECK_ARG(x && W1 && b1 && W2 && b2 && gamma && beta && h && y && mean && rstd && mask,
               "rs_ffn_fwd_bf16: null operand");
  RS_CHECK_ARG(aligned16(x) && aligned16(h) && aligned16(y) && aligned16(b1) && aligned16(b2) &&
                   aligned16(gamma) && aligned16(beta),
               "rs_ffn_fwd_bf16: operands must be 16-byte aligned");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_ffn_fwd_bf16: dropout needs a key, 0 <= p < 1");
  RS_CHECK_ARG((int64_t)M * F < ((int64_t)1 << 32), "rs_ffn_fwd_bf16: M*F must be < 2^32");
  if (M == 0) return 0;
  FfnArgs a{};
  a.M = M; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.b2 = b2; a.gamma = gamma; a.beta = beta;
  a.eps = eps; a.h = h; a.y = y; a.mean = mean; a.rstd = rstd; a.mask = mask; a.p = p; a.key = key;
  a.site1 = site1; a.site2 = site2;
  const size_t lds = fwd_lds(F);
  const int bx = grid_for(M, lds);
  if (p > 0.f) ffn_fwd_bf16_kernel<256, true><<<bx, 512, lds, as_stream(stream)>>>(a);
  else ffn_fwd_bf16_kernel<256, false><<<bx, 512, lds, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_ffn_fwd_bf16");
  return 0;
}

extern "C" int64_t rs_ffn_bwd_ln_ws_bytes(int M, int F) {
  return (int64_t)grid_for(M, bwd_lds(F)) * 128 * (int64_t)sizeof(float);
}

extern "C" int rs_ffn_bwd_ln_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                                  const float* W2, const uint64_t* mask, const float* dff,
                                  const float* dres, const float* h1, const float* gamma1,
                                  const float* mean1, const float* rstd1, float* dh1, float* dsa,
                                  float* dgamma1, float* dbeta1, void* f1, void* dpre, float p,
                                  const int64_t* key, int site, float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && M % 16 == 0 && F == 256, "rs_ffn_bwd_ln_bf16: need M %% 16 == 0 and F == 256 (M=%d F=%d)", M, F);
  RS_CHECK_ARG(x && W1 && b1 && W2 && mask && dff && dres && h1 && gamma1 && mean1 && rstd1 && dh1 &&
                   dgamma1 && dbeta1 && ws && (!f1) == (!dpre),
               "rs_ffn_bwd_ln_bf16: null operand");
  RS_CHECK_ARG(dh1 != dff && dh1 != h1 && (dh1 != dres || dff != dres),
               "rs_ffn_bwd_ln_bf16: dh1 may alias dres only when dff is not dres");
  RS_CHECK_ARG(aligned16(x) && aligned16(dff) && aligned16(dres) && aligned16(dh1) && aligned16(b1) &&
                   aligned16(h1) && aligned16(gamma1) && (!dsa || aligned16(dsa)) &&
                   ((uintptr_t)f1 & 7) == 0 && ((uintptr_t)dpre & 7) == 0,
               "rs_ffn_bwd_ln_bf16: misaligned operand");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || (key && dsa)), "rs_ffn_bwd_ln_bf16: dropout needs a key and dsa, 0 <= p < 1");
  if (M == 0) return 0;
  FfnArgs a{};
  a.M = M; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.mask = const_cast<uint64_t*>(mask);
  a.dff = dff; a.dres = dres; a.dx = dh1; a.f1 = reinterpret_cast<__bf16*>(f1);
  a.dpre = reinterpret_cast<__bf16*>(dpre); a.p = p; a.key = key;
  a.ln_h = h1; a.ln_gamma = gamma1; a.ln_mean = mean1; a.ln_rstd = rstd1; a.ln_da = dsa; a.ln_ws = ws;
  a.ln_site = site;
  const bool acts = f1 != nullptr;
  const size_t lds = bwd_lds(F, acts);
  const int nb = grid_for(M, bwd_lds(F));  // the partials' count (rs_ffn_bwd_ln_ws_bytes)
  hipStream_t st = as_stream(stream);
  if (acts) {
    if (p > 0.f) ffn_bwd_bf16_kernel<256, true, true><<<nb, 512, lds, st>>>(a);
    else ffn_bwd_bf16_kernel<256, true, false><<<nb, 512, lds, st>>>(a);
  } else {
    if (p > 0.f) ffn_bwd_bf16_kernel<256, true, true, false><<<nb, 512, lds, st>>>(a);
    else ffn_bwd_bf16_kernel<256, true, false, false><<<nb, 512, lds, st>>>(a);
  }
  RS_CHECK_LAUNCH("rs_ffn_bwd_ln_bf16");
  return partials_reduce2(ws, nb, 128, 64, 1.f, 1.f, dgamma1, dbeta1, st);
}

extern "C" int64_t rs_ffn_bwd_ln2_ws_bytes(int M, int F) { return 2 * rs_ffn_bwd_ln_ws_bytes(M, F); }

extern "C" int rs_ffn_bwd_ln2_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                                   const float* W2, const uint64_t* mask, const float* dy2,
                                   const float* h2, const float* gamma2, const float* mean2,
                                   const float* rstd2, float* dff, float* dgamma2, float* dbeta2,
                                   const float* h1, const float* gamma1, const float* mean1,
                                   const float* rstd1, float* dh1, float* dsa, float* dgamma1,
                                   float* dbeta1, float p, const int64_t* key, int site1, int site2,
                                   float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && M % 16 == 0 && F == 256, "rs_ffn_bwd_ln2_bf16: need M %% 16 == 0 and F == 256 (M=%d F=%d)", M, F);
  RS_CHECK_ARG(x && W1 && b1 && W2 && mask && dy2 && h2 && gamma2 && mean2 && rstd2 && dff && dgamma2 &&
                   dbeta2 && h1 && gamma1 && mean1 && rstd1 && dh1 && dgamma1 && dbeta1 && ws,
               "rs_ffn_bwd_ln2_bf16: null operand");
  // each 16-row group is read and written by one wave: only dh1 may alias dy2
  RS_CHECK_ARG(dff != dy2 && dff != h2 && dff != h1 && dff != dh1 && dff != dsa && dh1 != h2 && dh1 != h1 &&
                   (!dsa || (dsa != dy2 && dsa != h2 && dsa != h1 && dsa != dh1)),
               "rs_ffn_bwd_ln2_bf16: overlapping outputs");
  RS_CHECK_ARG(aligned16(x) && aligned16(dy2) && aligned16(h2) && aligned16(dff) && aligned16(dh1) &&
                   aligned16(b1) && aligned16(h1) && aligned16(gamma1) && aligned16(gamma2) &&
                   (!dsa || aligned16(dsa)),
               "rs_ffn_bwd_ln2_bf16: misaligned operand");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || (key && dsa)), "rs_ffn_bwd_ln2_bf16: dropout needs a key and dsa, 0 <= p < 1");
  if (M == 0) return 0;
  FfnArgs a{};
  a.M = M; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.mask = const_cast<uint64_t*>(mask);
  a.dx = dh1; a.p = p; a.key = key;
  a.ln_h = h1; a.ln_gamma = gamma1; a.ln_mean = mean1; a.ln_rstd = rstd1; a.ln_da = dsa; a.ln_site = site1;
  a.ln2_h = h2; a.ln2_dy = dy2; a.ln2_gamma = gamma2; a.ln2_mean = mean2; a.ln2_rstd = rstd2;
  a.dff_out = dff; a.ln2_site = site2;
  const int nb = grid_for(M, bwd_lds(F));  // the partials' count (rs_ffn_bwd_ln2_ws_bytes)
  a.ln_ws = ws;
  a.ln2_ws = ws + (int64_t)nb * 128;
  const size_t lds = bwd_ln2_lds(F);
  hipStream_t st = as_stream(stream);
  if (p > 0.f) ffn_bwd_bf16_kernel<256, true, true, false, true><<<nb, 512, lds, st>>>(a);
  else ffn_bwd_bf16_kernel<256, true, false, false, true><<<nb, 512, lds, st>>>(a);
  RS_CHECK_LAUNCH("rs_ffn_bwd_ln2_bf16");
  // both LayerNorms' gamma / beta partials in one reduce launch (same order of operations per job)
  return partials_reduce2x2(ws, a.ln2_ws, nb, 128, 64, 1.f, 1.f, dgamma1, dbeta1, dgamma2, dbeta2, st);
}

extern "C" int rs_ffn_bwd_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                               const float* W2, const uint64_t* mask, const float* dff,
                               const float* dres, float* dx, void* f1, void* dpre, float p,
                               void* stream) {
  RS_CHECK_ARG(M >= 0 && M % 16 == 0 && F == 256, "rs_ffn_bwd_bf16: need M %% 16 == 0 and F == 256 (M=%d F=%d)", M, F);
  RS_CHECK_ARG(x && W1 && b1 && W2 && mask && dff && dres && dx && (!f1) == (!dpre),
               "rs_ffn_bwd_bf16: null operand");
  RS_CHECK_ARG(dx != dff || dx == dres, "rs_ffn_bwd_bf16: dx may alias dres only");
  RS_CHECK_ARG(aligned16(x) && aligned16(dff) && aligned16(dres) && aligned16(dx) && aligned16(b1) &&
                   ((uintptr_t)f1 & 7) == 0 && ((uintptr_t)dpre & 7) == 0,
               "rs_ffn_bwd_bf16: misaligned operand");
  RS_CHECK_ARG(p >= 0.f && p < 1.f, "rs_ffn_bwd_bf16: 0 <= p < 1");
  if (M == 0) return 0;
  FfnArgs a{};
  a.M = M; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.mask = const_cast<uint64_t*>(mask);
  a.dff = dff; a.dres = dres; a.dx = dx; a.f1 = reinterpret_cast<__bf16*>(f1); a.dpre = reinterpret_cast<__bf16*>(dpre);
  a.p = p;
  const bool acts = f1 != nullptr;
  const size_t lds = bwd_lds(F, acts);
  if (acts) ffn_bwd_bf16_kernel<256><<<grid_for(M, lds), 512, lds, as_stream(stream)>>>(a);
  else ffn_bwd_bf16_kernel<256, false, false, false><<<grid_for(M, lds), 512, lds, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_ffn_bwd_bf16");
  return 0;
}

extern "C" int64_t rs_ffn_wgrad_ws_bytes(int M, int F) {
  return F == 256 && M > 0 ? (int64_t)wgrad_fused_grid(M) * WG_OUT * (int64_t)sizeof(float) : 0;
}

extern "C" int rs_ffn_wgrad_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                                 const float* W2, const uint64_t* mask, const float* dff, float p,
                                 float* dW1, float* db1, float* dW2, float* db2, float* ws, void* stream) {
  RS_CHECK_ARG(M >= 0 && M % 16 == 0 && F == 256, "rs_ffn_wgrad_bf16: need M %% 16 == 0 and F == 256 (M=%d F=%d)", M, F);
  RS_CHECK_ARG(x && W1 && b1 && W2 && mask && dff && dW1 && db1 && dW2 && db2 && (ws || M == 0),
               "rs_ffn_wgrad_bf16: null operand");
  RS_CHECK_ARG(aligned16(x) && aligned16(dff) && aligned16(W1) && aligned16(mask),
               "rs_ffn_wgrad_bf16: misaligned operand");
  RS_CHECK_ARG(p >= 0.f && p < 1.f, "rs_ffn_wgrad_bf16: 0 <= p < 1");
  if (M == 0) return 0;
  FfnArgs a{};
  a.M = M; a.x = x; a.W1 = W1; a.b1 = b1; a.W2 = W2; a.mask = const_cast<uint64_t*>(mask); a.dff = dff;
  a.p = p;
  const int G = wgrad_fused_grid(M);
  const int rpb = cdiv(cdiv(M, WG_ROWS), G) * WG_ROWS;
  hipStream_t st = as_stream(stream);
  ffn_wgrad_bf16_kernel<<<cdiv(M, rpb), 512, wgrad_fused_lds(), st>>>(a, ws, rpb);
  RS_CHECK_LAUNCH("rs_ffn_wgrad_bf16");
  if (reduce_deferring()) {  // queued for rs_reduce_flush: dW1 | dW2 | db1 | db2 += the column sums
    constexpr int FD = WG_F * D;
    float* outs[4] = {dW1, dW2, db1, db2};
    const int begins[4] = {0, FD, 2 * FD, 2 * FD + WG_F};
    const float al[4] = {1.f, 1.f, 1.f, 1.f}, be[4] = {1.f, 1.f, 1.f, 1.f};
    reduce_defer_job(ws, cdiv(M, rpb), WG_OUT, 4, outs, begins, al, be);
    return 0;
  }
  ffn_wgrad_reduce_kernel<<<cdiv(WG_OUT, 64), 1024, 0, st>>>(ws, cdiv(M, rpb), dW1, dW2, db1, db2);
  RS_CHECK_LAUNCH("rs_ffn_wgrad_bf16 reduce");
  return 0;
}

extern "C" int64_t rs_wgrad_ws_bytes(int Mo, int No, int rows) { return wgrad_ws_bytes(Mo, No, rows); }

extern "C" int rs_wgrad_bf16(int rows, int Mo, int No, const void* dy, int ldy, int dy_bf16,
                             const void* x, int ldx, int x_bf16, float beta, float* dW, int ldw,
                             float* db, float* ws, void* stream) {
  RS_CHECK_ARG(rows >= 0 && Mo > 0 && No > 0 && dy && x && dW && ws && ldw >= No && ldy >= Mo && ldx >= No,
               "rs_wgrad_bf16: bad arguments");
  const int ey = dy_bf16 ? 2 : 4, ex = x_bf16 ? 2 : 4;
  RS_CHECK_ARG(aligned16(dy) && aligned16(x) && (ldy * ey) % 16 == 0 && (ldx * ex) % 16 == 0 &&
                   (Mo * ey) % 16 == 0 && (No * ex) % 16 == 0,
               "rs_wgrad_bf16: rows must be 16-byte aligned and a whole number of 16-byte slots");
  StreamArgs s{};
  s.M = Mo; s.N = No; s.K = rows; s.alpha = 1.f; s.beta = beta;
  s.A = reinterpret_cast<const float*>(dy); s.lda = ldy;
  s.B = reinterpret_cast<const float*>(x); s.ldb = ldx;
  s.C = dW; s.ldc = ldw; s.epi = RS_GEMM_BF16; s.rowsum = db; s.ws = ws; s.transB = 0;
  return wgrad_bf16_launch(s, dy_bf16 != 0, x_bf16 != 0, as_stream(stream));
}
