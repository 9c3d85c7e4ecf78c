// Self-attention for ONE query row per sample: the final encoder layer.
//
// SequenceEncoder.forward returns context[b, clamp(sum(valid) - 1, 0)] only
// (SequenceEncoder.py:58-74, trap T7), so in the last TransformerEncoderLayer every other query
// row is dead: its value never reaches the loss and its gradient is exactly zero. The final layer
// therefore needs attention for the selected query i_b = last[b] over all L keys / values, and
// its backward produces dQ for that row only while dK / dV stay dense (every valid key
// contributed to the selected row).
//
// One wave per (sample, head), one lane per key (chunks of 64 keys, L <= 256): scores, softmax,
// dropout and P V reduce across the wave. Work is B H L hd; bytes are K / V rows (+ the writes of
// dqkv in the backward), so these kernels are HBM-bound on qkv. Dropout draws are those of
// rs_attn_fwd for element ((b H + h) L + i_b) L + j. With RS_GEMM_BF16 the operands are rounded to
// bf16 where the MFMA kernels round them (q, k, v, dO, P∘Z, dS), products accumulate in fp32.
#include <type_traits>

#include "common.h"
#include "rng.h"

namespace rs {
namespace {

constexpr int kMaxChunks = 4;  // L <= 256

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float r16(float x) { return (float)(__bf16)x; }

// Wave totals of HD per-lane channels, transposed: each butterfly step halves the channels a lane
// carries (it keeps the half its partner does not), so HD + log2(64 / HD) - 1 shuffles replace
// wsum's 6 HD (96 at head_dim 16). Lane l ends with the total of channel l >> RowShift<HD>.
template <int HD>
struct RowShift { static constexpr int v = HD == 8 ? 3 : (HD == 16 ? 2 : (HD == 32 ? 1 : 0)); };
template <int HD>
__device__ __forceinline__ float wsum_t(float (&x)[HD], int lane) {
  constexpr int NS = 6 - RowShift<HD>::v;  // log2(HD) halving steps over lane bits 5, 4, ...
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int M = 32 >> s, h = HD >> (s + 1);
    const bool hi = (lane & M) != 0;
#pragma unroll
    for (int j = 0; j < h; ++j) {
      float a = x[j], b = x[j + h];
      // (empty asm: keeps the two selects on values -- folded into one select of the array index,
      // they became a compare/select chain over all HD registers per access)
      asm("" : "+v"(a), "+v"(b));
      x[j] = (hi ? b : a) + __shfl_xor(hi ? a : b, M, 64);
    }
  }
  float v = x[0];
#pragma unroll
  for (int s = 0; s < RowShift<HD>::v; ++s) v += __shfl_xor(v, (32 / HD) >> s, 64);
  return v;
}

// HD consecutive elements of a qkv row slice, fp32 or bf16 storage (HD % 4 == 0)
template <int HD>
__device__ __forceinline__ void ldrow(const float* p, float (&x)[HD]) {
#pragma unroll
  for (int c = 0; c < HD; c += 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + c);
    x[c] = v.x; x[c + 1] = v.y; x[c + 2] = v.z; x[c + 3] = v.w;
  }
}
typedef __bf16 bf4r __attribute__((ext_vector_type(4)));
template <int HD>
__device__ __forceinline__ void ldrow(const __bf16* p, float (&x)[HD]) {
#pragma unroll
  for (int c = 0; c < HD; c += 4) {
    const bf4r v = *reinterpret_cast<const bf4r*>(p + c);
    x[c] = (float)v[0]; x[c + 1] = (float)v[1]; x[c + 2] = (float)v[2]; x[c + 3] = (float)v[3];
  }
}
template <int HD>
__device__ __forceinline__ void strow(float* p, const float (&x)[HD]) {
#pragma unroll
  for (int c = 0; c < HD; c += 4)
    *reinterpret_cast<float4*>(p + c) = make_float4(x[c], x[c + 1], x[c + 2], x[c + 3]);
}
template <int HD>
__device__ __forceinline__ void strow(__bf16* p, const float (&x)[HD]) {
#pragma unroll
  for (int c = 0; c < HD; c += 4) {
    bf4r v;
    v[0] = (__bf16)x[c]; v[1] = (__bf16)x[c + 1]; v[2] = (__bf16)x[c + 2]; v[3] = (__bf16)x[c + 3];
    *reinterpret_cast<bf4r*>(p + c) = v;
  }
}

template <int HD, bool DROP, bool BF, bool QB>
__global__ __launch_bounds__(256) void attn_rows_fwd_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad,
    const int64_t* __restrict__ last, float* __restrict__ out, float* __restrict__ lse, int B,
    int L, int d, int H, float scale, float pdrop, const int64_t* __restrict__ key, int site) {
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;  // whole wave
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * HD;
  const int i = (int)last[b];
  float q[HD];
  ldrow<HD>(base + (int64_t)i * ld, q);  // same address in every lane: one broadcast line
  if (BF)
#pragma unroll
    for (int c = 0; c < HD; ++c) q[c] = r16(q[c]);
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const int nch = (L + 63) / 64;
  float s[kMaxChunks];
  float m = -INFINITY;
#pragma unroll
  for (int ch = 0; ch < kMaxChunks; ++ch) {
    s[ch] = -INFINITY;
    const int j = ch * 64 + lane;
    if (ch < nch && j < L && key_pad[(int64_t)b * L + j] == 0) {
      float k[HD];
      ldrow<HD>(base + (int64_t)j * ld + d, k);
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < HD; ++c) acc += q[c] * (BF ? r16(k[c]) : k[c]);
      s[ch] = acc * scale;
      m = fmaxf(m, s[ch]);
    }
  }
  m = wmax(m);
  float l = 0.f, o[HD];
#pragma unroll
  for (int c = 0; c < HD; ++c) o[c] = 0.f;
#pragma unroll
  for (int ch = 0; ch < kMaxChunks; ++ch) {
    const int j = ch * 64 + lane;
    if (ch < nch && s[ch] != -INFINITY) {
      const float p = expf(s[ch] - m);
      l += p;
      float pz = DROP ? p * keep_mult(dk, ((uint64_t)bh * L + i) * L + j) : p;
      if (BF) pz = r16(pz);
      float v[HD];
      ldrow<HD>(base + (int64_t)j * ld + 2 * d, v);
#pragma unroll
      for (int c = 0; c < HD; ++c) o[c] += pz * (BF ? r16(v[c]) : v[c]);
    }
  }
  l = wsum(l);
  const float inv = 1.f / l;
  const float oc = wsum_t<HD>(o, lane) * inv;  // channel lane >> RowShift
  constexpr int SH = RowShift<HD>::v;
  if ((lane & ((1 << SH) - 1)) == 0) out[(int64_t)b * d + h * HD + (lane >> SH)] = oc;
  if (lane == 0) lse[bh] = m + logf(l);
}

template <int HD, bool DROP, bool BF, bool QB>
__global__ __launch_bounds__(256) void attn_rows_bwd_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad,
    const int64_t* __restrict__ last, const float* __restrict__ dout,
    const float* __restrict__ lse, void* __restrict__ dqkv_, int B, int L, int d, int H,
    float scale, float pdrop, const int64_t* __restrict__ key, int site) {
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * HD;
  QT* dbase = reinterpret_cast<QT*>(dqkv_) + (int64_t)b * L * ld + h * HD;
  const int i = (int)last[b];
  float q[HD], g[HD];
  ldrow<HD>(base + (int64_t)i * ld, q);
  ldrow<HD>(dout + (int64_t)b * d + h * HD, g);
  if (BF)
#pragma unroll
    for (int c = 0; c < HD; ++c) { q[c] = r16(q[c]); g[c] = r16(g[c]); }
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const float lsev = lse[bh];
  const int nch = (L + 63) / 64;
  float p[kMaxChunks], z[kMaxChunks], dpt[kMaxChunks];
  float Dp = 0.f;
#pragma unroll
  for (int ch = 0; ch < kMaxChunks; ++ch) {
    p[ch] = 0.f; z[ch] = 1.f; dpt[ch] = 0.f;
    const int j = ch * 64 + lane;
    if (ch < nch && j < L && key_pad[(int64_t)b * L + j] == 0) {
      float k[HD], v[HD];
      ldrow<HD>(base + (int64_t)j * ld + d, k);
      ldrow<HD>(base + (int64_t)j * ld + 2 * d, v);
      float sa = 0.f, da = 0.f;
#pragma unroll
      for (int c = 0; c < HD; ++c) {
        sa += q[c] * (BF ? r16(k[c]) : k[c]);
        da += g[c] * (BF ? r16(v[c]) : v[c]);
      }
      p[ch] = expf(sa * scale - lsev);
      z[ch] = DROP ? keep_mult(dk, ((uint64_t)bh * L + i) * L + j) : 1.f;
      dpt[ch] = da;
      Dp += p[ch] * z[ch] * da;
    }
  }
  // D_i = sum_j P_ij dP_ij (= dO_i . O_i)
  const float D = wsum(Dp);
  float dq[HD];
#pragma unroll
  for (int c = 0; c < HD; ++c) dq[c] = 0.f;
  // H == 4 (the encoder's four heads, d = 4 HD <= 64): the workgroup's waves are the four heads of
  // sample b, so each chunk's rows of dqkv are staged in LDS and the workgroup stores them as
  // whole rows (3d contiguous elements, 16-byte stores) -- per lane, the 8-byte pieces of 64
  // different rows per store instruction were the kernel's cost (C5: 0.175 ms per step)
  constexpr bool CO = HD <= 16;
  constexpr int SP = 12 * HD + 16 / (int)sizeof(QT);  // staged row pitch: 3d elements + 16 B
  __shared__ __attribute__((aligned(16))) QT St[CO ? 64 : 1][CO ? SP : 1];
  const bool coop = CO && H == 4;  // uniform over the workgroup (B H is a multiple of 4)
#pragma unroll
  for (int ch = 0; ch < kMaxChunks; ++ch) {
    const int j = ch * 64 + lane;
    if (ch < nch && j < L) {
      float ds = p[ch] * (z[ch] * dpt[ch] - D);  // 0 for masked keys (p = 0)
      float pz = p[ch] * z[ch];
      if (BF) { ds = r16(ds); pz = r16(pz); }
      float k[HD], dk_[HD], dv[HD], zero[HD];
      ldrow<HD>(base + (int64_t)j * ld + d, k);
#pragma unroll
      for (int c = 0; c < HD; ++c) {
        dq[c] += ds * (BF ? r16(k[c]) : k[c]);
        dk_[c] = ds * q[c] * scale;
        dv[c] = pz * g[c];
        zero[c] = 0.f;
      }
      if (coop) {
        QT* sr = &St[lane][h * HD];
        strow<HD>(sr, zero);  // dead query rows: zero gradient (the selected row's is not stored)
        strow<HD>(sr + d, dk_);
        strow<HD>(sr + 2 * d, dv);
      } else {
        QT* row = dbase + (int64_t)j * ld;
        if (j != i) strow<HD>(row, zero);  // dead query rows: zero gradient
        strow<HD>(row + d, dk_);
        strow<HD>(row + 2 * d, dv);
      }
    }
    if (CO && coop && ch < nch) {
      __syncthreads();
      constexpr int CPR = 12 * HD * (int)sizeof(QT) / 16;  // 16-byte chunks per row
      constexpr int QCH = CPR / 3;                          // ... of its dQ part
      const int r0 = ch * 64, nr = min(64, L - r0);
      QT* orow = reinterpret_cast<QT*>(dqkv_) + ((int64_t)b * L + r0) * ld;
      for (int e = threadIdx.x; e < nr * CPR; e += 256) {
        const int r = e / CPR, kc = e - r * CPR;
        if (r0 + r == i && kc < QCH) continue;  // the selected row's dQ: stored below
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(orow + (int64_t)r * ld) + 16 * kc) =
            *reinterpret_cast<const uint4*>(reinterpret_cast<const unsigned char*>(&St[r][0]) + 16 * kc);
      }
      __syncthreads();
    }
  }
  const float dqc = wsum_t<HD>(dq, lane) * scale;  // channel lane >> RowShift
  constexpr int SH = RowShift<HD>::v;
  if ((lane & ((1 << SH) - 1)) == 0) dbase[(int64_t)i * ld + (lane >> SH)] = (QT)dqc;
}

}  // namespace
}  // namespace rs

using namespace rs;

#define RS_ROWS_DISPATCH(KERNEL, ...)                                                             \
  do {                                                                                            \
    const dim3 grid(cdiv((int64_t)B * H, 4));                                                     \
    const int key_ = (hd == 8 ? 0 : hd == 16 ? 1 : hd == 32 ? 2 : 3) * 8 + (p > 0.f) * 4 + bf * 2 + qb; \
    switch (key_) {                                                                               \
      RS_ROWS_CASE(KERNEL, 8, 0, __VA_ARGS__) RS_ROWS_CASE(KERNEL, 16, 1, __VA_ARGS__)            \
      RS_ROWS_CASE(KERNEL, 32, 2, __VA_ARGS__) RS_ROWS_CASE(KERNEL, 64, 3, __VA_ARGS__)           \
      default: break;                                                                             \
    }                                                                                             \
  } while (0)
#define RS_ROWS_CASE(KERNEL, HDV, HI, ...)                                                        \
  case HI * 8 + 0: KERNEL<HDV, false, false, false><<<grid, 256, 0, st>>>(__VA_ARGS__); break;    \
  case HI * 8 + 2: KERNEL<HDV, false, true, false><<<grid, 256, 0, st>>>(__VA_ARGS__); break;     \
  case HI * 8 + 3: KERNEL<HDV, false, true, true><<<grid, 256, 0, st>>>(__VA_ARGS__); break;      \
  case HI * 8 + 4: KERNEL<HDV, true, false, false><<<grid, 256, 0, st>>>(__VA_ARGS__); break;     \
  case HI * 8 + 6: KERNEL<HDV, true, true, false><<<grid, 256, 0, st>>>(__VA_ARGS__); break;      \
  case HI * 8 + 7: KERNEL<HDV, true, true, true><<<grid, 256, 0, st>>>(__VA_ARGS__); break;

static int rows_check(const void* qkv, int B, int L, int d, int H, float p, const int64_t* key,
                      int flags, const char* fn) {
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1 && d % H == 0, "%s: bad shape", fn);
  RS_CHECK_ARG(L <= 64 * kMaxChunks, "%s: L=%d > %d", fn, L, 64 * kMaxChunks);
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "%s: bad dropout p=%f", fn, p);
  const int hd = d / H;
  RS_CHECK_ARG(hd == 8 || hd == 16 || hd == 32 || hd == 64, "%s: head_dim %d unsupported", fn, hd);
  RS_CHECK_ARG(!(flags & RS_ATTN_QKV_BF16) || (flags & RS_GEMM_BF16),
               "%s: bf16 qkv storage needs RS_GEMM_BF16", fn);
  RS_CHECK_ARG(aligned16(qkv) && d % 8 == 0, "%s: needs 16-byte aligned rows", fn);
  return 0;
}

extern "C" int rs_attn_rows_fwd(const float* qkv, const uint8_t* key_pad, const int64_t* last,
                                float* out, float* lse, int B, int L, int d, int H, float scale,
                                float p, const int64_t* key, int site, int flags, void* stream) {
  RS_CHECK_ARG(qkv && key_pad && last && out && lse, "rs_attn_rows_fwd: null pointer");
  RS_RET_IF(rows_check(qkv, B, L, d, H, p, key, flags, "rs_attn_rows_fwd"));
  RS_CHECK_ARG(aligned16(out), "rs_attn_rows_fwd: out must be 16-byte aligned");
  if (B == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int hd = d / H, bf = (flags & RS_GEMM_BF16) != 0, qb = (flags & RS_ATTN_QKV_BF16) != 0;
  RS_ROWS_DISPATCH(attn_rows_fwd_kernel, qkv, key_pad, last, out, lse, B, L, d, H, scale, p, key, site);
  RS_CHECK_LAUNCH("rs_attn_rows_fwd");
  return 0;
}

extern "C" int rs_attn_rows_bwd(const float* qkv, const uint8_t* key_pad, const int64_t* last,
                                const float* dout, const float* lse, float* dqkv, int B, int L,
                                int d, int H, float scale, float p, const int64_t* key, int site,
                                int flags, void* stream) {
  RS_CHECK_ARG(qkv && key_pad && last && dout && lse && dqkv, "rs_attn_rows_bwd: null pointer");
  RS_RET_IF(rows_check(qkv, B, L, d, H, p, key, flags, "rs_attn_rows_bwd"));
  RS_CHECK_ARG(aligned16(dout) && aligned16(dqkv), "rs_attn_rows_bwd: needs 16-byte aligned rows");
  if (B == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int hd = d / H, bf = (flags & RS_GEMM_BF16) != 0, qb = (flags & RS_ATTN_QKV_BF16) != 0;
  RS_ROWS_DISPATCH(attn_rows_bwd_kernel, qkv, key_pad, last, dout, lse, dqkv, B, L, d, H, scale, p,
                   key, site);
  RS_CHECK_LAUNCH("rs_attn_rows_bwd");
  return 0;
}
