// Masked multi-head self-attention core of the user-behaviour encoder (K6): the SDPA math path
// of nn.MultiheadAttention inside nn.TransformerEncoderLayer (SequenceEncoder.py:17-29), with
// the key-padding mask built from the first sequence feature (SequenceEncoder.py:36-46).
//
// Shapes on the hot path are tiny per (sample, head) — L <= 200 keys, head_dim 16 — so one
// workgroup owns one (sample, head): its K and V slices (L x hd fp32, 6.4 KB at L = 50) sit in
// LDS, one lane owns one query row and keeps q, the running output and the softmax statistics
// in registers; every K/V row read is an LDS broadcast. Scores never touch HBM; the forward
// saves only the per-row log-sum-exp (flash-style), the backward recomputes P from it.
//   fwd  HBM: qkv slice in (3*L*hd*4 B) + out (L*hd*4 B) + lse
//   bwd  two passes over the (query, key) pairs: lane-per-query for dQ, lane-per-key for dK/dV.
#include "common.h"
#include "rng.h"

namespace rs {
namespace {

// Workgroup -> (sample, head): the H heads of one sample read interleaved 64-byte slices of the
// same qkv rows, so they are placed on the same XCD (workgroups are dealt round-robin over the
// 8 XCDs: ids b and b+8 share one) and next to each other in dispatch order, which keeps each
// 128-byte line in one L2 instead of fetching it once per head from HBM. Speed only: any
// placement gives the same result. Returns false for padding workgroups.
__device__ __forceinline__ bool map_bh(int B, int H, int& b, int& h) {
  const int bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3;
  b = (slot / H) * 8 + xcd;
  h = slot % H;
  return b < B;
}

__host__ inline int bh_grid(int B, int H) { return ((B + 7) / 8) * 8 * H; }

template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ qkv,
                                                       const uint8_t* __restrict__ key_pad,
                                                       float* __restrict__ out,
                                                       float* __restrict__ lse, int B, int L,
                                                       int d, int H, float scale, float pdrop,
                                                       const int64_t* __restrict__ key, int site) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ks = smem;                // [L][HD]
  float* Vs = Ks + L * HD;         // [L][HD]
  float* msk = Vs + L * HD;        // [L] 1 = masked
  int b, h;
  if (!map_bh(B, H, b, h)) return;
  const int bh = b * H + h;
  const int ld = 3 * d;
  const float* base = qkv + (int64_t)b * L * ld;
  for (int e = threadIdx.x; e < L * HD / 4; e += blockDim.x) {
    const int j = e / (HD / 4), c = (e % (HD / 4)) * 4;
    *reinterpret_cast<float4*>(&Ks[j * HD + c]) =
        *reinterpret_cast<const float4*>(&base[(int64_t)j * ld + d + h * HD + c]);
    *reinterpret_cast<float4*>(&Vs[j * HD + c]) =
        *reinterpret_cast<const float4*>(&base[(int64_t)j * ld + 2 * d + h * HD + c]);
  }
  for (int j = threadIdx.x; j < L; j += blockDim.x) msk[j] = key_pad[(int64_t)b * L + j] ? 1.f : 0.f;
  __syncthreads();
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);

  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    float q[HD];
    const float* qp = base + (int64_t)i * ld + h * HD;
#pragma unroll
    for (int c = 0; c < HD; ++c) q[c] = qp[c];
    float m = -INFINITY;
    for (int j = 0; j < L; ++j) {
      if (msk[j] != 0.f) continue;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < HD; ++c) s += q[c] * Ks[j * HD + c];
      m = fmaxf(m, s * scale);
    }
    float l = 0.f, o[HD];
#pragma unroll
    for (int c = 0; c < HD; ++c) o[c] = 0.f;
    for (int j = 0; j < L; ++j) {
      if (msk[j] != 0.f) continue;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < HD; ++c) s += q[c] * Ks[j * HD + c];
      const float p = expf(s * scale - m);
      l += p;
      // attention-probability dropout acts on softmax(s) (= p / l): scale the V weight only
      const float pz = DROP ? p * keep_mult(dk, ((uint64_t)bh * L + i) * L + j) : p;
#pragma unroll
      for (int c = 0; c < HD; ++c) o[c] += pz * Vs[j * HD + c];
    }
    const float inv = 1.f / l;
    float* op = out + ((int64_t)b * L + i) * d + h * HD;
#pragma unroll
    for (int c = 0; c < HD; ++c) op[c] = o[c] * inv;
    lse[(int64_t)bh * L + i] = m + logf(l);
  }
}

template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const float* __restrict__ qkv,
                                                       const uint8_t* __restrict__ key_pad,
                                                       const float* __restrict__ out,
                                                       const float* __restrict__ dout,
                                                       const float* __restrict__ lse,
                                                       float* __restrict__ dqkv, int B, int L,
                                                       int d, int H, float scale, float pdrop,
                                                       const int64_t* __restrict__ key, int site) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Qs = smem;                 // [L][HD]
  float* Ks = Qs + L * HD;
  float* Vs = Ks + L * HD;
  float* Gs = Vs + L * HD;          // dO
  float* Ls = Gs + L * HD;          // lse [L]
  float* Ds = Ls + L;               // delta [L]
  float* msk = Ds + L;              // [L]
  int b, h;
  if (!map_bh(B, H, b, h)) return;
  const int bh = b * H + h;
  const int ld = 3 * d;
  const float* base = qkv + (int64_t)b * L * ld;
  for (int e = threadIdx.x; e < L * HD / 4; e += blockDim.x) {
    const int j = e / (HD / 4), c = (e % (HD / 4)) * 4;
    const float* row = base + (int64_t)j * ld + h * HD + c;
    *reinterpret_cast<float4*>(&Qs[j * HD + c]) = *reinterpret_cast<const float4*>(row);
    *reinterpret_cast<float4*>(&Ks[j * HD + c]) = *reinterpret_cast<const float4*>(row + d);
    *reinterpret_cast<float4*>(&Vs[j * HD + c]) = *reinterpret_cast<const float4*>(row + 2 * d);
    *reinterpret_cast<float4*>(&Gs[j * HD + c]) =
        *reinterpret_cast<const float4*>(&dout[((int64_t)b * L + j) * d + h * HD + c]);
  }
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    msk[j] = key_pad[(int64_t)b * L + j] ? 1.f : 0.f;
    Ls[j] = lse[(int64_t)bh * L + j];
    const float* op = out + ((int64_t)b * L + j) * d + h * HD;
    const float* gp = dout + ((int64_t)b * L + j) * d + h * HD;
    float dl = 0.f;
#pragma unroll
    for (int c = 0; c < HD; ++c) dl += gp[c] * op[c];
    Ds[j] = dl;
  }
  __syncthreads();
  DropKey dkey;
  if (DROP) dkey = make_key(key, site, pdrop);

  float* dbase = dqkv + (int64_t)b * L * ld;
  // dQ: lane per query
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    float q[HD], g[HD], dq[HD];
#pragma unroll
    for (int c = 0; c < HD; ++c) { q[c] = Qs[i * HD + c]; g[c] = Gs[i * HD + c]; dq[c] = 0.f; }
    const float li = Ls[i], di = Ds[i];
    for (int j = 0; j < L; ++j) {
      if (msk[j] != 0.f) continue;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int c = 0; c < HD; ++c) { s += q[c] * Ks[j * HD + c]; dp += g[c] * Vs[j * HD + c]; }
      const float p = expf(s * scale - li);
      const float z = DROP ? keep_mult(dkey, ((uint64_t)bh * L + i) * L + j) : 1.f;
      const float ds = p * (z * dp - di);
#pragma unroll
      for (int c = 0; c < HD; ++c) dq[c] += ds * Ks[j * HD + c];
    }
    float* dp_ = dbase + (int64_t)i * ld + h * HD;
#pragma unroll
    for (int c = 0; c < HD; ++c) dp_[c] = dq[c] * scale;
  }
  // dK, dV: lane per key
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    float k[HD], v[HD], dk[HD], dv[HD];
#pragma unroll
    for (int c = 0; c < HD; ++c) {
      k[c] = Ks[j * HD + c]; v[c] = Vs[j * HD + c]; dk[c] = 0.f; dv[c] = 0.f;
    }
    if (msk[j] == 0.f) {
      for (int i = 0; i < L; ++i) {
        float s = 0.f, dp = 0.f;
#pragma unroll
        for (int c = 0; c < HD; ++c) { s += Qs[i * HD + c] * k[c]; dp += Gs[i * HD + c] * v[c]; }
        const float p = expf(s * scale - Ls[i]);
        const float z = DROP ? keep_mult(dkey, ((uint64_t)bh * L + i) * L + j) : 1.f;
        const float ds = p * (z * dp - Ds[i]);
        const float pz = p * z;
#pragma unroll
        for (int c = 0; c < HD; ++c) { dk[c] += ds * Qs[i * HD + c]; dv[c] += pz * Gs[i * HD + c]; }
      }
    }
    float* kp = dbase + (int64_t)j * ld + d + h * HD;
    float* vp = dbase + (int64_t)j * ld + 2 * d + h * HD;
#pragma unroll
    for (int c = 0; c < HD; ++c) { kp[c] = dk[c] * scale; vp[c] = dv[c]; }
  }
}

int threads_for(int L) {
  int t = ((L + 63) / 64) * 64;
  return t > 256 ? 256 : t;
}

}  // namespace
}  // namespace rs

using namespace rs;

#define RS_ATTN_DISPATCH(HDV, DROPV, KERNEL, ...)                                         \
  switch (HDV * 2 + (DROPV ? 1 : 0)) {                                                    \
    case 16: KERNEL<8, false><<<grid, thr, lds, st>>>(__VA_ARGS__); break;                \
    case 17: KERNEL<8, true><<<grid, thr, lds, st>>>(__VA_ARGS__); break;                 \
    case 32: KERNEL<16, false><<<grid, thr, lds, st>>>(__VA_ARGS__); break;               \
    case 33: KERNEL<16, true><<<grid, thr, lds, st>>>(__VA_ARGS__); break;                \
    case 64: KERNEL<32, false><<<grid, thr, lds, st>>>(__VA_ARGS__); break;               \
    case 65: KERNEL<32, true><<<grid, thr, lds, st>>>(__VA_ARGS__); break;                \
    case 128: KERNEL<64, false><<<grid, thr, lds, st>>>(__VA_ARGS__); break;              \
    case 129: KERNEL<64, true><<<grid, thr, lds, st>>>(__VA_ARGS__); break;               \
    default: break;                                                                       \
  }

extern "C" int rs_attn_fwd(const float* qkv, const uint8_t* key_pad, float* out, float* lse,
                           int B, int L, int d, int H, float scale, float p, const int64_t* key,
                           int site, void* stream) {
  RS_CHECK_ARG(qkv && key_pad && out && lse, "rs_attn_fwd: null pointer");
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1 && d % H == 0, "rs_attn_fwd: bad shape");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_attn_fwd: bad dropout p=%f", p);
  const int hd = d / H;
  RS_CHECK_ARG(hd == 8 || hd == 16 || hd == 32 || hd == 64, "rs_attn_fwd: head_dim %d unsupported", hd);
  if (B == 0) return 0;
  const size_t lds = (size_t)(2 * L * hd + L) * sizeof(float);
  RS_CHECK_ARG(lds <= 64 * 1024, "rs_attn_fwd: L=%d hd=%d exceeds LDS", L, hd);
  RS_CHECK_ARG(d % 4 == 0 && aligned16(qkv) && aligned16(out), "rs_attn_fwd: needs 16-byte aligned rows");
  dim3 grid(bh_grid(B, H));
  int thr = threads_for(L);
  hipStream_t st = as_stream(stream);
  RS_ATTN_DISPATCH(hd, p > 0.f, attn_fwd_kernel, qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site);
  RS_CHECK_LAUNCH("rs_attn_fwd");
  return 0;
}

extern "C" int rs_attn_bwd(const float* qkv, const uint8_t* key_pad, const float* out,
                           const float* dout, const float* lse, float* dqkv, int B, int L, int d,
                           int H, float scale, float p, const int64_t* key, int site,
                           void* stream) {
  RS_CHECK_ARG(qkv && key_pad && out && dout && lse && dqkv, "rs_attn_bwd: null pointer");
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1 && d % H == 0, "rs_attn_bwd: bad shape");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_attn_bwd: bad dropout p=%f", p);
  const int hd = d / H;
  RS_CHECK_ARG(hd == 8 || hd == 16 || hd == 32 || hd == 64, "rs_attn_bwd: head_dim %d unsupported", hd);
  if (B == 0) return 0;
  const size_t lds = (size_t)(4 * L * hd + 3 * L) * sizeof(float);
  RS_CHECK_ARG(lds <= 64 * 1024, "rs_attn_bwd: L=%d hd=%d exceeds LDS", L, hd);
  RS_CHECK_ARG(d % 4 == 0 && aligned16(qkv) && aligned16(dout), "rs_attn_bwd: needs 16-byte aligned rows");
  dim3 grid(bh_grid(B, H));
  int thr = threads_for(L);
  hipStream_t st = as_stream(stream);
  RS_ATTN_DISPATCH(hd, p > 0.f, attn_bwd_kernel, qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale,
                   p, key, site);
  RS_CHECK_LAUNCH("rs_attn_bwd");
  return 0;
}
