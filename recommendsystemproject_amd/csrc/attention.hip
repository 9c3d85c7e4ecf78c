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
#include <type_traits>

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

// ============================================================================ MFMA path
// head_dim 16, L <= 64 (the C2/C3 encoder: d = 64, H = 4, L = 50): one wave per (sample, head),
// f32 MFMA 16x16x4 (exact f32 products, same rate as the VALU but a quarter of the issue slots
// and the VALU left free for exp / masks / dropout hashes). NT = ceil(L/16) tiles of 16.
//
// Score tiles are computed transposed, S^T[key][query] = K Q^T: with the K fragment on the MFMA
// row side each lane ends up owning ONE query (lane & 15) and 4 consecutive keys per tile
// (4 * (lane >> 4) + e), so a query's softmax statistics reduce over the lane's own 4 NT values
// plus two cross-lane xor shuffles (16, 32), and the lane's probabilities are directly the A
// fragment of P V (k = key index), no data movement. Fragment loads are float4 rows of qkv:
// lane (r = lane & 15, q = lane >> 4) holds X[row 16 t + r][4q .. 4q + 3], and MFMA s of a
// 4-step k chain consumes component s (k = 4q + s), the permuted-k order used by rowgemm.
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
// LDS row pitch of the per-wave [L][16] tiles: lanes (c, q) read rows 4q + s, so a pitch of 20
// words puts the four q groups on disjoint bank quarters (16 words would be a 4-way conflict)
constexpr int kRowP = 20;

// dropout index ((b*H + h)*L + i)*L + j in 32 bits (the host checks B*H*L*L < 2^32):
// keep_mult32 (rng.h)

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float xsum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}
__device__ __forceinline__ float xmax(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}

// one wave per (b, h); 4 waves per workgroup = 4 consecutive (b, h) (the heads of one sample)
template <int NT, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_mfma_kernel(
    const float* __restrict__ qkv, const uint8_t* __restrict__ key_pad, float* __restrict__ out,
    float* __restrict__ lse, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site) {
  constexpr int LP = NT * 16;
  __shared__ __attribute__((aligned(16))) float Vsm[4][LP][kRowP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;  // whole wave exits together (no block barrier below)
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  const float* base = qkv + (int64_t)b * L * ld + h * 16;
  float(*Vs)[kRowP] = Vsm[wave];
  f4 qf[NT], kf[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int row = t * 16 + r;
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    qf[t] = row < L ? ld4(base + (int64_t)row * ld + 4 * q) : z;
    kf[t] = row < L ? ld4(base + (int64_t)row * ld + d + 4 * q) : z;
    *reinterpret_cast<f4*>(&Vs[row][4 * q]) = row < L ? ld4(base + (int64_t)row * ld + 2 * d + 4 * q) : z;
  }
  // key validity for this lane's keys 16 t + 4 q + e
  bool kok[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = t * 16 + 4 * q + e;
      kok[t][e] = j < L && key_pad[(int64_t)b * L + j] == 0;
    }
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const float scale2 = scale * kLog2e;
  __builtin_amdgcn_wave_barrier();  // Vs written by this wave only
#pragma unroll
  for (int tq = 0; tq < NT; ++tq) {
    f4 sv[NT];
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = mfma4(kf[tk][s4], qf[tq][s4], acc);
      sv[tk] = acc;
    }
    // softmax over keys for query i = 16 tq + r (same op order as the VALU kernel:
    // max of scale*s, then exp(scale*s - max))
    // exp(x) = exp2(x * log2 e): one v_exp_f32 per probability (the softmax is VALU-bound)
    float m = -INFINITY;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (kok[tk][e]) m = fmaxf(m, sv[tk][e] * scale2);
    m = xmax(m);
    float l = 0.f;
    const int i = tq * 16 + r;
    const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      float mk[4] = {1.f, 1.f, 1.f, 1.f};
      if (DROP) keep4_32(dk, rowbase + tk * 16 + 4 * q, mk);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = kok[tk][e] ? exp2f(sv[tk][e] * scale2 - m) : 0.f;
        l += pv;
        sv[tk][e] = DROP ? pv * mk[e] : pv;
      }
    }
    l = xsum(l);
    // O[i][c] = sum_j pz[i][j] V[j][c]: A = this lane's probabilities (row i = lane & 15,
    // k = key), B = V[key][c = lane & 15]
    f4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tk = 0; tk < NT; ++tk)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) o = mfma4(sv[tk][s4], Vs[tk * 16 + 4 * q + s4][r], o);
    // o[e] = O[16 tq + 4 q + e][c = r]; its 1/l lives in lanes with (lane & 15) == 4 q + e
    if (q == 0 && i < L) lse[(int64_t)bh * L + i] = (m + log2f(l)) * kLn2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float le = __shfl(l, 4 * q + e, 64);
      const int row = tq * 16 + 4 * q + e;
      if (row < L) out[((int64_t)b * L + row) * d + h * 16 + r] = o[e] * (1.f / le);
    }
  }
}

template <int NT, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_mfma_kernel(
    const float* __restrict__ qkv, const uint8_t* __restrict__ key_pad,
    const float* __restrict__ out, const float* __restrict__ dout, const float* __restrict__ lse,
    float* __restrict__ dqkv, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site) {
  constexpr int LP = NT * 16;
  constexpr int TP = 20;  // transpose buffer [LP keys][16 queries of the current tile], pitch 20
  __shared__ __attribute__((aligned(16))) float Qsm[4][LP][kRowP];
  __shared__ __attribute__((aligned(16))) float Ksm[4][LP][kRowP];
  __shared__ __attribute__((aligned(16))) float Gsm[4][LP][kRowP];
  __shared__ __attribute__((aligned(16))) float Tsm[4][LP * TP];  // 5 KB per wave
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  const float* base = qkv + (int64_t)b * L * ld + h * 16;
  const float* gbase = dout + (int64_t)b * L * d + h * 16;
  const float* obase = out + (int64_t)b * L * d + h * 16;
  float(*Qs)[kRowP] = Qsm[wave];
  float(*Ks)[kRowP] = Ksm[wave];
  float(*Gs)[kRowP] = Gsm[wave];
  float* T = Tsm[wave];
  f4 qf[NT], kf[NT], vf[NT], gf[NT];
  float Di[NT], lsei[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int row = t * 16 + r;
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    const bool ok = row < L;
    qf[t] = ok ? ld4(base + (int64_t)row * ld + 4 * q) : z;
    kf[t] = ok ? ld4(base + (int64_t)row * ld + d + 4 * q) : z;
    vf[t] = ok ? ld4(base + (int64_t)row * ld + 2 * d + 4 * q) : z;
    gf[t] = ok ? ld4(gbase + (int64_t)row * d + 4 * q) : z;
    const f4 of = ok ? ld4(obase + (int64_t)row * d + 4 * q) : z;
    *reinterpret_cast<f4*>(&Qs[row][4 * q]) = qf[t];
    *reinterpret_cast<f4*>(&Ks[row][4 * q]) = kf[t];
    *reinterpret_cast<f4*>(&Gs[row][4 * q]) = gf[t];
    // D_i = sum_c dO[i][c] O[i][c] (query i = row, this lane's 4 columns, then across q)
    Di[t] = xsum(gf[t][0] * of[0] + gf[t][1] * of[1] + gf[t][2] * of[2] + gf[t][3] * of[3]);
    lsei[t] = ok ? lse[(int64_t)bh * L + row] * kLog2e : 0.f;  // base-2 log-sum-exp
  }
  bool kok[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = t * 16 + 4 * q + e;
      kok[t][e] = j < L && key_pad[(int64_t)b * L + j] == 0;
    }
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const float scale2 = scale * kLog2e;
  __builtin_amdgcn_wave_barrier();
  float* dbase = dqkv + (int64_t)b * L * ld + h * 16;
  // per query tile: P^T, dS^T (keys x queries), dQ; P∘Z and dS go to T for dV / dK
  f4 dv_acc[NT], dk_acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dv_acc[t] = dk_acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tq = 0; tq < NT; ++tq) {
    const int i = tq * 16 + r;
    const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
    f4 ps[NT], ds[NT];
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      f4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        sacc = mfma4(kf[tk][s4], qf[tq][s4], sacc);   // S^T[key][query]
        pacc = mfma4(vf[tk][s4], gf[tq][s4], pacc);   // dP^T[key][query] = V dO^T
      }
      float mk[4] = {1.f, 1.f, 1.f, 1.f};
      if (DROP) keep4_32(dk, rowbase + tk * 16 + 4 * q, mk);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = (kok[tk][e] && i < L) ? exp2f(sacc[e] * scale2 - lsei[tq]) : 0.f;
        const float z = DROP ? mk[e] : 1.f;
        ds[tk][e] = pv * (z * pacc[e] - Di[tq]);
        ps[tk][e] = pv * z;
      }
    }
    // dQ[i][c] = scale * sum_j dS[i][j] K[j][c]
    f4 dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tk = 0; tk < NT; ++tk)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dq = mfma4(ds[tk][s4], Ks[tk * 16 + 4 * q + s4][r], dq);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = tq * 16 + 4 * q + e;
      if (row < L) dbase[(int64_t)row * ld + r] = dq[e] * scale;
    }
    // dV[j][c] += sum_i PZ[i][j] dO[i][c]: A must be indexed (key = lane & 15, k = query):
    // transpose this query tile's PZ^T through T (T[key][query])
#pragma unroll
    for (int tk = 0; tk < NT; ++tk)
#pragma unroll
      for (int e = 0; e < 4; ++e) T[(tk * 16 + 4 * q + e) * TP + r] = ps[tk][e];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      const f4 a = ld4(&T[(tk * 16 + r) * TP + 4 * q]);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dv_acc[tk] = mfma4(a[s4], Gs[tq * 16 + 4 * q + s4][r], dv_acc[tk]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tk = 0; tk < NT; ++tk)
#pragma unroll
      for (int e = 0; e < 4; ++e) T[(tk * 16 + 4 * q + e) * TP + r] = ds[tk][e];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      const f4 a = ld4(&T[(tk * 16 + r) * TP + 4 * q]);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dk_acc[tk] = mfma4(a[s4], Qs[tq * 16 + 4 * q + s4][r], dk_acc[tk]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // dK / dV rows: acc[e] = X[key 16 tk + 4 q + e][c = r]
#pragma unroll
  for (int tk = 0; tk < NT; ++tk)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = tk * 16 + 4 * q + e;
      if (row < L) {
        dbase[(int64_t)row * ld + d + r] = dk_acc[tk][e] * scale;
        dbase[(int64_t)row * ld + 2 * d + r] = dv_acc[tk][e];
      }
    }
}

// ------------------------------------------------------------------ bf16 MFMA (bf16 mode)
// Same structure as the f32 MFMA kernels (one wave per (b, h), S^T tiles with the key on the
// row so each lane owns one query), on v_mfma_f32_16x16x16_bf16: with head_dim 16 every 16x16
// product is ONE instruction instead of four 16x16x4 f32 ones. Operand maps (16x16x16): lane
// (r = l&15, q = l>>4) supplies A[r][4q + j] and B[4q + j][r], j < 4 -- the same registers the
// f32 kernels feed one k-slice at a time, so Q/K/V/dO rows load as before and the softmax /
// dropout / dS arithmetic (fp32) is unchanged. The B operands that need a column per lane
// (V for P V; K, Q, dO for dQ, dK, dV) are read once per wave through LDS before the loops.
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf4v __attribute__((ext_vector_type(4)));

// two v_cvt_pk_bf16_f32 (round to nearest even, as the element-wise casts; those compiled to four
// single-element converts and two v_perm_b32)
__device__ __forceinline__ s4v bf4(const f4& v) {
  typedef __bf16 bf2v __attribute__((ext_vector_type(2)));
  typedef float f2v __attribute__((ext_vector_type(2)));
  const bf2v lo = __builtin_convertvector(f2v{v[0], v[1]}, bf2v);
  const bf2v hi = __builtin_convertvector(f2v{v[2], v[3]}, bf2v);
  return __builtin_bit_cast(s4v, __builtin_shufflevector(lo, hi, 0, 1, 2, 3));
}
__device__ __forceinline__ f4 mfma16(const s4v& a, const s4v& b, const f4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// column r, rows 16t + 4q + j of a per-wave [LP][P] fp32 image
template <int NT, int P>
__device__ __forceinline__ void col_frags(const float* X, int r, int q, s4v (&out)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = X[(t * 16 + 4 * q + j) * P + r];
    out[t] = bf4(v);
  }
}

// qkv / dqkv storage: fp32, or bf16 (RS_ATTN_QKV_BF16). Q, K and V are only ever MFMA operands
// here (rounded to bf16 by bf4), so bf16 storage gives the same products with half the bytes.
__device__ __forceinline__ f4 ldq(const float* p) { return ld4(p); }
__device__ __forceinline__ f4 ldq(const __bf16* p) {
  const bf4v h = *reinterpret_cast<const bf4v*>(p);  // 8-byte load; bf16 -> fp32 is exact
  return f4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}
__device__ __forceinline__ void stq(float* p, float v) { *p = v; }
__device__ __forceinline__ void stq(__bf16* p, float v) { *p = (__bf16)v; }

// Per-lane key-validity bits: bit 4t + e <-> key 16t + 4q + e (the lane's keys in S^T tile t),
// from one coalesced byte load per lane and a wave ballot (L <= 64).
template <int NT>
__device__ __forceinline__ uint32_t key_bits(const uint8_t* __restrict__ key_pad, int b, int L,
                                             int lane, int q) {
  const bool valid = lane < L && key_pad[(int64_t)b * L + lane] == 0;
  const uint64_t vm = __ballot(valid);
  uint32_t kb = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) kb |= (uint32_t)((vm >> (16 * t + 4 * q)) & 0xFu) << (4 * t);
  return kb;
}

// dropout multipliers of keys 16 tk + 4q .. +3 of query row i: with L even the row base
// ((bh L + i) L) and the 4-aligned key offset are even, so two pair hashes cover the 4 keys
// (the same draws keep4_32 makes; odd L keeps the general path)
__device__ __forceinline__ void attn_keep4(const DropKey& dk, bool leven, uint32_t idx0, float (&mk)[4]) {
  if (leven) {
    keep_pair32(dk, idx0 >> 1, mk[0], mk[1]);
    keep_pair32(dk, (idx0 >> 1) + 1, mk[2], mk[3]);
  } else {
    keep4_32(dk, idx0, mk);
  }
}

// the same draws as keep decisions (kept <-> multiplier 1/(1-p)): the kernels below fold the
// 1/(1-p) into one product per output element and select instead of multiplying
__device__ __forceinline__ void attn_keep4b(const DropKey& dk, bool leven, uint32_t idx0, bool (&kp)[4]) {
  if (leven) {
    const uint32_t h0 = pair_hash32(dk, idx0 >> 1), h1 = pair_hash32(dk, (idx0 >> 1) + 1);
    kp[0] = (h0 & 0xffffu) >= dk.thresh;
    kp[1] = (h0 >> 16) >= dk.thresh;
    kp[2] = (h1 & 0xffffu) >= dk.thresh;
    kp[3] = (h1 >> 16) >= dk.thresh;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = idx0 + i, hh = pair_hash32(dk, x >> 1);
      kp[i] = ((x & 1) ? (hh >> 16) : (hh & 0xffffu)) >= dk.thresh;
    }
  }
}

// Score-tile accumulator init: 0 for valid keys, -inf for padded ones (bit 4t + e of the lane's
// key bits), so the MFMA itself masks the scores: no per-element select in the max or the exp.
template <int NT>
__device__ __forceinline__ void key_bias(uint32_t kbits, f4 (&kbias)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) kbias[t][e] = ((kbits >> (4 * t + e)) & 1u) ? 0.f : -INFINITY;
}
// IEEE maximum (v_maximum3_f32 on gfx950): unlike fmaxf it needs no canonicalising v_max_f32
// of every MFMA result first
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }

// transposed bf16 fragment of a per-wave [16][WP] image W (row = query, 16-bit elements): lane
// (r, q) receives W[4q + j][16 tk + r], j < 4 -- the A operand [key r][query 4q + j] of a product
// that sums over the tile's queries (ds_read_b64_tr_b16; EXEC must be full: the callers' waves
// exit whole or not at all)
__device__ __forceinline__ s4v tr_col(const __bf16* W, int wp, int tk, int lane) {
  typedef __attribute__((address_space(3))) s4v* lptr;
  const int g = lane >> 4, l16 = lane & 15;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(W + (4 * g + (l16 >> 2)) * wp + 16 * tk + 4 * (l16 & 3)));
}

// 16x16 tile held as acc[e] = X[row 4q + e][col r] -> rows of 4 consecutive columns per lane
// through the wave's LDS image T (pitch TP): lane l gets row l >> 2, columns 4 (l & 3) .. + 3
template <int TP>
__device__ __forceinline__ f4 tile_rows(float* T, const f4& acc, int r, int q, int lane) {
#pragma unroll
  for (int e = 0; e < 4; ++e) T[(4 * q + e) * TP + r] = acc[e];
  __builtin_amdgcn_wave_barrier();
  const f4 v = ld4(&T[(lane >> 2) * TP + 4 * (lane & 3)]);
  __builtin_amdgcn_wave_barrier();
  return v;
}
__device__ __forceinline__ void st4q(float* p, const f4& v) { *reinterpret_cast<f4*>(p) = v; }
__device__ __forceinline__ void st4q(__bf16* p, const f4& v) {
  bf4v h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  *reinterpret_cast<bf4v*>(p) = h;
}

// ZB (with DROP): the keep decisions of the lane's 4 NT (query, key) elements of query tile tq are
// also stored, bit 4 tk + e, as zbits[(bh NT + tq) 64 + lane] (16 bits, NT <= 4) for the backward,
// which then reads them instead of drawing them again
template <int NT, bool DROP, bool QB, bool ZB = false>
__global__ __launch_bounds__(256) void attn_fwd_bf16_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad, float* __restrict__ out,
    float* __restrict__ lse, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site, uint16_t* __restrict__ zbits = nullptr) {
  constexpr int LP = NT * 16;
  __shared__ __attribute__((aligned(16))) float Vsm[4][LP][kRowP];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;  // whole wave exits together (no block barrier below)
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * 16;
  float(*Vs)[kRowP] = Vsm[wave];
  s4v qb[NT], kb[NT], vb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int row = t * 16 + r;
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    qb[t] = bf4(row < L ? ldq(base + (int64_t)row * ld + 4 * q) : z);
    kb[t] = bf4(row < L ? ldq(base + (int64_t)row * ld + d + 4 * q) : z);
    *reinterpret_cast<f4*>(&Vs[row][4 * q]) = row < L ? ldq(base + (int64_t)row * ld + 2 * d + 4 * q) : z;
  }
  const uint32_t kbits = key_bits<NT>(key_pad, b, L, lane, q);
  f4 kbias[NT];
  key_bias<NT>(kbits, kbias);
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const bool leven = (L & 1) == 0;
  const float scale2 = scale * kLog2e;
  __builtin_amdgcn_wave_barrier();            // Vs written by this wave only
  col_frags<NT, kRowP>(&Vs[0][0], r, q, vb);  // B of P V: V[16 tk + 4q + j][c = r]
  __builtin_amdgcn_wave_barrier();
  float* T = &Vs[0][0];  // V is in registers now: the image is free for the output transpose
#pragma unroll
  for (int tq = 0; tq < NT; ++tq) {
    f4 sv[NT];
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) sv[tk] = mfma16(kb[tk], qb[tq], kbias[tk]);  // masked: -inf
    // max of the raw scores, scaled once (scale2 > 0 and rounding is monotonic: bitwise the max
    // of the scaled scores); a row with every key masked uses 0 (P = 0, l = 0, as before)
    float m = -INFINITY;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) m = vmax(vmax(vmax(m, sv[tk][0]), sv[tk][1]), vmax(sv[tk][2], sv[tk][3]));
    m = xmax(m);
    const float ms = m == -INFINITY ? 0.f : m * scale2;
    float l = 0.f;
    const int i = tq * 16 + r;
    const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
    uint32_t zw = 0;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      bool kp[4] = {true, true, true, true};
      if (DROP) attn_keep4b(dk, leven, rowbase + tk * 16 + 4 * q, kp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[tk][e], scale2, -ms));
        l += pv;
        sv[tk][e] = kp[e] ? pv : 0.f;  // P∘Z (1/(1-p) applied to the output row below)
        if (ZB) zw |= kp[e] ? (1u << (4 * tk + e)) : 0u;
      }
    }
    if (ZB) zbits[((int64_t)bh * NT + tq) * 64 + lane] = (uint16_t)zw;
    l = xsum(l);
    f4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) o = mfma16(bf4(sv[tk]), vb[tk], o);
    if (q == 0 && i < L) lse[(int64_t)bh * L + i] = (ms + __builtin_amdgcn_logf(l)) * kLn2;
    // rows 4q + e of the tile need the 1/l of query 4q + e (lane 4q + e)
    const float rl = DROP ? __builtin_amdgcn_rcpf(l) * dk.scale : __builtin_amdgcn_rcpf(l);
    f4 on;
#pragma unroll
    for (int e = 0; e < 4; ++e) on[e] = o[e] * __shfl(rl, 4 * q + e, 64);
    const f4 v = tile_rows<kRowP>(T, on, r, q, lane);
    const int row = tq * 16 + (lane >> 2);
    if (row < L) st4q(out + ((int64_t)b * L + row) * d + h * 16 + 4 * (lane & 3), v);
  }
}

// 3 waves per SIMD (<= 168 VGPRs). ZB (with DROP): the keep decisions come from the forward's
// zbits (attn_fwd_bf16_kernel) instead of the hash -- the same draws, none of the hash's VALU work
template <int NT, bool DROP, bool QB, bool ZB = false>
__global__ __launch_bounds__(256, 3) void attn_bwd_bf16_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad,
    const float* __restrict__ out, const float* __restrict__ dout, const float* __restrict__ lse,
    void* __restrict__ dqkv_, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site, const uint16_t* __restrict__ zbits = nullptr) {
  constexpr int LP = NT * 16;
  // pitch 24: the transpose's ds_read_b128 (rows r, columns 4q) is conflict-free; its b32 writes
  // are 2-way, which costs nothing for ds_write_b32 (MI355X_MICROARCH.md §LDS)
  constexpr int TP = 24;
  // bf16 [16 queries][WP] images of one query tile's P∘Z and dS (row = query, 4 keys per 8-byte
  // store), read back transposed (tr_col); WP = LP + 16: 80 at LP = 64 puts the eight rows of a
  // 32-lane half's transposed reads on disjoint banks
  constexpr int WP = LP + 16;
  constexpr int XW = (LP * TP > 16 * TP + 16 * WP) ? LP * TP : 16 * TP + 16 * WP;
  // one image per wave (6.5 KB at LP = 64): Q, K and dO pass through it once (column
  // fragments), then rows [0, 16) are the output transposes and the rest the P∘Z / dS images
  __shared__ __attribute__((aligned(16))) float Xsm[4][XW];
  // the Q and dO column fragments (each used once per query tile) wait in LDS, one 8-byte slot
  // per lane (conflict-free b64 accesses): held in registers they pushed the kernel past its
  // 168-VGPR budget (3 waves per SIMD) and the spill stores were ~56 MB of scratch writes per
  // launch at C2 (PMC WRITE_SIZE 135 MB against 79 MB of dqkv)
  __shared__ __attribute__((aligned(16))) s4v Fsm[4][2][NT][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int bh = blockIdx.x * 4 + wave;
  if (bh >= B * H) return;
  const int b = bh / H, h = bh % H;
  const int ld = 3 * d;
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * 16;
  const float* gbase = dout + (int64_t)b * L * d + h * 16;
  float* T = Xsm[wave];
  s4v qb[NT], kb[NT], vb[NT], gb[NT];
  float lsei[NT];
  // column fragments (B operands of dQ = dS K, dK = dS^T Q, dV = PZ^T dO) via the LDS image
  s4v kc[NT];
  {
    f4 qf[NT], kf[NT], gf[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = t * 16 + r;
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      const bool ok = row < L;
      qf[t] = ok ? ldq(base + (int64_t)row * ld + 4 * q) : z;
      kf[t] = ok ? ldq(base + (int64_t)row * ld + d + 4 * q) : z;
      vb[t] = bf4(ok ? ldq(base + (int64_t)row * ld + 2 * d + 4 * q) : z);
      gf[t] = ok ? ld4(gbase + (int64_t)row * d + 4 * q) : z;
      // base-2 log-sum-exp; +inf past L and 0 for a row with every key masked (lse = -inf): the
      // exp below then gives P = 0 for those rows as the masked selects used to
      const float ls = ok ? lse[(int64_t)bh * L + row] : 0.f;
      lsei[t] = !ok ? INFINITY : (ls == -INFINITY ? 0.f : ls * kLog2e);
    }
#pragma unroll
    for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        *reinterpret_cast<f4*>(&T[(t * 16 + r) * TP + 4 * q]) = pass == 0 ? qf[t] : (pass == 1 ? kf[t] : gf[t]);
      __builtin_amdgcn_wave_barrier();
      if (pass == 1) {
        col_frags<NT, TP>(T, r, q, kc);
      } else {
        s4v cf[NT];
        col_frags<NT, TP>(T, r, q, cf);
#pragma unroll
        for (int t = 0; t < NT; ++t) Fsm[wave][pass >> 1][t][lane] = cf[t];
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      qb[t] = bf4(qf[t]);
      kb[t] = bf4(kf[t]);
      gb[t] = bf4(gf[t]);
    }
  }
  uint32_t zw[NT];
  if (ZB)
#pragma unroll
    for (int t = 0; t < NT; ++t) zw[t] = zbits[((int64_t)bh * NT + t) * 64 + lane];
  const uint32_t kbits = key_bits<NT>(key_pad, b, L, lane, q);
  f4 kbias[NT];
  key_bias<NT>(kbits, kbias);
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const bool leven = (L & 1) == 0;
  const float scale2 = scale * kLog2e;
  const float zs = DROP ? dk.scale : 1.f;  // the kept elements' 1/(1-p), applied per output
  QT* dbase = reinterpret_cast<QT*>(dqkv_) + (int64_t)b * L * ld + h * 16;
  __bf16* Wpz = reinterpret_cast<__bf16*>(T + 16 * TP);  // [16][WP] P∘Z / zs
  __bf16* Wds = Wpz + 16 * WP;                            // [16][WP] dS
  f4 dv_acc[NT], dk_acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dv_acc[t] = dk_acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tq = 0; tq < NT; ++tq) {
    const int i = tq * 16 + r;
    const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
    f4 pvs[NT], dpz[NT];  // P and dP∘Z / zs of the lane's (query i, keys 16 tk + 4q + e)
    float Dp = 0.f;
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      const f4 sacc = mfma16(kb[tk], qb[tq], kbias[tk]);               // S^T[key][query], masked -inf
      const f4 pacc = mfma16(vb[tk], gb[tq], f4{0.f, 0.f, 0.f, 0.f});  // dP^T = V dO^T
      bool kp[4] = {true, true, true, true};
      if (ZB) {
#pragma unroll
        for (int e = 0; e < 4; ++e) kp[e] = (zw[tq] >> (4 * tk + e)) & 1u;
      } else if (DROP) {
        attn_keep4b(dk, leven, rowbase + tk * 16 + 4 * q, kp);
      }
      f4 pz;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // lsei is +inf past L and 0 for a row with no valid key: P = 0 there without a select
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[e], scale2, -lsei[tq]));
        pvs[tk][e] = pv;
        dpz[tk][e] = kp[e] ? pacc[e] : 0.f;
        pz[e] = kp[e] ? pv : 0.f;
        Dp = __builtin_fmaf(pv, dpz[tk][e], Dp);
      }
      // P∘Z row slice -> W (A operand of dV = (P∘Z)^T dO after the transposed read)
      *reinterpret_cast<s4v*>(&Wpz[r * WP + 16 * tk + 4 * q]) = bf4(pz);
    }
    // D_i = sum_j P_ij (dP∘Z)_ij (= dO_i . O_i): from the register tiles, no O read
    const float Di = xsum(Dp) * zs;
    f4 dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      f4 ds;
#pragma unroll
      for (int e = 0; e < 4; ++e) ds[e] = pvs[tk][e] * __builtin_fmaf(dpz[tk][e], zs, -Di);
      const s4v dsb = bf4(ds);
      *reinterpret_cast<s4v*>(&Wds[r * WP + 16 * tk + 4 * q]) = dsb;
      dq = mfma16(dsb, kc[tk], dq);  // dS[query][key] K
    }
    __builtin_amdgcn_wave_barrier();
    // dV[key][c] += (P∘Z)^T dO and dK[key][c] += dS^T Q: A = [key = lane & 15][query 4q + j]
#pragma unroll
    for (int tk = 0; tk < NT; ++tk) {
      dv_acc[tk] = mfma16(tr_col(Wpz, WP, tk, lane), Fsm[wave][1][tq][lane], dv_acc[tk]);
      dk_acc[tk] = mfma16(tr_col(Wds, WP, tk, lane), Fsm[wave][0][tq][lane], dk_acc[tk]);
    }
    {
      const f4 v = tile_rows<TP>(T, dq * scale, r, q, lane);
      const int row = tq * 16 + (lane >> 2);
      if (row < L) st4q(dbase + (int64_t)row * ld + 4 * (lane & 3), v);
    }
    __builtin_amdgcn_wave_barrier();
  }
  // dK / dV rows: acc[e] = X[key 16 tk + 4 q + e][c = r]
#pragma unroll
  for (int tk = 0; tk < NT; ++tk) {
    const f4 vk = tile_rows<TP>(T, dk_acc[tk] * scale, r, q, lane);
    const f4 vv = tile_rows<TP>(T, dv_acc[tk] * zs, r, q, lane);
    const int row = tk * 16 + (lane >> 2);
    if (row < L) {
      st4q(dbase + (int64_t)row * ld + d + 4 * (lane & 3), vk);
      st4q(dbase + (int64_t)row * ld + 2 * d + 4 * (lane & 3), vv);
    }
  }
}

// ------------------------------------------------------- bf16 MFMA, long histories (64 < L <= 256)
// C5's encoder (L = 200): the per-wave kernels above hold every tile of one (b, h) in registers,
// which stops at L = 64. Here one 4-wave workgroup owns one (b, h); K and V (forward) or Q, K, V
// and dO (backward) sit once in LDS as fp32 [LP][kRowP] images and the waves split the tiles.
//  forward: wave w takes query tiles w, w + 4, ...; per query tile the same S^T / softmax / P V
//           sequence as attn_fwd_bf16_kernel (all NT key tiles in registers, 64 key-valid bits);
//           Q is staged in LDS with K and V, so the tile loop has no global-memory latency.
//  backward, single pass with no atomics (attn_bwd_long1_bf16_kernel): wave w takes key tiles
//           w, w + 4, ... and computes S = Q K^T and dP = dO V^T with the QUERY on the row, so the
//           lane's P∘Z and dS tiles are directly the A operands of dV = (P∘Z)^T dO and
//           dK = dS^T Q; dQ = dS K from the same tiles (below). D_i = dO_i . O_i comes from the
//           forward output. (Measured and removed: the FlashAttention-2 split that recomputed S^T
//           and dP^T in a second, query-parallel phase for dQ -- twice the exp / hash work.)
// Dropout draws are the per-element keep_mult32 of index ((b H + h) L + i) L + j, as everywhere.
template <int NT>
__device__ __forceinline__ uint64_t key_bits_long(const uint8_t* __restrict__ key_pad, int b,
                                                  int L, int lane, int q) {
  uint64_t kb = 0;
#pragma unroll
  for (int g = 0; g < (NT + 3) / 4; ++g) {
    const int j = 64 * g + lane;
    const uint64_t vm = __ballot(j < L && key_pad[(int64_t)b * L + j] == 0);
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
      if (4 * g + tt < NT) kb |= ((vm >> (16 * tt + 4 * q)) & 0xFull) << (4 * (4 * g + tt));
  }
  return kb;
}

// rows [0, LP) of the head-h slice of matrix `which` (0 = Q, 1 = K, 2 = V) of qkv, zero past L,
// into an fp32 [LP][kRowP] LDS image; 16-byte loads, 4 threads per 64-byte row slice
template <int LP, typename QT>
__device__ __forceinline__ void load_head_image(const QT* __restrict__ base, int ld, int L,
                                                int off, float (*X)[kRowP]) {
  for (int e = threadIdx.x; e < LP * 4; e += 256) {
    const int row = e >> 2, c4 = (e & 3) * 4;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < L) v = ldq(base + (int64_t)row * ld + off + c4);
    *reinterpret_cast<f4*>(&X[row][c4]) = v;
  }
}

// phase-A dropout multipliers of (query rb-row e, key j), e < 4, for the lane holding key j of 4
// consecutive queries (row bases rb0 + e L): with L even, keys j and j ^ 1 of one query are one
// hash pair, held by neighbour lanes r and r ^ 1; each lane hashes two of the four pairs and
// passes the half it does not need across (one hash per two elements, as in the forward)
__device__ __forceinline__ void keep_col4(const DropKey& dk, bool leven, uint32_t rb0, uint32_t L,
                                          uint32_t j, int r, float (&mk)[4]) {
  if (leven) {
    const int p = r & 1;
    float mine[2], recv[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t e = 2 * p + s;
      const uint32_t h = pair_hash32(dk, (rb0 + e * L + (j & ~1u)) >> 1);
      const float lo = (h & 0xffffu) >= dk.thresh ? dk.scale : 0.f;
      const float hi = (h >> 16) >= dk.thresh ? dk.scale : 0.f;
      mine[s] = p ? hi : lo;
      recv[s] = __shfl_xor(p ? lo : hi, 1, 64);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) mk[e] = ((e >> 1) == p) ? mine[e & 1] : recv[e & 1];
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) mk[e] = keep_mult32(dk, rb0 + e * L + j);
  }
}

// bf16 images of the long kernels: Q, K, V and dO are MFMA operands only (rounded to bf16
// wherever they are used), so they are staged once as bf16 -- half the LDS of the fp32 images,
// which lets three workgroups share a CU -- and their fragments are read as they stand
constexpr int kRowPB = 24;  // bf16 image row pitch (48 B)
template <int LP, typename QT>
__device__ __forceinline__ void load_head_image16(const QT* __restrict__ base, int ld, int L, int off,
                                                  __bf16 (*X)[kRowPB]) {
  for (int e = threadIdx.x; e < LP * 4; e += 256) {
    const int row = e >> 2, c4 = (e & 3) * 4;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < L) v = ldq(base + (int64_t)row * ld + off + c4);
    *reinterpret_cast<s4v*>(&X[row][c4]) = bf4(v);
  }
}
__device__ __forceinline__ s4v row_frag16(const __bf16 (*X)[kRowPB], int row, int q) {
  return *reinterpret_cast<const s4v*>(&X[row][4 * q]);
}
// column r, rows t0 + 4q + j of a bf16 image: the B operand fragment
__device__ __forceinline__ s4v col_frag16(const __bf16 (*X)[kRowPB], int t0, int r, int q) {
  s4v o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = __builtin_bit_cast(short, X[t0 + 4 * q + j][r]);
  return o;
}

#ifndef RS_LONG_FWD_MINW
#define RS_LONG_FWD_MINW 3  // three workgroups per CU: bf16 images (LDS) and V re-read (VGPRs)
#endif
template <int NT, bool DROP, bool QB>
__global__ __launch_bounds__(256, RS_LONG_FWD_MINW) void attn_fwd_long_bf16_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad, float* __restrict__ out,
    float* __restrict__ lse, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site) {
  constexpr int LP = NT * 16;
  __shared__ __attribute__((aligned(16))) __bf16 Qs[LP][kRowPB];
  __shared__ __attribute__((aligned(16))) __bf16 Ks[LP][kRowPB];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[LP][kRowPB];
  __shared__ __attribute__((aligned(16))) float Tsm[4][16 * kRowP];
  // score-tile accumulator init per key: 0 (valid) or -inf (padded, or past L): the MFMA masks
  __shared__ __attribute__((aligned(16))) float Kb[LP];
  int b, h;
  if (!map_bh(B, H, b, h)) return;  // uniform over the workgroup
  const int bh = b * H + h;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ld = 3 * d;
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * 16;
  load_head_image16<LP>(base, ld, L, 0, Qs);  // Q too: no global load inside the tile loop
  load_head_image16<LP>(base, ld, L, d, Ks);
  load_head_image16<LP>(base, ld, L, 2 * d, Vs);
  for (int j = threadIdx.x; j < LP; j += 256) Kb[j] = (j < L && key_pad[(int64_t)b * L + j] == 0) ? 0.f : -INFINITY;
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const bool leven = (L & 1) == 0;
  const float scale2 = scale * kLog2e;
  __syncthreads();
  // K fragments in registers; V's column fragments re-read from the bf16 image where the P V
  // products need them (their registers kept the kernel at two waves per SIMD)
  s4v kb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) kb[t] = row_frag16(Ks, t * 16 + r, q);
  float* T = Tsm[wave];
  // query tiles below NTF = 4 floor(NT / 4) go round-robin to the waves; the NT % 4 tiles past
  // them are shared (see the end)
  constexpr int NTF = 4 * (NT / 4), NR = NT - NTF;
  for (int tq = wave; tq < NTF; tq += 4) {
    const int i = tq * 16 + r;
    const f4 z = {0.f, 0.f, 0.f, 0.f};
    const s4v qb = row_frag16(Qs, i, q);
    // online softmax over chunks of CH key tiles (flash-style rescale of the running sum and of
    // the P V accumulator when the max grows): only CH score tiles live at a time -- all NT of
    // them held the kernel at two waves per SIMD
    constexpr int CH = 4;
    // m: running max of the raw (masked) scores; ms = m * scale2, or 0 while no key was valid
    float m = -INFINITY, ms = 0.f, l = 0.f;
    f4 o = z;
    const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
#pragma unroll
    for (int c0 = 0; c0 < NT; c0 += CH) {
      f4 sv[CH];
      float cm = -INFINITY;
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int tk = c0 + u;
        if (tk >= NT) break;
        sv[u] = mfma16(kb[tk], qb, ld4(&Kb[tk * 16 + 4 * q]));
        cm = vmax(vmax(vmax(cm, sv[u][0]), sv[u][1]), vmax(sv[u][2], sv[u][3]));
      }
      cm = xmax(cm);
      const float mn = vmax(m, cm);
      const float msn = mn == -INFINITY ? 0.f : mn * scale2;
      if (c0 > 0) {
        // rescale by 2^(ms - msn) (l and o are 0 while no key was valid); rows 4q + e of o need
        // query 4q + e's factor
        const float al = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - msn);
        l *= al;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] *= __shfl(al, 4 * q + e, 64);
      }
      m = mn;
      ms = msn;
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int tk = c0 + u;
        if (tk >= NT) break;
        bool kp[4] = {true, true, true, true};
        if (DROP) attn_keep4b(dk, leven, rowbase + tk * 16 + 4 * q, kp);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[u][e], scale2, -ms));
          l += pv;
          sv[u][e] = kp[e] ? pv : 0.f;  // P∘Z / (1/(1-p)): the factor goes on the output row
        }
        o = mfma16(bf4(sv[u]), col_frag16(Vs, tk * 16, r, q), o);
      }
    }
    l = xsum(l);
    if (q == 0 && i < L) lse[(int64_t)bh * L + i] = (ms + __builtin_amdgcn_logf(l)) * kLn2;
    const float rl = DROP ? __builtin_amdgcn_rcpf(l) * dk.scale : __builtin_amdgcn_rcpf(l);
    f4 on;
#pragma unroll
    for (int e = 0; e < 4; ++e) on[e] = o[e] * __shfl(rl, 4 * q + e, 64);
    const f4 v = tile_rows<kRowP>(T, on, r, q, lane);
    const int row = tq * 16 + (lane >> 2);
    if (row < L) st4q(out + ((int64_t)b * L + row) * d + h * 16 + 4 * (lane & 3), v);
  }
  if constexpr (NR > 0) {
    // Shared query tiles (C5, L = 200: tile 12 of 13, which made wave 0 do 4 tiles against 3):
    // wave w takes key tiles tk = w mod 4 of each, the partial (max, sum, P V) of the four waves
    // are merged through LDS in wave order (the online-softmax rescale), and wave x writes tile
    // NTF + x.
    __shared__ float mlp[4][NR][2][16];
    __shared__ __attribute__((aligned(16))) f4 olp[4][NR][64];
#pragma unroll
    for (int x = 0; x < NR; ++x) {
      const int tq = NTF + x;
      const int i = tq * 16 + r;
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      const s4v qb = row_frag16(Qs, i, q);
      f4 sv[NT];
      float m = -INFINITY;
#pragma unroll
      for (int tk = 0; tk < NT; ++tk) {
        if ((tk & 3) != wave) continue;  // wave-uniform
        sv[tk] = mfma16(kb[tk], qb, ld4(&Kb[tk * 16 + 4 * q]));
        m = vmax(vmax(vmax(m, sv[tk][0]), sv[tk][1]), vmax(sv[tk][2], sv[tk][3]));
      }
      m = xmax(m);
      m = m == -INFINITY ? -INFINITY : m * scale2;  // the merge below reads -inf as "no valid key"
      const float ms = m == -INFINITY ? 0.f : m;
      float l = 0.f;
      const uint32_t rowbase = ((uint32_t)bh * (uint32_t)L + (uint32_t)i) * (uint32_t)L;
      f4 o = z;
#pragma unroll
      for (int tk = 0; tk < NT; ++tk) {
        if ((tk & 3) != wave) continue;
        bool kp[4] = {true, true, true, true};
        if (DROP) attn_keep4b(dk, leven, rowbase + tk * 16 + 4 * q, kp);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[tk][e], scale2, -ms));
          l += pv;
          sv[tk][e] = kp[e] ? pv : 0.f;
        }
        o = mfma16(bf4(sv[tk]), col_frag16(Vs, tk * 16, r, q), o);
      }
      l = xsum(l);
      if (q == 0) {
        mlp[wave][x][0][r] = m;
        mlp[wave][x][1][r] = l;
      }
      olp[wave][x][lane] = o;
    }
    __syncthreads();
    if (wave < NR) {
      const int x = wave, tq = NTF + x;
      // this lane's rows: queries 4q + e (the MFMA output layout); the lse of query r (q == 0)
      f4 on;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int qi = 4 * q + e;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) M = fmaxf(M, mlp[w][x][0][qi]);
        float lt = 0.f, ot = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float mw = mlp[w][x][0][qi];
          const float f = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);
          lt += f * mlp[w][x][1][qi];
          ot += f * olp[w][x][lane][e];
        }
        on[e] = ot * (DROP ? __builtin_amdgcn_rcpf(lt) * dk.scale : __builtin_amdgcn_rcpf(lt));
      }
      const int i = tq * 16 + r;
      if (q == 0 && i < L) {
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; ++w) M = fmaxf(M, mlp[w][x][0][r]);
        float lt = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float mw = mlp[w][x][0][r];
          lt += (mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M)) * mlp[w][x][1][r];
        }
        lse[(int64_t)bh * L + i] = (M + __builtin_amdgcn_logf(lt)) * kLn2;
      }
      const f4 v = tile_rows<kRowP>(T, on, r, q, lane);
      const int row = tq * 16 + (lane >> 2);
      if (row < L) st4q(out + ((int64_t)b * L + row) * d + h * 16 + 4 * (lane & 3), v);
    }
  }
}

// Single-pass backward: key-parallel (the lane's query-on-row tiles feed dV and dK), plus dQ.
// dQ = dS K contracts over keys, so the lane's dS tile (query on the row) is transposed through
// the wave's LDS image into an A fragment; each wave keeps partial dQ tiles for every query tile
// in registers and the four partials are summed in wave order at the end (deterministic). P and
// dP are computed once per (query, key) pair instead of twice (one exp, half a hash per pair).
// Balance: wave w owns key tiles w, w + 4, ... below NTF = 4 floor(NT / 4); the NT % 4 tiles past
// them are shared, wave w taking their pairs with query tiles tq = w mod 4, and their dK / dV
// partials are summed in wave order at the end. (C5, L = 200, NT = 13: the busiest wave had 4 key
// tiles = 52 (query, key) tile pairs against 39 for the others; now 43 / 42 / 42 / 42.)
template <int NT, bool DROP, bool QB>
__global__ __launch_bounds__(256, 3) void attn_bwd_long1_bf16_kernel(
    const void* __restrict__ qkv_, const uint8_t* __restrict__ key_pad,
    const float* __restrict__ out, const float* __restrict__ dout, const float* __restrict__ lse,
    void* __restrict__ dqkv_, int B, int L, int d, int H, float scale, float pdrop,
    const int64_t* __restrict__ key, int site) {
  constexpr int LP = NT * 16;
  constexpr int NW0 = NT / 4;       // key tiles owned by each wave
  constexpr int NTF = 4 * NW0;      // the first shared key tile
  constexpr int NR = NT - NTF;      // shared key tiles
  constexpr int NW = NW0 + NR;      // key tiles a wave visits
  constexpr int TP = 20;
  // Q, K, V, dO as bf16; then the wave-ordered dQ and shared-tile dK / dV accumulators (fp32)
  __shared__ __attribute__((aligned(16))) __bf16 img[4][LP][kRowPB];
  static_assert((LP * 16 + NR * 2 * 256) * 4 <= 4 * LP * kRowPB * 2, "accumulators fit the image");
  __shared__ __attribute__((aligned(16))) float L2s[LP];  // lse * log2(e)
  __shared__ __attribute__((aligned(16))) float Ds[LP];   // D_i = dO_i . O_i
  __shared__ float Kv[LP];                                // 1: key j is valid
  // per wave: the NW dS tiles of one query tile staged as bf16 (the dQ product's operand rounding,
  // so the same bits) for the transpose, all written before one barrier and read after it -- the
  // key tiles' chains overlap instead of meeting a barrier pair each; then the fp32 [16][TP]
  // image of tile_rows. (52 KB in all: three workgroups per CU)
  constexpr int TPB = 20;
  constexpr int TB_HALFS = NW * 16 * TPB > 2 * 16 * TP ? NW * 16 * TPB : 2 * 16 * TP;
  __shared__ __attribute__((aligned(16))) __bf16 Tbs[4][TB_HALFS];
  __bf16(*Qs)[kRowPB] = img[0];
  __bf16(*Ks)[kRowPB] = img[1];
  __bf16(*Vs)[kRowPB] = img[2];
  __bf16(*Gs)[kRowPB] = img[3];
  int b, h;
  if (!map_bh(B, H, b, h)) return;  // uniform over the workgroup
  const int bh = b * H + h;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = lane & 15, q = lane >> 4;
  const int ld = 3 * d;
  typedef typename std::conditional<QB, __bf16, float>::type QT;
  const QT* base = reinterpret_cast<const QT*>(qkv_) + (int64_t)b * L * ld + h * 16;
  load_head_image16<LP>(base, ld, L, 0, Qs);
  load_head_image16<LP>(base, ld, L, d, Ks);
  load_head_image16<LP>(base, ld, L, 2 * d, Vs);
  load_head_image16<LP>(dout + (int64_t)b * L * d + h * 16, d, L, 0, Gs);
  for (int i = threadIdx.x; i < LP; i += 256) {
    float Di = 0.f, li = 0.f, kv = 0.f;
    if (i < L) {
      const float* o = out + ((int64_t)b * L + i) * d + h * 16;
      const float* g = dout + ((int64_t)b * L + i) * d + h * 16;
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        const f4 ov = ld4(o + c), gv = ld4(g + c);
        Di += ov[0] * gv[0] + ov[1] * gv[1] + ov[2] * gv[2] + ov[3] * gv[3];
      }
      const float ls = lse[(int64_t)bh * L + i];
      li = ls == -INFINITY ? 0.f : ls * kLog2e;  // a row with no valid key: P = 0 below
      kv = key_pad[(int64_t)b * L + i] == 0 ? 1.f : 0.f;
    } else {
      li = INFINITY;  // query rows past L: P = 0 without a select
    }
    Ds[i] = Di;
    L2s[i] = li;
    Kv[i] = kv;
  }
  DropKey dk;
  if (DROP) dk = make_key(key, site, pdrop);
  const bool leven = (L & 1) == 0;
  const float scale2 = scale * kLog2e;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  float* T = reinterpret_cast<float*>(Tbs[wave]);
  __bf16* Tb = Tbs[wave];
  QT* dbase = reinterpret_cast<QT*>(dqkv_) + (int64_t)b * L * ld + h * 16;
  __syncthreads();

  s4v kr[NW], vr[NW], kc[NW];
  float kval[NW];
  f4 dk_acc[NW], dv_acc[NW], dq_acc[NT];
#pragma unroll
  for (int u = 0; u < NW; ++u) {
    const int tk = u < NW0 ? wave + 4 * u : NTF + (u - NW0);
    kr[u] = row_frag16(Ks, tk * 16 + r, q);
    vr[u] = row_frag16(Vs, tk * 16 + r, q);
    kc[u] = col_frag16(Ks, tk * 16, r, q);
    kval[u] = Kv[tk * 16 + r];
    dk_acc[u] = dv_acc[u] = z;
  }
#pragma unroll
  for (int tq = 0; tq < NT; ++tq) {
    const s4v qr = row_frag16(Qs, tq * 16 + r, q);
    const s4v gr = row_frag16(Gs, tq * 16 + r, q);
    const s4v qc[1] = {col_frag16(Qs, tq * 16, r, q)};
    const s4v gc[1] = {col_frag16(Gs, tq * 16, r, q)};
    const f4 l2 = ld4(&L2s[tq * 16 + 4 * q]);
    const f4 Dq = ld4(&Ds[tq * 16 + 4 * q]);
    dq_acc[tq] = z;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int tk = u < NW0 ? wave + 4 * u : NTF + (u - NW0);
      if (u >= NW0 && (tq & 3) != wave) continue;  // a shared tile: this query tile's wave only
      const f4 sacc = mfma16(qr, kr[u], z);  // S[query 16 tq + 4q + e][key 16 tk + r]
      const f4 pacc = mfma16(gr, vr[u], z);  // dP[query][key] = dO_i . V_j
      float mk[4] = {1.f, 1.f, 1.f, 1.f};
      if (DROP)
        keep_col4(dk, leven, ((uint32_t)bh * (uint32_t)L + (uint32_t)(tq * 16 + 4 * q)) * (uint32_t)L,
                  (uint32_t)L, (uint32_t)(tk * 16 + r), r, mk);
      f4 pz, ds;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // l2 is +inf past L and 0 for a row with no valid key; the key's validity is lane-uniform
        float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[e], scale2, -l2[e]));
        pv = kval[u] != 0.f ? pv : 0.f;
        pz[e] = pv * mk[e];
        ds[e] = pv * __builtin_fmaf(mk[e], pacc[e], -Dq[e]);
      }
      dv_acc[u] = mfma16(bf4(pz), gc[0], dv_acc[u]);  // (P∘Z)^T dO
      const s4v dsb = bf4(ds);
      dk_acc[u] = mfma16(dsb, qc[0], dk_acc[u]);  // dS^T Q
      // dS with the key on the k side: Tb[u][query][key] -> lane (r, q) reads row r, keys 4q..4q+3
      // (measured: an 8-byte [key][query] row store read back with tr_col spilled at this
      // kernel's 168-VGPR budget)
      const bf4v dh = __builtin_bit_cast(bf4v, dsb);
#pragma unroll
      for (int e = 0; e < 4; ++e) Tb[u * 16 * TPB + (4 * q + e) * TPB + r] = dh[e];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      if (u >= NW0 && (tq & 3) != wave) continue;
      const s4v dst = *reinterpret_cast<const s4v*>(&Tb[u * 16 * TPB + r * TPB + 4 * q]);
      dq_acc[tq] = mfma16(dst, kc[u], dq_acc[tq]);  // dS K: [query 4q + e][c = r]
    }
    __builtin_amdgcn_wave_barrier();
  }
  // dK / dV rows of this wave's own key tiles
#pragma unroll
  for (int u = 0; u < NW0; ++u) {
    const int tk = wave + 4 * u;
    const f4 vk = tile_rows<TP>(T, dk_acc[u] * scale, r, q, lane);
    const f4 vv = tile_rows<TP>(T, dv_acc[u], r, q, lane);
    const int row = tk * 16 + (lane >> 2);
    if (row < L) {
      st4q(dbase + (int64_t)row * ld + d + 4 * (lane & 3), vk);
      st4q(dbase + (int64_t)row * ld + 2 * d + 4 * (lane & 3), vv);
    }
  }
  // dQ partials (every query tile) and the shared key tiles' dK / dV partials summed in wave order
  // through one fp32 accumulator in the (now free) images: ((w0 + w1) + w2) + w3
  __syncthreads();  // the images are free
  float* accq = reinterpret_cast<float*>(&img[0][0][0]);  // [LP][16]
  f4* accs = reinterpret_cast<f4*>(accq + LP * 16);       // [NR][dk, dv][lane]
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int tq = 0; tq < NT; ++tq)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float* pp = accq + (tq * 16 + 4 * q + e) * 16 + r;
          *pp = (w == 0 ? 0.f : *pp) + dq_acc[tq][e];
        }
#pragma unroll
      for (int x = 0; x < NR; ++x) {
        f4* pk = accs + (x * 2 + 0) * 64 + lane;
        f4* pv = accs + (x * 2 + 1) * 64 + lane;
        *pk = (w == 0 ? z : *pk) + dk_acc[NW0 + x];
        *pv = (w == 0 ? z : *pv) + dv_acc[NW0 + x];
      }
    }
    __syncthreads();
  }
  if constexpr (NR > 0) {
    if (wave < NR) {  // wave x finishes shared key tile NTF + x
      const int x = wave;
      const f4 vk = tile_rows<TP>(T, accs[(x * 2 + 0) * 64 + lane] * scale, r, q, lane);
      const f4 vv = tile_rows<TP>(T, accs[(x * 2 + 1) * 64 + lane], r, q, lane);
      const int row = (NTF + x) * 16 + (lane >> 2);
      if (row < L) {
        st4q(dbase + (int64_t)row * ld + d + 4 * (lane & 3), vk);
        st4q(dbase + (int64_t)row * ld + 2 * d + 4 * (lane & 3), vv);
      }
    }
  }
  for (int e = threadIdx.x; e < LP * 4; e += 256) {
    const int row = e >> 2, c4 = (e & 3) * 4;
    if (row >= L) continue;
    st4q(dbase + (int64_t)row * ld + c4, ld4(accq + row * 16 + c4) * scale);
  }
}

int threads_for(int L) {
  int t = ((L + 63) / 64) * 64;
  return t > 256 ? 256 : t;
}

}  // namespace
}  // namespace rs

using namespace rs;

// bf16 compute mode, head_dim 16, 64 < L <= 256 (fp32 or bf16 qkv): the long-history MFMA kernels
// (L <= 64 takes the wave-per-(b, h) kernels above them in the dispatch)
static bool long_bf16_ok(int hd, int L, int B, int H, int flags) {
  return hd == 16 && L > 64 && L <= 256 && (flags & RS_GEMM_BF16) &&
         (int64_t)B * H * L * L < ((int64_t)1 << 32) && !getenv_flag("RSYS_ATTN_VALU");
}

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
                           int site, int flags, void* stream, uint16_t* zbits) {
  RS_CHECK_ARG(qkv && key_pad && out && lse, "rs_attn_fwd: null pointer");
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1 && d % H == 0, "rs_attn_fwd: bad shape");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_attn_fwd: bad dropout p=%f", p);
  const int hd = d / H;
  RS_CHECK_ARG(hd == 8 || hd == 16 || hd == 32 || hd == 64, "rs_attn_fwd: head_dim %d unsupported", hd);
  if (B == 0) return 0;
  const size_t lds = (size_t)(2 * L * hd + L) * sizeof(float);
  RS_CHECK_ARG(lds <= 64 * 1024 || long_bf16_ok(hd, L, B, H, flags), "rs_attn_fwd: L=%d hd=%d exceeds LDS", L, hd);
  RS_CHECK_ARG(d % 4 == 0 && aligned16(qkv) && aligned16(out), "rs_attn_fwd: needs 16-byte aligned rows");
  RS_CHECK_ARG(!(flags & RS_ATTN_QKV_BF16) || ((flags & RS_GEMM_BF16) && hd == 16 && L <= 256 &&
                                                 !getenv_flag("RSYS_ATTN_VALU")),
               "rs_attn_fwd: bf16 qkv storage needs the bf16 MFMA path (head_dim 16, L <= 256)");
  hipStream_t st = as_stream(stream);
  if (hd == 16 && L <= 64 && (int64_t)B * H * L * L < ((int64_t)1 << 32) && !getenv_flag("RSYS_ATTN_VALU")) {
    const int nt = (L + 15) / 16;
    const dim3 g4(cdiv((int64_t)B * H, 4));
    const bool bf = (flags & RS_GEMM_BF16) != 0;
    const bool qb = (flags & RS_ATTN_QKV_BF16) != 0;
#define RS_AF(NTV)                                                                                  \
  if (nt == NTV) {                                                                                  \
    if (qb && p > 0.f && zbits) attn_fwd_bf16_kernel<NTV, true, true, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site, zbits); \
    else if (bf && !qb && p > 0.f && zbits) attn_fwd_bf16_kernel<NTV, true, false, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site, zbits); \
    else if (qb && p > 0.f) attn_fwd_bf16_kernel<NTV, true, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (qb) attn_fwd_bf16_kernel<NTV, false, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (bf && p > 0.f) attn_fwd_bf16_kernel<NTV, true, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (bf) attn_fwd_bf16_kernel<NTV, false, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (p > 0.f) attn_fwd_mfma_kernel<NTV, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else attn_fwd_mfma_kernel<NTV, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
  }
    RS_AF(1) RS_AF(2) RS_AF(3) RS_AF(4)
#undef RS_AF
    RS_CHECK_LAUNCH("rs_attn_fwd mfma");
    return 0;
  }
  if (long_bf16_ok(hd, L, B, H, flags)) {
    const dim3 gl(bh_grid(B, H));
#define RS_AFL(NTV)                                                                                 \
  if (nt == NTV) {                                                                                  \
    if (qb && p > 0.f) attn_fwd_long_bf16_kernel<NTV, true, true><<<gl, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (qb) attn_fwd_long_bf16_kernel<NTV, false, true><<<gl, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else if (p > 0.f) attn_fwd_long_bf16_kernel<NTV, true, false><<<gl, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
    else attn_fwd_long_bf16_kernel<NTV, false, false><<<gl, 256, 0, st>>>(qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site); \
  }
    const int nt = (L + 15) / 16;
    const bool qb = (flags & RS_ATTN_QKV_BF16) != 0;
    RS_AFL(5) RS_AFL(6) RS_AFL(7) RS_AFL(8) RS_AFL(9) RS_AFL(10) RS_AFL(11)
    RS_AFL(12) RS_AFL(13) RS_AFL(14) RS_AFL(15) RS_AFL(16)
#undef RS_AFL
    RS_CHECK_LAUNCH("rs_attn_fwd long bf16");
    return 0;
  }
  dim3 grid(bh_grid(B, H));
  int thr = threads_for(L);
  RS_ATTN_DISPATCH(hd, p > 0.f, attn_fwd_kernel, qkv, key_pad, out, lse, B, L, d, H, scale, p, key, site);
  RS_CHECK_LAUNCH("rs_attn_fwd");
  return 0;
}

extern "C" int rs_attn_bwd(const float* qkv, const uint8_t* key_pad, const float* out,
                           const float* dout, const float* lse, float* dqkv, int B, int L, int d,
                           int H, float scale, float p, const int64_t* key, int site, int flags,
                           void* stream, const uint16_t* zbits) {
  RS_CHECK_ARG(qkv && key_pad && out && dout && lse && dqkv, "rs_attn_bwd: null pointer");
  RS_CHECK_ARG(B >= 0 && L >= 1 && H >= 1 && d % H == 0, "rs_attn_bwd: bad shape");
  RS_CHECK_ARG(p >= 0.f && p < 1.f && (p == 0.f || key), "rs_attn_bwd: bad dropout p=%f", p);
  const int hd = d / H;
  RS_CHECK_ARG(hd == 8 || hd == 16 || hd == 32 || hd == 64, "rs_attn_bwd: head_dim %d unsupported", hd);
  if (B == 0) return 0;
  const size_t lds = (size_t)(4 * L * hd + 3 * L) * sizeof(float);
  RS_CHECK_ARG(lds <= 64 * 1024 || long_bf16_ok(hd, L, B, H, flags), "rs_attn_bwd: L=%d hd=%d exceeds LDS", L, hd);
  RS_CHECK_ARG(d % 4 == 0 && aligned16(qkv) && aligned16(dout), "rs_attn_bwd: needs 16-byte aligned rows");
  RS_CHECK_ARG(!(flags & RS_ATTN_QKV_BF16) || ((flags & RS_GEMM_BF16) && hd == 16 && L <= 256 &&
                                                 !getenv_flag("RSYS_ATTN_VALU")),
               "rs_attn_bwd: bf16 qkv storage needs the bf16 MFMA path (head_dim 16, L <= 256)");
  hipStream_t st = as_stream(stream);
  if (hd == 16 && L <= 64 && (int64_t)B * H * L * L < ((int64_t)1 << 32) && !getenv_flag("RSYS_ATTN_VALU")) {
    RS_CHECK_ARG(aligned16(out), "rs_attn_bwd: needs 16-byte aligned rows");
    const int nt = (L + 15) / 16;
    const dim3 g4(cdiv((int64_t)B * H, 4));
    const bool bf = (flags & RS_GEMM_BF16) != 0;
    const bool qb = (flags & RS_ATTN_QKV_BF16) != 0;
#define RS_AB(NTV)                                                                                  \
  if (nt == NTV) {                                                                                  \
    if (qb && p > 0.f && zbits) attn_bwd_bf16_kernel<NTV, true, true, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site, zbits); \
    else if (bf && !qb && p > 0.f && zbits) attn_bwd_bf16_kernel<NTV, true, false, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site, zbits); \
    else if (qb && p > 0.f) attn_bwd_bf16_kernel<NTV, true, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (qb) attn_bwd_bf16_kernel<NTV, false, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (bf && p > 0.f) attn_bwd_bf16_kernel<NTV, true, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (bf) attn_bwd_bf16_kernel<NTV, false, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (p > 0.f) attn_bwd_mfma_kernel<NTV, true><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else attn_bwd_mfma_kernel<NTV, false><<<g4, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
  }
    RS_AB(1) RS_AB(2) RS_AB(3) RS_AB(4)
#undef RS_AB
    RS_CHECK_LAUNCH("rs_attn_bwd mfma");
    return 0;
  }
  if (long_bf16_ok(hd, L, B, H, flags)) {
    RS_CHECK_ARG(aligned16(out), "rs_attn_bwd: needs 16-byte aligned rows");
    const dim3 gl(bh_grid(B, H));
#define RS_ABL(NTV)                                                                                 \
  if (nt == NTV) {                                                                                  \
    if (qb && p > 0.f) attn_bwd_long1_bf16_kernel<NTV, true, true><<<gl, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (qb) attn_bwd_long1_bf16_kernel<NTV, false, true><<<gl, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else if (p > 0.f) attn_bwd_long1_bf16_kernel<NTV, true, false><<<gl, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
    else attn_bwd_long1_bf16_kernel<NTV, false, false><<<gl, 256, 0, st>>>(qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale, p, key, site); \
  }
    const int nt = (L + 15) / 16;
    const bool qb = (flags & RS_ATTN_QKV_BF16) != 0;
    RS_ABL(5) RS_ABL(6) RS_ABL(7) RS_ABL(8) RS_ABL(9) RS_ABL(10) RS_ABL(11)
    RS_ABL(12) RS_ABL(13) RS_ABL(14) RS_ABL(15) RS_ABL(16)
#undef RS_ABL
    RS_CHECK_LAUNCH("rs_attn_bwd long bf16");
    return 0;
  }
  dim3 grid(bh_grid(B, H));
  int thr = threads_for(L);
  RS_ATTN_DISPATCH(hd, p > 0.f, attn_bwd_kernel, qkv, key_pad, out, dout, lse, dqkv, B, L, d, H, scale,
                   p, key, site);
  RS_CHECK_LAUNCH("rs_attn_bwd");
  return 0;
}
