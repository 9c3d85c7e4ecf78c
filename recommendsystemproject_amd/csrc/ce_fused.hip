// In-batch sampled-softmax loss with the batch similarity never stored (bf16 compute mode).
//
// Reference: TwoTowerModel.compute_loss (TwoTowerModel.py:81-140): logits = U I^T / T, the
// off-diagonal entries whose item ids collide set to -1e9 (trap T12), the N hard-negative
// logits U_i . H_in / T appended, cross_entropy(logits, arange(B)), mean over the batch.
//
// The unfused path writes S = U I^T ([B, B] fp32, 64 MB at B = 4096), reads it twice for the
// log-sum-exp, rewrites it as dS and reads it twice more for dU = dS I and dI = dS^T U. Here the
// 32 x 32 tiles of S are recomputed on v_mfma_f32_32x32x16_bf16 wherever they are needed and
// consumed in registers:
//   fwd : per user, an online (max, sum-exp) over its item tiles -> partials per column split;
//   dU  : per user block, dS^T tiles (items x users) become the B operand of dU^T += I^T dS^T
//         with no data movement (an accumulator tile summed over its ROW index is already a
//         bf16 operand after pairwise packing); I^T comes from the staged item tile through
//         ds_read_b64_tr_b16;
//   dI  : the same kernel with the roles of U and I exchanged (dI^T += U^T dS).
// One kernel template serves all three: the wave OWNS 32 rows (users for fwd / dU, items for
// dI) whose bf16 fragments stay in registers, and streams 32-row tiles of the other matrix
// through LDS. Column splits give >= 256 workgroups at B = 4096; their partials are reduced in
// a fixed order (deterministic).
//
// fp32 compute mode runs the same kernels on v_mfma_f32_32x32x2_f32 (exact f32 products, a
// k-ordered fma chain; 64 cycles per instruction and SIMD, 1/16 of the bf16 rate): the streamed
// tiles are staged in LDS as fp32, the owned fragments are fp32 registers, and the dS^T
// accumulator elements are the B operand of the gradient MFMA as they stand (no packing).
// At that rate recomputing S twice in the backward cost half of its MFMA time (64 of 128
// instructions per tile), so the fp32 forward also stores S ([B][ldS] fp32, 64 MB at B = 4096,
// written as the tiles are produced) and the backward reads each tile's 4 KB back one tile ahead
// instead: the same bits as the recomputation (the products U[u][k] I[i][k] and their k order
// are the same in all three modes), half the backward's flops for 2 x B^2 x 4 bytes of reads.
#include <type_traits>

#include "common.h"

namespace rs {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));

constexpr int kOwnW = 32;    // owned rows per wave
constexpr int kWaves = 4;    // owned rows per workgroup: 128
constexpr int kTile = 32;    // streamed rows per tile
constexpr float kMasked = -1e9f;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

struct HStrideArgs {
  int64_t row, slot;  // hard-negative H element (i, n, c) at i*row + n*slot + c
};

struct CeArgs {
  const float* own;     // [B, D] owned rows (U for fwd / dU, I for dI)
  const float* str;     // [B, D] streamed rows
  int B;
  float invT;
  const int64_t* ids;   // nullable: item ids (collision mask)
  int64_t id_stride;
  int split_rows;       // streamed rows per column split (multiple of kTile)
  const float* lse;     // bwd: [B] natural log-sum-exp per user
  const float* grad_out;  // bwd: d loss (nullable -> 1)
  float* part_m;        // fwd: [NS][B]
  float* part_s;        // fwd: [NS][B]
  float* diag;          // fwd: [B] S_ii / T
  float* part_d;        // bwd: [NS][B][D]
  float* S;             // fp32 mode: [B][ldS] raw U I^T, written by the forward, read by the backward
  int ldS;
  const __bf16* strb;   // bf16 backward: the streamed rows pre-rounded to bf16 (the same bits the
                        // staging rounds to), half the bytes per tile: twice the tiles per batch
};

__device__ __forceinline__ bf16x8 cvt8(const floatx4& a, const floatx4& b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

__device__ __forceinline__ bf16x8 tr_frag(const __bf16* lo, const __bf16* hi) {
  typedef __attribute__((address_space(3))) shortx4* lptr;
  const shortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lo));
  const shortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(hi));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// MODE 0: forward statistics (own = U, str = I)
// MODE 1: dU (own = U, str = I; lse of the owned user)
// MODE 2: dI (own = I, str = U; lse of the streamed user)
// streamed tiles staged per batch of kBT: one batch's loads are in flight while the previous
// batch is consumed from the other LDS half. With one tile per stage every tile exposed an L2/MALL
// round trip (the loop ran at ~3,600 cycles per tile against ~600 of MFMA and exp work). The
// backward stages kBT / 2 tiles per batch: its gradient accumulators leave no room for a 4-tile
// register stage at two waves per SIMD.
// fp32 tiles take twice the LDS: the forward stages 2 tiles per batch, the backward 1 (the LDS
// image holds 2 x 2 tiles, 68 KB: two workgroups per CU).
constexpr int kBT = 4;
template <int MODE, bool F32, bool SB = false>
constexpr int batch_tiles() {
  return F32 ? (MODE == 0 ? kBT / 2 : kBT / 4) : ((MODE == 0 || SB) ? kBT : kBT / 2);
}

// v_exp_f32 directly: exp2f() adds a denormal-range fix-up (compare, select, ldexp) per call
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

template <int D, bool F32>
struct CeLds {
  using E = std::conditional_t<F32, float, __bf16>;
  // row pitch: bf16 D + 8 (ds_read_b64_tr_b16 / b128 conflict-free), fp32 D + 4 (the b128 reads
  // of 16 consecutive rows cover the 64 banks once)
  static constexpr int PT = F32 ? D + 4 : D + 8;
  static constexpr int NT = F32 ? kBT / 2 : kBT;  // tiles per LDS half
  E Ts[2][NT * kTile * PT];
  int64_t sid[2][NT * kTile];
  float slse[2][NT * kTile];
};

template <int D, int MODE, bool F32, bool SB = false>
__device__ __forceinline__ void ce_tile_body(const CeArgs& a, const int split, CeLds<D, F32>& L) {
  static_assert(!SB || (!F32 && MODE != 0), "bf16-streamed tiles: the bf16 backward");
  using E = typename CeLds<D, F32>::E;
  constexpr int KS = D / 16;          // 32x32x16 k-steps over the embedding (bf16)
  constexpr int PT = CeLds<D, F32>::PT;
  constexpr int DB = D / 32;          // 32-wide blocks of the gradient
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int B = a.B;
  const int o = blockIdx.x * (kOwnW * kWaves) + wave * kOwnW + c;  // this lane's owned row
  const bool o_ok = o < B;
  const int t_begin = split * a.split_rows;
  const int t_end = min(B, t_begin + a.split_rows);

  // owned fragments: B operand of the S tile. bf16: lane (c, h) holds own[o][16 s + 8 h .. +7];
  // fp32: own[o][h D/2 + s] for k-step s (k-steps pair embedding columns s and D/2 + s)
  constexpr bool SLOAD = F32 && MODE != 0;  // S tiles read back instead of recomputed
  bf16x8 ob[F32 ? 1 : KS];
  float obf[F32 && !SLOAD ? D / 2 : 1];
  if constexpr (SLOAD) {
  } else if constexpr (F32) {
#pragma unroll
    for (int s4 = 0; s4 < D / 8; ++s4) {
      floatx4 x = {0.f, 0.f, 0.f, 0.f};
      if (o_ok) x = *reinterpret_cast<const floatx4*>(a.own + (int64_t)o * D + h * (D / 2) + 4 * s4);
#pragma unroll
      for (int j = 0; j < 4; ++j) obf[4 * s4 + j] = x[j];
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      floatx4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = x0;
      if (o_ok) {
        const float* p = a.own + (int64_t)o * D + 16 * s + 8 * h;
        x0 = *reinterpret_cast<const floatx4*>(p);
        x1 = *reinterpret_cast<const floatx4*>(p + 4);
      }
      ob[s] = cvt8(x0, x1);
    }
  }
  const int64_t id_o = (a.ids && o_ok) ? a.ids[(int64_t)o * a.id_stride] : 0;
  const int o_base = blockIdx.x * (kOwnW * kWaves) + __builtin_amdgcn_readfirstlane(wave) * kOwnW;
  const bool wave_ok = o_base + kOwnW <= B;                           // every owned row valid
  const float sc2 = a.invT * kLog2e;  // S -> log2-domain logits
  float g = 0.f, lse2_o = 0.f;
  if constexpr (MODE != 0) {
    g = (a.grad_out ? *a.grad_out : 1.f) / (float)B * a.invT;  // d loss / d S = dlogits / T
    if constexpr (MODE == 1) lse2_o = o_ok ? a.lse[o] * kLog2e : 0.f;
  }
  float run_m = -INFINITY, run_s = 0.f;  // fwd: online statistics (log2 domain) of this lane's values
  floatx16 gacc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) gacc[i][e] = 0.f;

  // batch staging: kBT tiles of 32 rows x D fp32 -> bf16 LDS, float4 per slot
  constexpr int NTHR = 64 * kWaves;
  constexpr int SL = kTile * D / 4 / NTHR;  // float4 slots per thread per tile
  constexpr int SLB = kTile * D / 8 / NTHR;  // bf16x8 slots per thread per tile (SB)
  constexpr int BT = batch_tiles<MODE, F32, SB>();  // tiles per batch
  constexpr int BR = BT * kTile;            // rows per batch
  static_assert(BR <= NTHR, "one id / lse per thread and batch row");
  struct Stage {
    floatx4 v[SB ? 1 : BT][SB ? 1 : SL];
    bf16x8 vb[SB ? BT : 1][SB ? SLB : 1];
    int64_t id;
    float l;
  };
  Stage R;
  // loads are unconditional (row index clamped to B - 1; rows >= B are masked when consumed):
  // a guarded load would sit in its own branch, and the waitcnt pass then drains vmcnt(0) at the
  // join -- waiting for the prefetch it was meant to overlap
  auto load_batch = [&](int t0) {
    if constexpr (SB) {
#pragma unroll
      for (int k = 0; k < BT; ++k)
#pragma unroll
        for (int i = 0; i < SLB; ++i) {
          const int slot = tid + NTHR * i;
          const int row = slot / (D / 8), col = (slot % (D / 8)) * 8;
          const int t = min(t0 + k * kTile + row, B - 1);
          R.vb[k][i] = *reinterpret_cast<const bf16x8*>(a.strb + (int64_t)t * D + col);
        }
    } else {
#pragma unroll
      for (int k = 0; k < BT; ++k)
#pragma unroll
        for (int i = 0; i < SL; ++i) {
          const int slot = tid + NTHR * i;
          const int row = slot / (D / 4), col = (slot % (D / 4)) * 4;
          const int t = min(t0 + k * kTile + row, B - 1);
          R.v[k][i] = *reinterpret_cast<const floatx4*>(a.str + (int64_t)t * D + col);
        }
    }
    const int t = min(t0 + (tid & (BR - 1)), B - 1);
    R.id = a.ids ? a.ids[(int64_t)t * a.id_stride] : 0;
    if constexpr (MODE == 2) R.l = a.lse[t] * kLog2e;  // staged in the log2 domain
  };
  auto store_batch = [&](int hf) {
    if constexpr (SB) {
#pragma unroll
      for (int k = 0; k < BT; ++k)
#pragma unroll
        for (int i = 0; i < SLB; ++i) {
          const int slot = tid + NTHR * i;
          const int row = k * kTile + slot / (D / 8), col = (slot % (D / 8)) * 8;
          *reinterpret_cast<bf16x8*>(&L.Ts[hf][row * PT + col]) = R.vb[k][i];
        }
    }
#pragma unroll
    for (int k = 0; k < (SB ? 0 : BT); ++k)
#pragma unroll
      for (int i = 0; i < SL; ++i) {
        const int slot = tid + NTHR * i;
        const int row = k * kTile + slot / (D / 4), col = (slot % (D / 4)) * 4;
        if constexpr (F32) {
          *reinterpret_cast<floatx4*>(&L.Ts[hf][row * PT + col]) = R.v[k][i];
        } else {
          bf16x4 v;
          v[0] = (__bf16)R.v[k][i][0]; v[1] = (__bf16)R.v[k][i][1];
          v[2] = (__bf16)R.v[k][i][2]; v[3] = (__bf16)R.v[k][i][3];
          *reinterpret_cast<bf16x4*>(&L.Ts[hf][row * PT + col]) = v;
        }
      }
    if (tid < BR) {
      L.sid[hf][tid] = R.id;
      if constexpr (MODE == 2) L.slse[hf][tid] = R.l;
    }
  };
  float dg = 0.f;  // fwd: S_oo / T, captured by the lane that meets the diagonal
  bool has_dg = false;
  // fp32 backward: the S tile at streamed rows t0.. of this lane's element layout (row t = t0 +
  // 8(e>>2) + 4h + (e&3), owned column o), loaded one tile ahead. dU (MODE 1): S[o][t], four
  // float4 per lane; dI (MODE 2): S[t][o], 16 scalars, coalesced over the lanes' items. Rows and
  // columns past B are clamped (those elements are masked where consumed).
  const int o_c = min(o, B - 1);
  auto load_s = [&](int t0, floatx16& sv) {
    if constexpr (SLOAD) {
      if constexpr (MODE == 1) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const floatx4 v = *reinterpret_cast<const floatx4*>(a.S + (int64_t)o_c * a.ldS + min(t0, a.ldS - kTile) + 8 * g4 + 4 * h);
#pragma unroll
          for (int j = 0; j < 4; ++j) sv[4 * g4 + j] = v[j];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int t = min(t0 + 8 * (e >> 2) + 4 * h + (e & 3), B - 1);
          sv[e] = a.S[(int64_t)t * a.ldS + o_c];
        }
      }
    }
  };
  floatx16 snx;
  if constexpr (SLOAD) load_s(t_begin, snx);
  auto consume = [&](int hf, int k, int t0) {
    const E* T = &L.Ts[hf][k * kTile * PT];
    const int64_t* sidk = &L.sid[hf][k * kTile];
    // S^T tile: C[t][o] = str[t] . own[o]; A = streamed rows (lane c: row t0 + c)
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if constexpr (SLOAD) {
      acc = snx;
      load_s(t0 + kTile, snx);
    } else if constexpr (F32) {
      // one chain: the f32 MFMA's dependent latency equals its issue interval (64 cycles)
#pragma unroll
      for (int s4 = 0; s4 < D / 8; ++s4) {
        const floatx4 a4 = *reinterpret_cast<const floatx4*>(&T[c * PT + h * (D / 2) + 4 * s4]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[j], obf[4 * s4 + j], acc, 0, 0, 0);
      }
    } else {
      // two accumulator chains (even / odd k-steps) halve the dependent-MFMA latency
      floatx16 acc1 = acc;
#pragma unroll
      for (int s = 0; s < KS; s += 2) {
        const bf16x8 af0 = *reinterpret_cast<const bf16x8*>(&T[c * PT + 16 * s + 8 * h]);
        const bf16x8 af1 = *reinterpret_cast<const bf16x8*>(&T[c * PT + 16 * s + 16 + 8 * h]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af0, ob[s], acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af1, ob[s + 1], acc1, 0, 0, 0);
      }
      acc += acc1;
    }
    // element e of this lane: streamed row t = t0 + 8(e>>2) + 4h + (e&3), owned column o.
    // The tile's ids are read up front as vectors and the masks are selects: a per-element
    // `if (ids && ...) sid[...]` became a divergent branch with its own LDS round trip.
    // Exponentials run in the log2 domain (one v_exp_f32, the 1/T and log2(e) scales folded
    // into one multiply). The diagonal (t == o: never masked, the label logit) and the rows past
    // B sit in a few tiles only: tiles are aligned with the owned 32-row blocks, so the diagonal
    // lies in the tile with t0 == o_base, and the rows past B in the last tile -- a wave-uniform
    // test sends those tiles through the exact per-element path and all others skip it (the
    // epilogue was ~12 VALU operations per element against 1/2 MFMA).
    bool coll[16];
    {
      const bool have_ids = a.ids != nullptr;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
        const i64x2* sp = reinterpret_cast<const i64x2*>(&sidk[8 * g4 + 4 * h]);
        const i64x2 s01 = sp[0], s23 = sp[1];
        const int64_t sv[4] = {s01[0], s01[1], s23[0], s23[1]};
#pragma unroll
        for (int j = 0; j < 4; ++j) coll[4 * g4 + j] = have_ids & (sv[j] == id_o);
      }
    }
    const bool rare = (t0 == o_base) | (t0 + kTile > B) | !wave_ok;  // wave-uniform
    if constexpr (MODE == 0) {
      if constexpr (F32) {
        if (o_ok && a.S) {  // S is stored only when a backward will read it
          float* sp = a.S + (int64_t)o * a.ldS + t0 + 4 * h;
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4)
            *reinterpret_cast<floatx4*>(sp + 8 * g4) = floatx4{acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]};
        }
      }
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = coll[e] ? kMasked : acc[e] * sc2;
      if (rare) {
        asm volatile("" ::: "memory");  // keep the branch: if-converted, every tile paid for it
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int t = t0 + 8 * (e >> 2) + 4 * h + (e & 3);
          if (t == o) {
            v[e] = acc[e] * sc2;
            dg = acc[e] * a.invT;
            has_dg = true;
          }
          if (t >= B) v[e] = -INFINITY;
        }
      }
      float tm = fmaxf(fmaxf(v[0], v[1]), v[2]);
#pragma unroll
      for (int e = 3; e < 16; e += 2) tm = fmaxf(fmaxf(tm, v[e]), e + 1 < 16 ? v[e + 1] : v[e]);
      const float nm = fmaxf(run_m, tm);
      if (nm != -INFINITY) {  // a lane may see only padding rows (t >= B) so far
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) ss += fast_exp2(v[e] - nm);
        run_s = (run_m == -INFINITY ? 0.f : run_s * fast_exp2(run_m - nm)) + ss;
        run_m = nm;
      }
    } else {
      float lt[16];
      if constexpr (MODE == 2) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const floatx4 l4 = *reinterpret_cast<const floatx4*>(&L.slse[hf][k * kTile + 8 * g4 + 4 * h]);
#pragma unroll
          for (int j = 0; j < 4; ++j) lt[4 * g4 + j] = l4[j];
        }
      }
      float dv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float l2 = MODE == 1 ? lse2_o : lt[e];  // log2-domain log-sum-exp
        const float p = coll[e] ? 0.f : fast_exp2(acc[e] * sc2 - l2);  // collision: logit -1e9, P = 0
        dv[e] = g * p;
      }
      if (rare) {
        asm volatile("" ::: "memory");  // keep the branch (see MODE 0)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int t = t0 + 8 * (e >> 2) + 4 * h + (e & 3);
          const float l2 = MODE == 1 ? lse2_o : lt[e];
          // the label's -1 is NOT part of the bf16 operand: g (p_oo - 1) sits just below -g,
          // where every row rounds the same way (a systematic -0.06 % on dU / dI at B = 1024);
          // ce_reduce adds -g * (the other operand's row o) in fp32 instead
          if (t == o) dv[e] = g * fast_exp2(acc[e] * sc2 - l2);
          if (t >= B || !o_ok) dv[e] = 0.f;
        }
      }
      if constexpr (F32) {
        // grad^T[d][o] += sum_t str^T[d][t] dS^T[t][o], k-step s pairing tile rows
        // 8(s>>2) + (s&3) (half 0) and that + 4 (half 1): B = this lane's dv[s] as it stands,
        // A = the staged row's column 32 db + c
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int tr = 8 * (s >> 2) + 4 * h + (s & 3);
#pragma unroll
          for (int db = 0; db < DB; ++db)
            gacc[db] = __builtin_amdgcn_mfma_f32_32x32x2f32(T[tr * PT + 32 * db + c], dv[s], gacc[db], 0, 0, 0);
        }
      } else {
        // dS^T tile -> bf16 operand fragments (k-step 0: registers 0..7, k-step 1: 8..15)
        bf16x8 xf[2];
#pragma unroll
        for (int e = 0; e < 16; ++e) xf[e >> 3][e & 7] = (__bf16)dv[e];
        // grad^T[d][o] += sum_t str^T[d][t] dS^T[t][o]: A = transposed streamed tile,
        // element j of lane half h <-> tile row 16 kstep + 8 (j>>2) + 4 h + (j&3)
        const int g16 = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int r0 = 16 * k + 4 * (g16 >> 1) + lq;
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            const __bf16* p = &T[r0 * PT + 32 * db + 16 * (g16 & 1) + 4 * lp];
            const bf16x8 af = tr_frag(p, p + 8 * PT);
            gacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, xf[k], gacc[db], 0, 0, 0);
          }
        }
      }
    }
  };

  const int ntiles = t_begin < t_end ? (t_end - t_begin + kTile - 1) / kTile : 0;
  const int nb = (ntiles + BT - 1) / BT;
  if (ntiles > 0) {
    load_batch(t_begin);
    store_batch(0);
    if (nb > 1) load_batch(t_begin + BR);
  }
  __syncthreads();
  // batch b sits in half b & 1; batch b + 1's loads fly while it is consumed
  for (int b = 0; b < nb; ++b) {
    const int hf = b & 1;
    const int t0 = t_begin + b * BR;
    const int nt = min(BT, ntiles - b * BT);
#pragma unroll 1
    for (int k = 0; k < nt; ++k) consume(hf, k, t0 + k * kTile);
    if (b + 1 < nb) {
      store_batch(hf ^ 1);
      if (b + 2 < nb) load_batch(t0 + 2 * BR);
      __syncthreads();
    }
  }
  if constexpr (MODE == 0) {
    if (has_dg && o_ok) a.diag[o] = dg;
  }
  if constexpr (MODE == 0) {
    // merge the two lane halves (same owned row, different streamed rows)
    const float om = __shfl_xor(run_m, 32, 64), os = __shfl_xor(run_s, 32, 64);
    const float nm = fmaxf(run_m, om);
    const float ns = (nm == -INFINITY) ? 0.f
                                       : (run_m == -INFINITY ? 0.f : run_s * fast_exp2(run_m - nm)) +
                                             (om == -INFINITY ? 0.f : os * fast_exp2(om - nm));
    if (h == 0 && o_ok) {
      a.part_m[(int64_t)split * B + o] = nm * kLn2;  // back to natural units for ce_finish
      a.part_s[(int64_t)split * B + o] = ns;
    }
  } else {
    // gacc[db] element e: d = 32 db + 8(e>>2) + 4h + (e&3), owned row o = lane column
    if (o_ok) {
      float* out = a.part_d + ((int64_t)split * B + o) * D;
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const floatx4 v = {gacc[db][4 * e4], gacc[db][4 * e4 + 1], gacc[db][4 * e4 + 2], gacc[db][4 * e4 + 3]};
          *reinterpret_cast<floatx4*>(out + 32 * db + 8 * e4 + 4 * h) = v;
        }
    }
  }
}

template <int D, int MODE, bool F32>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(2))) void ce_tile_kernel(CeArgs a) {
  __shared__ __attribute__((aligned(16))) CeLds<D, F32> lds;
  ce_tile_body<D, MODE, F32>(a, blockIdx.y, lds);
}

// dU and dI in one launch (blockIdx.z): the two halves are independent given lse, and 1,024
// workgroups hide each other's tile latencies better than two back-to-back 512-workgroup grids
template <int D, bool F32, bool SB = false>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(2))) void ce_bwd_pair_kernel(CeArgs aU, CeArgs aI) {
  __shared__ __attribute__((aligned(16))) CeLds<D, F32> lds;  // one image shared by both halves
  if (blockIdx.z == 0) ce_tile_body<D, 1, F32, SB>(aU, blockIdx.y, lds);
  else ce_tile_body<D, 2, F32, SB>(aI, blockIdx.y, lds);
}

// the bf16 backward's streamed operands: U and I rounded to bf16 once (n elements each)
__global__ __launch_bounds__(256) void ce_round_bf16_kernel(const float* __restrict__ U, const float* __restrict__ I,
                                                            int64_t n, __bf16* __restrict__ Ub, __bf16* __restrict__ Ib) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
  if (i >= 2 * n) return;
  const bool second = i >= n;
  const float* src = second ? I + (i - n) : U + i;
  __bf16* dst = second ? Ib + (i - n) : Ub + i;
  const floatx4 v = *reinterpret_cast<const floatx4*>(src);
  bf16x4 h;
  h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
  *reinterpret_cast<bf16x4*>(dst) = h;
}

// per user row: merge the split statistics with the hard-negative logits -> lse, row loss
__device__ __forceinline__ void ce_finish_row(const float* __restrict__ part_m, const float* __restrict__ part_s,
                                              const float* __restrict__ diag, int NS, const float* __restrict__ U,
                                              const float* __restrict__ Hn, int64_t hs_row, int64_t hs_slot, int B,
                                              int N, int D, float invT, float* __restrict__ lse,
                                              float* __restrict__ row_loss, int i, int lane);

__global__ __launch_bounds__(256) void ce_finish_fwd_kernel(const float* __restrict__ part_m,
                                                            const float* __restrict__ part_s,
                                                            const float* __restrict__ diag, int NS,
                                                            const float* __restrict__ U,
                                                            const float* __restrict__ Hn,
                                                            int64_t hs_row, int64_t hs_slot, int B,
                                                            int N, int D, float invT,
                                                            float* __restrict__ lse,
                                                            float* __restrict__ row_loss,
                                                            const float* __restrict__ I,
                                                            __bf16* __restrict__ outb) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + wave;
  if (i < B) ce_finish_row(part_m, part_s, diag, NS, U, Hn, hs_row, hs_slot, B, N, D, invT, lse, row_loss, i,
                           lane);
  // rows i of U and I rounded to bf16 for the backward's streamed operands (outb: [2][B][D]; D even) -- the
  // backward's rounding launch folded into this short one
  if (outb && i < B)
    for (int c = 2 * lane; c < D; c += 128) {
      const float2 u = *reinterpret_cast<const float2*>(U + (int64_t)i * D + c);
      const float2 v = *reinterpret_cast<const float2*>(I + (int64_t)i * D + c);
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<bf16x2*>(outb + (int64_t)i * D + c) = bf16x2{(__bf16)u.x, (__bf16)u.y};
      *reinterpret_cast<bf16x2*>(outb + ((int64_t)B + i) * D + c) = bf16x2{(__bf16)v.x, (__bf16)v.y};
    }
}

__device__ __forceinline__ void ce_finish_row(const float* __restrict__ part_m, const float* __restrict__ part_s,
                                              const float* __restrict__ diag, int NS, const float* __restrict__ U,
                                              const float* __restrict__ Hn, int64_t hs_row, int64_t hs_slot, int B,
                                              int N, int D, float invT, float* __restrict__ lse,
                                              float* __restrict__ row_loss, int i, int lane) {
  float hl = -INFINITY;  // lane n < N: hard-negative logit n
  for (int n = 0; n < N; ++n) {
    const float* hp = Hn + (int64_t)i * hs_row + (int64_t)n * hs_slot;
    float sacc = 0.f;
    for (int cc = lane; cc < D; cc += 64) sacc += U[(int64_t)i * D + cc] * hp[cc];
    sacc = wave_sum(sacc) * invT;
    if (lane == n) hl = sacc;
  }
  float m = lane < NS ? part_m[(int64_t)lane * B + i] : -INFINITY;
  m = fmaxf(m, hl);
  m = wave_max(m);
  float s = 0.f;
  if (lane < NS) s += part_s[(int64_t)lane * B + i] * __expf(part_m[(int64_t)lane * B + i] - m);
  if (lane < N) s += __expf(hl - m);
  s = wave_sum(s);
  if (lane == 0) {
    const float l = m + logf(s);
    lse[i] = l;
    row_loss[i] = l - diag[i];
  }
}

// hard-negative logit gradients dhl[i, n] = g * exp(l_in - lse_i) (the in-batch part is fused)
__global__ __launch_bounds__(256) void ce_hard_bwd_kernel(const float* __restrict__ U,
                                                          const float* __restrict__ Hn,
                                                          int64_t hs_row, int64_t hs_slot, int B,
                                                          int N, int D, float invT,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ grad_out,
                                                          float* __restrict__ dhl) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + wave;
  if (i >= B) return;
  const float g = (grad_out ? *grad_out : 1.f) / (float)B * invT;
  for (int n = 0; n < N; ++n) {
    const float* hp = Hn + (int64_t)i * hs_row + (int64_t)n * hs_slot;
    float sacc = 0.f;
    for (int cc = lane; cc < D; cc += 64) sacc += U[(int64_t)i * D + cc] * hp[cc];
    sacc = wave_sum(sacc) * invT;
    if (lane == 0) dhl[(int64_t)i * N + n] = g * __expf(sacc - lse[i]);
  }
}

// out[r][d] = sum over splits (fixed order) of part[s][r][d] - g * lab[r][d]; two outputs in one
// launch (out2 = the sums of part2, the block after part's NS slabs, minus g * lab2), 8 slab loads
// in flight. lab / lab2 (the label term's operand: I for dU, U for dI) may be null (no label term).
__global__ void ce_reduce_kernel(const float* __restrict__ part, int NS, int64_t n,
                                 float* __restrict__ out, float* __restrict__ out2,
                                 const float* __restrict__ lab, const float* __restrict__ lab2,
                                 const float* __restrict__ grad_out, int B, float invT) {
  int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
  if (i >= (out2 ? 2 * n : n)) return;
  float* dst = out;
  if (i >= n) {
    i -= n;
    part += (int64_t)NS * n;
    dst = out2;
    lab = lab2;
  }
  floatx4 lv = {0.f, 0.f, 0.f, 0.f};
  if (lab) lv = *reinterpret_cast<const floatx4*>(lab + i);
  const float g = (grad_out ? *grad_out : 1.f) / (float)B * invT;  // as ce_tile_body's g
  floatx4 acc = *reinterpret_cast<const floatx4*>(part + i);
  int s = 1;
  for (; s + 8 <= NS; s += 8) {
    floatx4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const floatx4*>(part + (int64_t)(s + u) * n + i);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; s < NS; ++s) acc += *reinterpret_cast<const floatx4*>(part + (int64_t)s * n + i);
  *reinterpret_cast<floatx4*>(dst + i) = acc - g * lv;
}

// Column splits. Forward: ~2 workgroups per CU (512 at B = 4096), each wave latency-bound on its
// tile epilogue, so more waves win. Backward: half as many (256 workgroups per direction): every
// split writes a [B, D] fp32 partial that ce_reduce reads back, 8 MB per split at D = 128
// (measured at B = 4096: 16 splits 57 us, 8 splits 46 us, 4 splits 53 us).
int splits_for(int B, bool bwd) {
  const int blocks = cdiv(B, kOwnW * kWaves);
  int ns = cdiv(bwd ? 256 : 512, blocks);
  if (const char* e = getenv("RSYS_CE_SPLITS")) ns = atoi(e) > 0 ? atoi(e) : ns;  // tuning only
  const int max_ns = cdiv(B, kTile);
  if (ns > max_ns) ns = max_ns;
  if (ns > 64) ns = 64;  // ce_finish reads the partials with one lane each
  return ns < 1 ? 1 : ns;
}

template <int MODE, bool F32>
int launch_tiles(const CeArgs& a, int D, int NS, hipStream_t st) {
  const dim3 grid(cdiv(a.B, kOwnW * kWaves), NS);
  if (D == 128) ce_tile_kernel<128, MODE, F32><<<grid, 64 * kWaves, 0, st>>>(a);
  else ce_tile_kernel<64, MODE, F32><<<grid, 64 * kWaves, 0, st>>>(a);
  return 0;
}

}  // namespace
}  // namespace rs

using namespace rs;

// row pitch of the fp32 mode's stored S: whole 32-column tiles (the tiles past B stay in the row)
extern "C" int64_t rs_inbatch_ce_s_ld(int B) { return (int64_t)cdiv(B, kTile) * kTile; }

extern "C" int64_t rs_inbatch_ce_fused_ws_bytes(int B, int D) {
  const int64_t fwd = (int64_t)splits_for(B, false) * B * 2 + B;
  // dU and dI partials side by side, then the bf16 copies of U and I (B * D floats hold both)
  const int64_t bwd = (int64_t)2 * splits_for(B, true) * B * D + (int64_t)B * D + 8;
  return (fwd > bwd ? fwd : bwd) * (int64_t)sizeof(float);
}

namespace {

template <bool F32>
int ce_fused_fwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride, int64_t h_slot_stride,
                 const int64_t* item_ids, int64_t id_stride, int B, int N, int D, float T, float* lse,
                 float* row_loss, float* loss, float* S, float* ws, __bf16* uib, void* stream) {
  const char* fn = F32 ? "rs_inbatch_ce_fused_f32_fwd" : "rs_inbatch_ce_fused_fwd";
  RS_CHECK_ARG(!uib || aligned16(uib), "%s: ui_bf16 must be 16-byte aligned", fn);
  RS_CHECK_ARG(U && I && lse && row_loss && loss && ws, "%s: null pointer", fn);  // S: optional
  RS_CHECK_ARG(B >= 1 && (D == 64 || D == 128) && N >= 0 && N <= 64,
               "%s: needs D in {64, 128}, N <= 64 (B=%d N=%d D=%d)", fn, B, N, D);
  RS_CHECK_ARG(N == 0 || Hn, "%s: hard negatives need H", fn);
  RS_CHECK_ARG(aligned16(U) && aligned16(I), "%s: U, I must be 16-byte aligned", fn);
  hipStream_t st = as_stream(stream);
  const int NS = splits_for(B, false);
  CeArgs a{};
  a.own = U; a.str = I; a.B = B; a.invT = 1.f / T; a.ids = item_ids; a.id_stride = id_stride;
  a.S = S; a.ldS = (int)rs_inbatch_ce_s_ld(B);
  a.split_rows = cdiv(cdiv(B, NS), kTile) * kTile;
  a.part_m = ws; a.part_s = ws + (int64_t)NS * B; a.diag = ws + (int64_t)2 * NS * B;
  // the mean over the rows: rs_sum's own launch (round 5 measured the finish kernel's last-arriver
  // sum slower: 1,024 workgroups' tickets on one counter, 5 -> 19.5 us)
  const int NSr = cdiv(B, a.split_rows);
  launch_tiles<0, F32>(a, D, NSr, st);
  RS_CHECK_LAUNCH(F32 ? "rs_inbatch_ce_fused_f32_fwd tiles" : "rs_inbatch_ce_fused_fwd tiles");
  const HStrideArgs hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
  ce_finish_fwd_kernel<<<cdiv(B, 4), 256, 0, st>>>(a.part_m, a.part_s, a.diag, NSr, U, Hn, hs.row, hs.slot, B,
                                                   N, D, a.invT, lse, row_loss, I, F32 ? nullptr : uib);
  RS_CHECK_LAUNCH(F32 ? "rs_inbatch_ce_fused_f32_fwd finish" : "rs_inbatch_ce_fused_fwd finish");
  return rs_sum(row_loss, B, 1.f / (float)B, loss, stream);
}

template <bool F32>
int ce_fused_bwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride, int64_t h_slot_stride,
                 const int64_t* item_ids, int64_t id_stride, int B, int N, int D, float T, const float* lse,
                 const float* grad_out, float* dU, float* dI, float* dhl, const float* S, float* ws,
                 const __bf16* uib, void* stream) {
  const char* fn = F32 ? "rs_inbatch_ce_fused_f32_bwd" : "rs_inbatch_ce_fused_bwd";
  RS_CHECK_ARG(U && I && lse && dU && dI && ws && (!F32 || S), "%s: null pointer", fn);
  RS_CHECK_ARG(B >= 1 && (D == 64 || D == 128) && N >= 0 && N <= 64, "%s: bad shape", fn);
  RS_CHECK_ARG(N == 0 || (Hn && dhl), "%s: hard negatives need H, dhl", fn);
  RS_CHECK_ARG(aligned16(U) && aligned16(I) && aligned16(dU) && aligned16(dI),
               "%s: operands must be 16-byte aligned", fn);
  hipStream_t st = as_stream(stream);
  const int NS = splits_for(B, true);
  CeArgs a{};
  a.B = B; a.invT = 1.f / T; a.ids = item_ids; a.id_stride = id_stride; a.lse = lse; a.grad_out = grad_out;
  a.S = const_cast<float*>(S); a.ldS = (int)rs_inbatch_ce_s_ld(B);
  a.split_rows = cdiv(cdiv(B, NS), kTile) * kTile;
  a.part_d = ws;
  const int NSr = cdiv(B, a.split_rows);
  const int64_t n = (int64_t)B * D;
  // dU: users owned, items streamed; dI: items owned, users streamed -- one launch
  CeArgs aU = a, aI = a;
  aU.own = U; aU.str = I;
  aI.own = I; aI.str = U;
  aI.part_d = ws + (int64_t)NSr * n;
  const dim3 grid(cdiv(B, kOwnW * kWaves), NSr, 2);
  if constexpr (!F32) {
    // bf16: U and I rounded once (one small launch), so every workgroup streams half the bytes
    // and stages twice the tiles per batch with the same registers
    {
      // the forward's copies when it wrote them (rs_inbatch_ce_fused_fwd_uib), else one launch here
      const __bf16* Ub = uib;
      if (!uib) {
        __bf16* wb = reinterpret_cast<__bf16*>(ws + (int64_t)2 * NSr * n);
        ce_round_bf16_kernel<<<(int)cdiv(2 * n / 4, 256), 256, 0, st>>>(U, I, n, wb, wb + n);
        RS_CHECK_LAUNCH("rs_inbatch_ce_fused_bwd round");
        Ub = wb;
      }
      const __bf16* Ib = Ub + n;
      aU.strb = Ib;
      aI.strb = Ub;
      if (D == 128) ce_bwd_pair_kernel<128, false, true><<<grid, 64 * kWaves, 0, st>>>(aU, aI);
      else ce_bwd_pair_kernel<64, false, true><<<grid, 64 * kWaves, 0, st>>>(aU, aI);
      RS_CHECK_LAUNCH("rs_inbatch_ce_fused_bwd tiles");
      ce_reduce_kernel<<<(int)cdiv(2 * n / 4, 256), 256, 0, st>>>(ws, NSr, n, dU, dI, I, U, grad_out, B, a.invT);
      RS_CHECK_LAUNCH("rs_inbatch_ce_fused_bwd reduce");
      if (N) {
        const HStrideArgs hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
        ce_hard_bwd_kernel<<<cdiv(B, 4), 256, 0, st>>>(U, Hn, hs.row, hs.slot, B, N, D, a.invT, lse, grad_out, dhl);
        RS_CHECK_LAUNCH("rs_inbatch_ce_fused_bwd hard");
      }
      return 0;
    }
  } else {  // fp32: the fp32 rows streamed as they are
    if (D == 128) ce_bwd_pair_kernel<128, true><<<grid, 64 * kWaves, 0, st>>>(aU, aI);
    else ce_bwd_pair_kernel<64, true><<<grid, 64 * kWaves, 0, st>>>(aU, aI);
    RS_CHECK_LAUNCH("rs_inbatch_ce_fused_f32_bwd tiles");
    ce_reduce_kernel<<<(int)cdiv(2 * n / 4, 256), 256, 0, st>>>(ws, NSr, n, dU, dI, I, U, grad_out, B, a.invT);
    RS_CHECK_LAUNCH("rs_inbatch_ce_fused_f32_bwd reduce");
    if (N) {
      const HStrideArgs hs{h_row_stride > 0 ? h_row_stride : (int64_t)N * D, h_slot_stride > 0 ? h_slot_stride : D};
      ce_hard_bwd_kernel<<<cdiv(B, 4), 256, 0, st>>>(U, Hn, hs.row, hs.slot, B, N, D, a.invT, lse, grad_out, dhl);
      RS_CHECK_LAUNCH("rs_inbatch_ce_fused_f32_bwd hard");
    }
    return 0;
  }
}

}  // namespace

extern "C" int rs_inbatch_ce_fused_fwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                       int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                       int N, int D, float T, float* lse, float* row_loss, float* loss, float* ws,
                                       void* stream) {
  return ce_fused_fwd<false>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, row_loss,
                             loss, nullptr, ws, nullptr, stream);
}

// the same, also writing U and I as rounded to bf16 ([2][B][D], U then I) for
// rs_inbatch_ce_fused_bwd_uib: the backward's rounding launch folded into the forward's finish
extern "C" int rs_inbatch_ce_fused_fwd_uib(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                           int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                           int N, int D, float T, float* lse, float* row_loss, float* loss, float* ws,
                                           void* ui_bf16, void* stream) {
  RS_CHECK_ARG(ui_bf16, "rs_inbatch_ce_fused_fwd_uib: null ui_bf16");
  return ce_fused_fwd<false>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, row_loss,
                             loss, nullptr, ws, static_cast<__bf16*>(ui_bf16), stream);
}

extern "C" int rs_inbatch_ce_fused_f32_fwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                           int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                           int N, int D, float T, float* lse, float* row_loss, float* loss, float* S,
                                           float* ws, void* stream) {
  return ce_fused_fwd<true>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, row_loss,
                            loss, S, ws, nullptr, stream);
}

extern "C" int rs_inbatch_ce_fused_bwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                       int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                       int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                                       float* dI, float* dhl, float* ws, void* stream) {
  return ce_fused_bwd<false>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, grad_out,
                             dU, dI, dhl, nullptr, ws, nullptr, stream);
}

// ui_bf16: the forward's rounded copies (rs_inbatch_ce_fused_fwd_uib on the same U, I)
extern "C" int rs_inbatch_ce_fused_bwd_uib(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                           int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                           int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                                           float* dI, float* dhl, float* ws, const void* ui_bf16, void* stream) {
  RS_CHECK_ARG(ui_bf16 && aligned16(ui_bf16), "rs_inbatch_ce_fused_bwd_uib: ui_bf16 null or not 16-byte aligned");
  return ce_fused_bwd<false>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, grad_out,
                             dU, dI, dhl, nullptr, ws, static_cast<const __bf16*>(ui_bf16), stream);
}

extern "C" int rs_inbatch_ce_fused_f32_bwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                           int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                           int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                                           float* dI, float* dhl, const float* S, float* ws, void* stream) {
  return ce_fused_bwd<true>(U, I, Hn, h_row_stride, h_slot_stride, item_ids, id_stride, B, N, D, T, lse, grad_out,
                            dU, dI, dhl, S, ws, nullptr, stream);
}
