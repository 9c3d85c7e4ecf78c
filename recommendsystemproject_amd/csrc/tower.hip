// DSSM tower chain in training mode: GenericTower.feature_bn followed by MLP_Tower
// (GenericTower.py:229-236; Tower.py:16-41): BatchNorm1d -> [Linear -> BatchNorm1d -> ReLU ->
// Dropout] x n -> Linear -> F.normalize, at the batch sizes the towers run at (B = 4096 rows:
// every tensor of the chain is a few MB, so the chain is bound by the number of dependent
// phases, not by bytes or flops).
//
// One kernel per Linear. A BatchNorm needs whole-batch column statistics, so it is split
// across the two kernels around it:
//   * the PRODUCING GEMM's epilogue writes per-row-tile column statistics of its output z
//     (tile mean and M2 = sum (z - tile mean)^2, fp32) with write-through (sc1) stores and takes
//     a ticket; the workgroup that arrives last for its (group, column block) merges the tiles in
//     a fixed order (Chan's update, fp64) and publishes mean / rstd -- and, once every group of
//     the column block is in (a second ticket), updates the running statistics in group order.
//     The hand-off is the fence-free form of MI355X_MICROARCH.md (sc1 stores, every storing wave
//     drained, one agent-scope add per workgroup after a barrier, sc1 loads by the last adder).
//   * the CONSUMING GEMM's prologue loads mean / rstd / gamma / beta of its input columns and
//     applies BN (+ ReLU + dropout) to the A operand while staging it into LDS: the normalised
//     activation never makes a separate HBM round trip (n-block 0 writes it once, as the
//     weight-gradient operand).
// The final Linear's workgroups own whole rows, so F.normalize is its epilogue.
//
// Backward mirrors it: the dgrad GEMM of layer j computes dz_j = BN_j backward in its prologue
// from the incoming gradient and the means of g and g*xhat its predecessor published, and
// its epilogue applies the ReLU/dropout mask of the BatchNorm below (recomputed from the saved
// pre-BN z and statistics, bitwise the forward's decision) and hands that BatchNorm's tile
// sums (sum g, sum g*xhat) to its last arriver, which publishes the means and accumulates
// dgamma / dbeta. The l2-normalise backward is the last layer's prologue (row-local). feature_bn's dx is
// the same prologue with no GEMM behind it (N = 0).
//
// Products: fp32 mode on v_mfma_f32_16x16x4_f32 (exact fp32 products), bf16 mode on
// v_mfma_f32_16x16x32_bf16 (operands rounded as they are staged); accumulation, statistics,
// epilogues and every stored tensor stay fp32. Statistics are reduced in fixed orders only (no
// atomics): identical inputs give identical bits.
#include "common.h"
#include "rng.h"

namespace rs {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4t __attribute__((ext_vector_type(4)));

constexpr int KC = 32;     // k chunk per LDS stage
constexpr int KMAX = 512;  // widest layer input held in the LDS column tables
constexpr int TM_STATS = 128;
constexpr int MB = 16;  // tile values loaded per batch by a finishing workgroup

enum : int { PRO_BN = 1, PRO_L2B = 2, PRO_BNB = 3 };
enum : int { EPI_NONE = 0, EPI_STATS = 1, EPI_L2 = 2, EPI_BWD = 3 };

// statistics hand-off of one BatchNorm from its producing kernel (see the file comment)
struct Fin {
  float* part;      // [G][tiles][2][N] tile values, sc1 stores / loads
  int* cnt;         // [G * nb] first-level tickets, then [nb] second-level; zero on entry and exit
  double* scratch;  // [G][2][N] per-group results for the cross-group step (sc1)
  float* o0;        // forward: mean [G][N]; backward: mean(g) [G][N]
  float* o1;        // forward: rstd [G][N]; backward: mean(g * xhat) [G][N]
  float* run_mean;  // forward: running statistics (may be NULL), momentum, eps, num_batches
  float* run_var;
  int64_t* nbt;
  float momentum, eps;
  float* dgamma;    // backward: += sum g * xhat, += sum g (over every group)
  float* dbeta;
  int bwd, nb;      // nb: column blocks of 64 of this kernel
};

struct TwArgs {
  // C[G*Bg, N] = pro(A)[G*Bg, K] * op(W); W is [N][K] (wt = 0: forward Linear) or [K][N]
  // (wt = 1: input gradient through a Linear)
  const float* A;
  const float* A2;  // PRO_BNB: the pre-BN z (xhat); PRO_L2B: the normalised output y
  const float* W;
  const float* bias;
  int N, K, G, Bg, tiles;  // tiles: row tiles per group of THIS kernel
  int wt;
  int nbx;  // n-blocks of the grid
  // prologue: published statistics of the input BatchNorm [G][K] and its affine [K]
  const float* in_mean;
  const float* in_rstd;
  const float* in_w;
  const float* in_b;
  const float* in_mg;   // PRO_BNB
  const float* in_mgx;
  int relu;
  float drop_p;
  const int64_t* key;
  int site;
  const float* rownorm;  // PRO_L2B
  float l2eps;
  float* h_out;  // pro(A) written by n-block 0 (fp32)
  // epilogue
  float* C;
  float* norm_out;  // EPI_L2
  const float* eZ;  // EPI_BWD: pre-BN z of the BatchNorm below, its statistics and affine
  const float* e_mean;
  const float* e_rstd;
  const float* e_w;
  const float* e_b;
  int e_relu;
  float e_drop_p;
  const int64_t* e_key;
  int e_site;
  Fin fin;  // EPI_STATS / EPI_BWD
  unsigned long long* dbg;  // profiling only: per-workgroup phase timestamps (rs_tower_debug_buffer)
};

template <typename T>
struct OpT;
template <>
struct OpT<float> {
  static constexpr int PITCH = KC + 4;  // 144-byte rows: conflict-free b128 reads
};
template <>
struct OpT<__bf16> {
  static constexpr int PITCH = KC + 8;  // 80-byte rows: conflict-free b128 reads
};

template <typename T>
__device__ __forceinline__ void lds_put4(T* dst, const f4& v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<f4*>(dst) = v;
  } else {
    bf16x4t h;
    h[0] = (__bf16)v[0]; h[1] = (__bf16)v[1]; h[2] = (__bf16)v[2]; h[3] = (__bf16)v[3];
    *reinterpret_cast<bf16x4t*>(dst) = h;
  }
}

__device__ __forceinline__ int tile_rows(int tm, int Bg, int t) { return min(tm, Bg - t * tm); }

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() carries a workgroup release fence,
// which on gfx950 waits for every outstanding global store (and, with stores and loads mixed,
// every load) before the barrier; this waits for the LDS operations alone.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One ticket per workgroup: every thread's sc1 stores drained, the workgroup's barrier, one
// agent-scope add; returns true (uniformly) in the workgroup whose add came last.
__device__ __forceinline__ bool ticket(int* cnt, int last) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == last;
  }
  __syncthreads();
  return s_last != 0;
}

// The producer side of a BatchNorm hand-off. Threads tid < ncols hold this tile's values of
// columns n0 + tid: forward (tile mean, tile M2) over the tile's rows, backward (sum g, sum
// g*xhat). fin_publish stores them (sc1) and takes the ticket of (g, column block nb); it returns
// true in the workgroup that arrived last, which then calls fin_merge: merge the group's tiles in
// a fixed order (4 tile lanes per column, contiguous tile ranges, Chan's update in fp64, lanes
// combined in order), publish the group's results, and -- in the last of those (second ticket)
// -- do the cross-group step. Callers issue no other global store before these: the ticket's
// vmcnt(0) would wait for it.
__device__ __forceinline__ bool fin_publish(const Fin& f, int N, int tiles, int g, int tile,
                                            int nb, int ncols, float v0, float v1) {
  const int tid = threadIdx.x;
  if (tid < ncols) {
    float* pp = f.part + (size_t)(g * tiles + tile) * 2 * N + nb * 64 + tid;
    st_sc1(pp, v0);
    st_sc1(pp + N, v1);
  }
  return ticket(f.cnt + g * f.nb + nb, tiles - 1);
}

// What the last arriver read-modify-writes at the very end (the running statistics, or dgamma /
// dbeta, of column n0 + tid; num_batches_tracked), loaded by every workgroup before its ticket so
// that the merge's tail is not one more dependent round trip.
struct FinPre {
  float a = 0.f, b = 0.f;
  int64_t nbt = 0;
};
__device__ __forceinline__ FinPre fin_preload(const Fin& f, int nb, int ncols) {
  FinPre r;
  const int tid = threadIdx.x;
  if (tid < ncols) {
    const int col = nb * 64 + tid;
    if (f.bwd) {
      r.a = f.dgamma[col];
      r.b = f.dbeta[col];
    } else if (f.run_mean) {
      r.a = f.run_mean[col];
      r.b = f.run_var[col];
    }
  }
  if (tid == 0 && !f.bwd && nb == 0 && f.nbt) r.nbt = *f.nbt;
  return r;
}

// The last arriver's first batch of tile values, loaded right after its ticket so that the
// round trip runs under its own output stores (fin_merge consumes them)
struct MergeFirst {
  float av[MB], qv[MB];
};

__device__ __forceinline__ void fin_merge_load(const Fin& f, int N, int tiles, int g, int nb, int ncols,
                                               MergeFirst& mf) {
  const int tid = threadIdx.x;
  const int c = tid & 63, tl = tid >> 6;
  const int R = (tiles + 3) / 4, t_begin = tl * R, t_end = min(tiles, t_begin + R);
  const int cc = nb * 64 + min(c, max(ncols - 1, 0));
  const float* pb = f.part + (size_t)g * tiles * 2 * N + cc;
#pragma unroll
  for (int u = 0; u < MB; ++u) {
    const size_t o = (size_t)max(min(t_begin + u, t_end - 1), 0) * 2 * N;
    mf.av[u] = ld_sc1(pb + o);
    mf.qv[u] = ld_sc1(pb + o + N);
  }
}

template <bool PRE>
__device__ __forceinline__ void fin_merge(const Fin& f, int N, int G, int Bg, int tiles, int tm, int g, int nb,
                                          int ncols, const FinPre& pre, const MergeFirst& first) {
  __shared__ double comb[3][4][64];
  const int tid = threadIdx.x;
  const int n0 = nb * 64;
  // ---- last tile of (g, nb): merge
  const int c = tid & 63, tl = tid >> 6;
  const int R = (tiles + 3) / 4, t_begin = tl * R, t_end = min(tiles, t_begin + R);
  const int cc = n0 + min(c, max(ncols - 1, 0));
  const float* pb = f.part + (size_t)g * tiles * 2 * N + cc;
  double n_a = 0.0, a = 0.0, q = 0.0;  // forward: (n, mean, M2); backward: (-, sum g, sum g xhat)
  for (int t0 = t_begin; t0 < t_end; t0 += MB) {
    float av[MB], qv[MB];
    if (PRE && t0 == t_begin) {
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        av[u] = first.av[u];
        qv[u] = first.qv[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        const size_t o = (size_t)min(t0 + u, t_end - 1) * 2 * N;
        av[u] = ld_sc1(pb + o);
        qv[u] = ld_sc1(pb + o + N);
      }
    }
    if (f.bwd) {
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        if (t0 + u >= t_end) break;
        a += (double)av[u];
        q += (double)qv[u];
      }
    } else {
      // the batch's tiles combined in two passes (weighted mean, then M2 + n_t (mean_t - mean)^2:
      // one fp64 division per batch -- the per-tile Chan update's two divisions per tile were a
      // dependent chain of ~4 us in the last arriver), then merged into (n_a, a, q) by Chan
      double nb = 0.0, sb = 0.0;
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        const double nt = t0 + u < t_end ? (double)min(tm, Bg - (t0 + u) * tm) : 0.0;
        nb += nt;
        sb += nt * (double)av[u];
      }
      const double mb = sb / nb;
      double qb = 0.0;
#pragma unroll
      for (int u = 0; u < MB; ++u) {
        const double nt = t0 + u < t_end ? (double)min(tm, Bg - (t0 + u) * tm) : 0.0;
        const double d = (double)av[u] - mb;
        qb += nt > 0.0 ? (double)qv[u] + nt * d * d : 0.0;
      }
      const double n = n_a + nb, d = mb - a;
      a += d * (nb / n);
      q += qb + d * d * (n_a * nb / n);
      n_a = n;
    }
  }
  comb[0][tl][c] = n_a;
  comb[1][tl][c] = a;
  comb[2][tl][c] = q;
  lds_barrier();
  if (G == 1) {  // one group: publish and do the cross-group step here (no second ticket)
    if (tid < ncols) {
      const int col = n0 + c;
      double n_s = comb[0][0][c], A = comb[1][0][c], Q = comb[2][0][c];
      for (int l = 1; l < 4; ++l) {
        if (f.bwd) {
          A += comb[1][l][c];
          Q += comb[2][l][c];
        } else if (comb[0][l][c] > 0.0) {
          const double nt = comb[0][l][c], n = n_s + nt, d = comb[1][l][c] - A;
          A += d * (nt / n);
          Q += comb[2][l][c] + d * d * (n_s * nt / n);
          n_s = n;
        }
      }
      if (f.bwd) {
        f.o0[col] = (float)(A / (double)Bg);
        f.o1[col] = (float)(Q / (double)Bg);
        f.dgamma[col] = pre.a + (float)Q;
        f.dbeta[col] = pre.b + (float)A;
      } else {
        double var = Q / (double)Bg;
        if (var < 0.0) var = 0.0;
        f.o0[col] = (float)A;
        f.o1[col] = (float)(1.0 / sqrt(var + (double)f.eps));
        if (f.run_mean) {
          const double unb = Bg > 1 ? Q / (double)(Bg - 1) : var;
          f.run_mean[col] = (1.f - f.momentum) * pre.a + f.momentum * (float)A;
          f.run_var[col] = (1.f - f.momentum) * pre.b + f.momentum * (float)unb;
        }
      }
    }
    if (tid == 0) {
      if (!f.bwd && nb == 0 && f.nbt) *f.nbt = pre.nbt + 1;
      __hip_atomic_store(f.cnt + nb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (tid < ncols) {
    double n_s = comb[0][0][c], A = comb[1][0][c], Q = comb[2][0][c];
    for (int l = 1; l < 4; ++l) {
      if (f.bwd) {
        A += comb[1][l][c];
        Q += comb[2][l][c];
      } else if (comb[0][l][c] > 0.0) {
        const double nt = comb[0][l][c], n = n_s + nt, d = comb[1][l][c] - A;
        A += d * (nt / n);
        Q += comb[2][l][c] + d * d * (n_s * nt / n);
        n_s = n;
      }
    }
    const int col = n0 + c;
    double* sc = f.scratch + (size_t)g * 2 * N + col;
    if (f.bwd) {
      f.o0[g * N + col] = (float)(A / (double)Bg);
      f.o1[g * N + col] = (float)(Q / (double)Bg);
      st_sc1(sc, A);
      st_sc1(sc + N, Q);
    } else {
      double var = Q / (double)Bg;
      if (var < 0.0) var = 0.0;
      f.o0[g * N + col] = (float)A;
      f.o1[g * N + col] = (float)(1.0 / sqrt(var + (double)f.eps));
      st_sc1(sc, A);
      st_sc1(sc + N, Bg > 1 ? Q / (double)(Bg - 1) : var);  // unbiased, for running_var
    }
  }
  if (tid == 0) __hip_atomic_store(f.cnt + g * f.nb + nb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int* cnt2 = f.cnt + G * f.nb + nb;
  if (!ticket(cnt2, G - 1)) return;
  // ---- every group of column block nb is in: cross-group step, groups in order
  if (tid < ncols) {
    const int col = n0 + tid;
    // the groups' values GB at a time (one round trip per batch, not per group: G = 11 item
    // groups with 10 hard negatives), consumed in group order
    constexpr int GB = 8;
    if (f.bwd) {
      double tw = 0.0, tb = 0.0;
      for (int g0 = 0; g0 < G; g0 += GB) {
        double vb[GB], vw[GB];
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          const size_t o = (size_t)min(g0 + u, G - 1) * 2 * N + col;
          vb[u] = ld_sc1(f.scratch + o);
          vw[u] = ld_sc1(f.scratch + o + N);
        }
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          if (g0 + u >= G) break;
          tb += vb[u];
          tw += vw[u];
        }
      }
      f.dgamma[col] = pre.a + (float)tw;
      f.dbeta[col] = pre.b + (float)tb;
    } else if (f.run_mean) {
      float rm = pre.a, rv = pre.b;
      for (int g0 = 0; g0 < G; g0 += GB) {
        double vm[GB], vu[GB];
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          const size_t o = (size_t)min(g0 + u, G - 1) * 2 * N + col;
          vm[u] = ld_sc1(f.scratch + o);
          vu[u] = ld_sc1(f.scratch + o + N);
        }
#pragma unroll
        for (int u = 0; u < GB; ++u) {
          if (g0 + u >= G) break;
          rm = (1.f - f.momentum) * rm + f.momentum * (float)vm[u];
          rv = (1.f - f.momentum) * rv + f.momentum * (float)vu[u];
        }
      }
      f.run_mean[col] = rm;
      f.run_var[col] = rv;
    }
  }
  if (tid == 0) {
    if (!f.bwd && nb == 0 && f.nbt) *f.nbt = pre.nbt + G;
    __hip_atomic_store(cnt2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Column tables of the prologue (LDS): one load round trip.
//   PRO_BN : c0 = mean, c1 = rstd * gamma, c2 = beta
//   PRO_BNB: c0 = mean, c1 = rstd, c2 = gamma * rstd, c3 = mean(g), c4 = mean(g * xhat)
template <int PRO>
__device__ void prologue_tables(const TwArgs& p, int g, float* c0, float* c1, float* c2,
                                float* c3, float* c4) {
  const int K = p.K;
  constexpr int U = KMAX / 256;  // columns per thread; loads of all of them issued first
  float v0[U], v1[U], v2[U], v3[U], v4[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = min((int)threadIdx.x + 256 * u, K - 1);
    v0[u] = p.in_mean[g * K + k];
    v1[u] = p.in_rstd[g * K + k];
    v2[u] = p.in_w[k];
    if constexpr (PRO == PRO_BN) {
      v3[u] = p.in_b[k];
    } else {
      v3[u] = p.in_mg[g * K + k];
      v4[u] = p.in_mgx[g * K + k];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = threadIdx.x + 256 * u;
    if (k >= K) break;
    if constexpr (PRO == PRO_BN) {
      c0[k] = v0[u];
      c1[k] = __fmul_rn(v1[u], v2[u]);
      c2[k] = v3[u];
    } else {
      c0[k] = v0[u];
      c1[k] = v1[u];
      c2[k] = v2[u] * v1[u];
      c3[k] = v3[u];
      c4[k] = v4[u];
    }
  }
  (void)c3;
  (void)c4;
  (void)v4;
}

// the prologue transform of 4 consecutive columns k..k+3 of global row m (local row rl)
template <int PRO>
__device__ __forceinline__ f4 pro_apply(const TwArgs& p, f4 a, f4 a2, int m, int rl, int k,
                                        const float* c0, const float* c1, const float* c2,
                                        const float* c3, const float* c4, const float* rdot,
                                        const float* rden, const float* rcl,
                                        const DropKey& dk, bool drop) {
  f4 v;
  if constexpr (PRO == PRO_BN) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaf(a[e] - c0[k + e], c1[k + e], c2[k + e]);
    if (p.relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (drop) {  // element index m*K + k is even (K, k multiples of 4): two pair hashes
      const uint32_t pr = ((uint32_t)m * (uint32_t)p.K + (uint32_t)k) >> 1;
      float mk[4];
      keep_pair32(dk, pr, mk[0], mk[1]);
      keep_pair32(dk, pr + 1, mk[2], mk[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= mk[e];
    }
  } else if constexpr (PRO == PRO_BNB) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (a2[e] - c0[k + e]) * c1[k + e];
      v[e] = c2[k + e] * (a[e] - c3[k + e] - xh * c4[k + e]);
    }
  } else {  // PRO_L2B: d(F.normalize) with the row's dot(y, dy) and max(norm, eps)
    const float dot = rdot[rl], den = rden[rl];
    const bool clamped = rcl[rl] != 0.f;  // norm <= eps: F.normalize divides by eps
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = clamped ? a[e] / den : (a[e] - a2[e] * dot) / den;
  }
  (void)c3;
  (void)c4;
  (void)rdot;
  (void)rden;
  (void)rcl;
  (void)m;
  (void)rl;
  return v;
}

template <typename T, int TM, int TN, int PRO, int EPI, int DCH = 1>
__global__ __launch_bounds__(256) void tower_kernel(TwArgs p) {
  constexpr int PITCH = OpT<T>::PITCH;
  // the 4 waves tile the TM x TN output as WR row groups of 16 rows x WC column groups of TN / WC
  // columns (TM = 64: 4 x 1, 32: 2 x 2, 16: 1 x 4)
  static_assert(TM == 16 || TM == 32 || TM == 64, "row tile");
  constexpr int WR = TM / 16, WC = 4 / WR;
  constexpr int MT = 1;                 // 16-row m tiles per wave
  constexpr int NTL = TN / (16 * WC);   // 16-column n tiles per wave
  constexpr int AR = TM * (KC / 4);     // A float4 slots per chunk
  constexpr int LA = (AR + 255) / 256;  // A float4 loads per thread per chunk
  constexpr int LW = (TN * (KC / 4) + 255) / 256;
  constexpr bool GEMM = EPI != EPI_NONE;
  constexpr bool SUMS = EPI == EPI_STATS || EPI == EPI_BWD;  // column sums + hand-off
  constexpr bool TWO = PRO == PRO_BNB || PRO == PRO_L2B;  // second A-shaped input
  // k chunks of loads in flight per thread: the host picks DCH >= the chunk count where the
  // registers allow it, so every operand load of the workgroup goes out in one round trip
  constexpr int D = DCH;
  constexpr int TP = TN + 1;      // epilogue tile pitch (floats)

  // one LDS buffer: the double-buffered operand stages, reused by the epilogue's column tile
  constexpr int STAGE_BYTES = GEMM ? 2 * (TM + TN) * PITCH * (int)sizeof(T) : 16;
  constexpr int EPI_BYTES = SUMS ? 2 * TM * TP * 4 : 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES];
  typedef T stage_a[GEMM ? TM : 1][PITCH];
  typedef T stage_b[GEMM ? TN : 1][PITCH];
  stage_a* As = reinterpret_cast<stage_a*>(smem);
  stage_b* Bs = reinterpret_cast<stage_b*>(smem + 2 * sizeof(stage_a));
  constexpr int NTAB = PRO == PRO_BNB ? 5 : (PRO == PRO_BN ? 3 : 1);
  constexpr int TABK = PRO == PRO_L2B ? 1 : KMAX;
  __shared__ float tab[NTAB][TABK];
  __shared__ float ctab[4][GEMM ? TN : 1];  // output-column constants: bias | e_mean, e_rstd, e_w, e_b
  __shared__ float rdot[PRO == PRO_L2B ? TM : 1], rden[PRO == PRO_L2B ? TM : 1],
      rcl[PRO == PRO_L2B ? TM : 1];
  __shared__ float red[2][4][GEMM ? TN : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // XCD-aware placement: workgroups are dealt to the 8 XCDs round-robin by linear id, so the
  // n-blocks of one row tile get ids of equal residue mod 8 (one XCD, whose L2 then serves their
  // shared A rows after the first miss); the grid is padded to whole groups of 8 row tiles
  int nblk, rt;
  if constexpr (GEMM) {
    const int L = blockIdx.x, slot = L >> 3;
    nblk = slot % p.nbx;
    rt = (slot / p.nbx) * 8 + (L & 7);
    if (rt >= p.G * p.tiles) return;
  } else {
    nblk = 0;
    rt = blockIdx.y;
  }
  const int g = rt / p.tiles, tile = rt % p.tiles;
  const int nt = tile_rows(TM, p.Bg, tile);  // valid rows of this tile
  const int mbase = g * p.Bg + tile * TM;
  const int n0 = nblk * TN;
  const int K = p.K, N = p.N;
  const bool hwrite = p.h_out && nblk == 0;
  const f4 zero4 = f4{0.f, 0.f, 0.f, 0.f};

  float* c0 = tab[0];
  float* c1 = tab[NTAB > 1 ? 1 : 0];
  float* c2 = tab[NTAB > 2 ? 2 : 0];
  float* c3 = tab[NTAB > 3 ? 3 : 0];
  float* c4 = tab[NTAB > 4 ? 4 : 0];

  DropKey dk{};
  const bool drop = PRO == PRO_BN && p.drop_p > 0.f;
  if (drop) dk = make_key(p.key, p.site, p.drop_p);

#define TW_MARK(i)                                                                  \
  do {                                                                              \
    if (p.dbg && threadIdx.x == 0)                                                  \
      p.dbg[((size_t)rt * p.nbx + nblk) * 8 + (i)] = wall_clock64();                   \
  } while (0)
  TW_MARK(0);

  if constexpr (!GEMM) {
    // N = 0: the transformed A is the output (feature_bn's dx)
    prologue_tables<PRO>(p, g, c0, c1, c2, c3, c4);
    __syncthreads();
    const int k4n = K / 4;
    for (int idx = tid; idx < nt * k4n; idx += 256) {
      const int rl = idx / k4n, k = (idx % k4n) * 4;
      const size_t o = (size_t)(mbase + rl) * K + k;
      const f4 a = *reinterpret_cast<const f4*>(p.A + o);
      f4 a2{};
      if constexpr (TWO) a2 = *reinterpret_cast<const f4*>(p.A2 + o);
      const f4 v = pro_apply<PRO>(p, a, a2, mbase + rl, rl, k, c0, c1, c2, c3, c4, rdot, rden, rcl, dk, drop);
      *reinterpret_cast<f4*>(p.h_out + o) = v;
    }
    return;
  } else {
    static_assert((LA * 256 == AR || (LA == 1 && AR < 256)) && LW * 256 == TN * 8, "tile loads");
    f4 ra[D][LA], ra2[D][LA], rw[D][LW];
    // Loads are unconditional (clamped to a valid address) and the chunk index is clamped, so the
    // pipelined body is straight-line code; out-of-range values are zeroed by selects where the
    // chunk is consumed (a select right after the load would make the load's wait the issuing
    // step's). No global store happens inside the pipeline: with loads and stores mixed the
    // compiler's waitcnt pass drains every load in flight.
    auto load = [&](int kc, f4 (&ra)[LA], f4 (&ra2)[LA], f4 (&rw)[LW]) {
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int idx = tid + 256 * u;
        const int rl = idx >> 3, k = kc * KC + (idx & 7) * 4;
        const size_t o = (size_t)(mbase + min(rl, nt - 1)) * K + min(k, K - 4);
        ra[u] = *reinterpret_cast<const f4*>(p.A + o);
        if constexpr (TWO) ra2[u] = *reinterpret_cast<const f4*>(p.A2 + o);
      }
#pragma unroll
      for (int u = 0; u < LW; ++u) {
        const int idx = tid + 256 * u;
        size_t o;
        if (!p.wt) {
          const int n = n0 + (idx >> 3), k = kc * KC + (idx & 7) * 4;
          o = (size_t)min(n, N - 1) * K + min(k, K - 4);
        } else {
          const int k = kc * KC + idx / (TN / 4), n = n0 + (idx % (TN / 4)) * 4;
          o = (size_t)min(k, K - 1) * N + min(n, N - 4);
        }
        rw[u] = *reinterpret_cast<const f4*>(p.W + o);
      }
    };
    auto store = [&](int kc, int buf, f4 (&ra)[LA], f4 (&ra2)[LA], f4 (&rw)[LW]) {
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int idx = tid + 256 * u;
        const int rl = min(idx >> 3, TM - 1), kl = (idx & 7) * 4, k = kc * KC + kl;
        const bool ok = (AR % 256 == 0 || idx < AR) && rl < nt && k < K;
        const int kt = min(k, K - 4);  // tables are read in range even for padding columns
        f4 v = pro_apply<PRO>(p, ra[u], ra2[u], mbase + rl, rl, kt, c0, c1, c2, c3, c4, rdot, rden, rcl, dk, drop);
        v = ok ? v : zero4;
        // h = pro(A) (the weight gradient's operand, fp32) stored by n-block 0 as it is staged:
        // every load of the workgroup was issued before the loop (D >= the chunk count) or is
        // older than these stores, so no wait for them is needed before the kernel's end
        if (hwrite && ok) *reinterpret_cast<f4*>(p.h_out + (size_t)(mbase + rl) * K + k) = v;
        if (AR % 256 == 0 || idx < AR) lds_put4<T>(&As[buf][rl][kl], v);
      }
#pragma unroll
      for (int u = 0; u < LW; ++u) {
        const int idx = tid + 256 * u;
        if (!p.wt) {
          const int nl = idx >> 3, kl = (idx & 7) * 4;
          const bool ok = n0 + nl < N && kc * KC + kl < K;
          lds_put4<T>(&Bs[buf][nl][kl], ok ? rw[u] : zero4);
        } else {
          const int kl = idx / (TN / 4), nl = (idx % (TN / 4)) * 4;
          const bool ok = kc * KC + kl < K && n0 + nl < N;
          const f4 w = ok ? rw[u] : zero4;
#pragma unroll
          for (int e = 0; e < 4; ++e) Bs[buf][nl + e][kl] = (T)w[e];
        }
      }
    };

    const int nk = (K + KC - 1) / KC;
    // the first D chunks' loads go out before the prologue's: one round trip covers both
#pragma unroll
    for (int st = 0; st < D; ++st) load(min(st, nk - 1), ra[st], ra2[st], rw[st]);

    const int wrow = (wave % WR) * 16, wcol = (wave / WR) * (TN / WC);
    const int r16 = lane & 15, q = lane >> 4;
    // epilogue operands of this tile, issued now and consumed after the loop: the pre-BN z of the
    // BatchNorm below (EPI_BWD), and the output-column constants (LDS)
    f4 ez[MT][NTL];
    if constexpr (EPI == EPI_BWD) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NTL; ++j)
          ez[i][j] = *reinterpret_cast<const f4*>(p.eZ + (size_t)(mbase + min(wrow + 16 * i + r16, nt - 1)) * N +
                                                  min(n0 + wcol + 16 * j + 4 * q, N - 4));
    }
    if (tid < TN) {
      const int n = min(n0 + tid, N - 1);
      if constexpr (EPI == EPI_BWD) {
        ctab[0][tid] = p.e_mean[g * N + n];
        ctab[1][tid] = p.e_rstd[g * N + n];
        ctab[2][tid] = p.e_relu ? p.e_w[n] : 0.f;
        ctab[3][tid] = p.e_relu ? p.e_b[n] : 0.f;
      } else {
        ctab[0][tid] = p.bias[n];
      }
    }
    if constexpr (PRO != PRO_L2B) prologue_tables<PRO>(p, g, c0, c1, c2, c3, c4);
    if constexpr (PRO == PRO_L2B) {
      // row dots over the whole row (K = the output width), TPR adjacent lanes per row
      constexpr int TPR = 256 / TM;
      const int rl = tid / TPR, part = tid % TPR;
      const int rr = min(rl, nt - 1);
      const float* dd = p.A + (size_t)(mbase + rr) * K;
      const float* yy = p.A2 + (size_t)(mbase + rr) * K;
      float sacc = 0.f;
      for (int k = part * 4; k < K; k += TPR * 4) {
        const f4 dv = *reinterpret_cast<const f4*>(dd + k);
        const f4 yv = *reinterpret_cast<const f4*>(yy + k);
        sacc += dv[0] * yv[0] + dv[1] * yv[1] + dv[2] * yv[2] + dv[3] * yv[3];
      }
#pragma unroll
      for (int o = 1; o < TPR; o <<= 1) sacc += __shfl_xor(sacc, o, 64);
      if (part == 0) {
        const float nrm = p.rownorm[mbase + rr];
        rden[rl] = fmaxf(nrm, p.l2eps);
        rdot[rl] = sacc;
        rcl[rl] = nrm > p.l2eps ? 0.f : 1.f;
      }
    }
    __syncthreads();  // no global store has been issued yet: a plain barrier

    f4 acc[MT][NTL];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NTL; ++j) acc[i][j] = zero4;

    TW_MARK(1);
    // D chunks in flight per thread: a chunk's loads are issued D iterations before it is staged
    // the chunk count is padded to a multiple of D (padding chunks stage zeros): no exit inside
    // the unrolled body, so the waitcnt pass sees straight-line code with D chunks in flight
    const int nkp = (nk + D - 1) / D * D;
    // the last group of D chunks issues no further loads (two straight-line bodies, chosen per
    // group by a uniform branch: with D >= the chunk count every load went out before the loop)
    auto group = [&](int kc0, bool more) {
#pragma unroll
      for (int st = 0; st < D; ++st) {
        const int kc = kc0 + st;
        const int buf = kc & 1;
        store(kc, buf, ra[st], ra2[st], rw[st]);
        lds_barrier();
        if (more) load(min(kc + D, nk - 1), ra[st], ra2[st], rw[st]);
        if constexpr (sizeof(T) == 2) {
          bf16x8t af[MT], bfr[NTL];
#pragma unroll
          for (int i = 0; i < MT; ++i) af[i] = *reinterpret_cast<const bf16x8t*>(&As[buf][wrow + 16 * i + r16][q * 8]);
#pragma unroll
          for (int j = 0; j < NTL; ++j) bfr[j] = *reinterpret_cast<const bf16x8t*>(&Bs[buf][wcol + 16 * j + r16][q * 8]);
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NTL; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int t = 0; t < KC / 16; ++t) {
            f4 a4[MT], b4[NTL];
#pragma unroll
            for (int i = 0; i < MT; ++i) a4[i] = *reinterpret_cast<const f4*>(&As[buf][wrow + 16 * i + r16][16 * t + 4 * q]);
#pragma unroll
            for (int j = 0; j < NTL; ++j) b4[j] = *reinterpret_cast<const f4*>(&Bs[buf][wcol + 16 * j + r16][16 * t + 4 * q]);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NTL; ++j)
                  acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b4[j][s], a4[i][s], acc[i][j], 0, 0, 0);
          }
        }
      }
    };
    for (int kc0 = 0; kc0 < nkp; kc0 += D) {
      if (kc0 + D < nkp) group(kc0, true);
      else group(kc0, false);
    }
    TW_MARK(2);

    auto store_c = [&]() {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int rl = wrow + 16 * i + r16;
        if (rl >= nt) continue;
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          const int n = n0 + wcol + 16 * j + 4 * q;
          if (n < N) *reinterpret_cast<f4*>(p.C + (size_t)(mbase + rl) * N + n) = acc[i][j];
        }
      }
    };
    // ---- epilogue: lane holds rows wrow + 16 i + r16, columns n0 + wcol + 16 j + 4 q + (0..3)
    if constexpr (EPI == EPI_L2) {
      float ss[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        ss[i] = 0.f;
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int nl = wcol + 16 * j + 4 * q + e;
            acc[i][j][e] += n0 + nl < N ? ctab[0][nl] : 0.f;
            ss[i] += acc[i][j][e] * acc[i][j][e];
          }
        }
        ss[i] += __shfl_xor(ss[i], 16, 64);
        ss[i] += __shfl_xor(ss[i], 32, 64);
      }
      if constexpr (WC > 1) {
        // the row's column groups sit in WC waves: their partial sums of squares meet in LDS and
        // are added in column-group order (the same bits in every wave)
        __shared__ float l2red[WC][TM];
        lds_barrier();
        if (q == 0) l2red[wave / WR][wrow + r16] = ss[0];
        lds_barrier();
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WC; ++w) t += l2red[w][wrow + r16];
        ss[0] = t;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int rl = wrow + 16 * i + r16;
        const float nrm = sqrtf(ss[i]);
        const float den = fmaxf(nrm, p.l2eps);
        if (rl < nt && q == 0 && wcol == 0) p.norm_out[mbase + rl] = nrm;
#pragma unroll
        for (int j = 0; j < NTL; ++j) acc[i][j] /= den;
      }
      store_c();
      TW_MARK(6);
      TW_MARK(7);
    } else {
      // EPI_STATS: z = acc + bias; EPI_BWD: g = mask(acc) of the BatchNorm below. Both go through
      // an LDS tile (value, and g * xhat) whose columns 256 threads sum over the valid rows
      static_assert(TN == 64, "the statistics hand-off works on 64-column blocks");
      DropKey ek{};
      const bool edrop = EPI == EPI_BWD && p.e_drop_p > 0.f;
      if (edrop) ek = make_key(p.e_key, p.e_site, p.e_drop_p);
      lds_barrier();  // every wave is done reading the operand stages the tile reuses
      float* t0 = reinterpret_cast<float*>(smem);
      float* t1 = t0 + TM * TP;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int rl = wrow + 16 * i + r16;
        const int m = mbase + rl;
#pragma unroll
        for (int j = 0; j < NTL; ++j) {
          const int nl = wcol + 16 * j + 4 * q;
          float mk[4] = {1.f, 1.f, 1.f, 1.f};
          if constexpr (EPI == EPI_BWD) {
            if (edrop) {  // m*N + n even: two pair hashes
              const uint32_t pr = ((uint32_t)m * (uint32_t)N + (uint32_t)(n0 + nl)) >> 1;
              keep_pair32(ek, pr, mk[0], mk[1]);
              keep_pair32(ek, pr + 1, mk[2], mk[3]);
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (EPI == EPI_STATS) {
              acc[i][j][e] += ctab[0][nl + e];
              t0[rl * TP + nl + e] = acc[i][j][e];
            } else {
              const float zc = ez[i][j][e] - ctab[0][nl + e];
              float gv = acc[i][j][e];
              if (p.e_relu) {
                // the forward's exact expression (pro_apply<PRO_BN>): y > 0 <=> yb > 0 and kept
                const float yb = fmaf(zc, __fmul_rn(ctab[1][nl + e], ctab[2][nl + e]), ctab[3][nl + e]);
                gv = yb > 0.f ? gv * mk[e] : 0.f;
              }
              acc[i][j][e] = gv;
              t0[rl * TP + nl + e] = gv;
              t1[rl * TP + nl + e] = gv * (zc * ctab[1][nl + e]);
            }
          }
        }
      }
      lds_barrier();
      TW_MARK(3);
      // column sums: thread (c, rq) sums rows rq*TM/4 .. of column c (rows past nt excluded)
      const int c = tid & 63, rq = tid >> 6;
      constexpr int RQ = TM / 4;
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int u = 0; u < RQ; ++u) {
        const int r = rq * RQ + u;
        const bool ok = r < nt;
        s0 += ok ? t0[r * TP + c] : 0.f;
        if constexpr (EPI == EPI_BWD) s1 += ok ? t1[r * TP + c] : 0.f;
      }
      red[0][rq][c] = s0;
      if constexpr (EPI == EPI_BWD) red[1][rq][c] = s1;
      lds_barrier();
      float v0, v1;
      if constexpr (EPI == EPI_STATS) {
        // tile mean, then M2 about it from the same LDS tile
        v0 = (red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c]) / (float)nt;
        float m2 = 0.f;
#pragma unroll
        for (int u = 0; u < RQ; ++u) {
          const int r = rq * RQ + u;
          const float d = t0[r * TP + c] - v0;
          m2 += r < nt ? d * d : 0.f;
        }
        red[1][rq][c] = m2;
        lds_barrier();
        v1 = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
      } else {
        v0 = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
        v1 = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
      }
      TW_MARK(4);
      const int ncols = min(TN, N - n0);
      const FinPre pre = fin_preload(p.fin, nblk, ncols);
      const bool last = fin_publish(p.fin, N, p.tiles, g, tile, nblk, ncols, v0, v1);
      TW_MARK(5);
      // the last arriver issues its merge's first loads, then its own output stores (their
      // latency under the loads'), then merges
      MergeFirst mf;
      if (last) fin_merge_load(p.fin, N, p.tiles, g, nblk, ncols, mf);
      store_c();
      TW_MARK(6);
      if (last) fin_merge<true>(p.fin, N, p.G, p.Bg, p.tiles, TM, g, nblk, ncols, pre, mf);
      TW_MARK(7);
    }
  }
}

// feature_bn's input statistics: tile (mean, M2) per column of x [G*Bg, C] over TM_STATS rows,
// handed to the last arriver of each (group, 64-column block) like a GEMM epilogue's
__global__ __launch_bounds__(256) void tower_stats_kernel(const float* __restrict__ x, int Bg,
                                                          int C, int G, int tiles, Fin fin,
                                                          int64_t* __restrict__ rng_state,
                                                          int64_t* __restrict__ key_out) {
  // the MLP's dropout key of this step (rs_rng_next folded in: one dependent launch less)
  if (rng_state && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    key_out[0] = rng_state[0];
    key_out[1] = rng_state[1];
    rng_state[1] = rng_state[1] + 1;
  }
  constexpr int R = TM_STATS / 4;  // rows per thread
  __shared__ float red[4][64];
  __shared__ float tmean[64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int g = blockIdx.y / tiles, tile = blockIdx.y % tiles;
  const int nt = tile_rows(TM_STATS, Bg, tile);
  const size_t base = (size_t)g * Bg + (size_t)tile * TM_STATS;
  const int cc = min(c, C - 1);
  float v[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int r = rl + 4 * u;
    v[u] = r < nt ? x[(base + r) * C + cc] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < R; ++u) s += v[u];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0) tmean[cl] = (red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]) / (float)nt;
  __syncthreads();
  const float mu = tmean[cl];
  float m2 = 0.f;
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const float d = v[u] - mu;
    m2 += rl + 4 * u < nt ? d * d : 0.f;
  }
  __syncthreads();
  red[rl][cl] = m2;
  __syncthreads();
  const float m2t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
  const int ncols = min(64, C - (int)blockIdx.x * 64);
  const FinPre pre = fin_preload(fin, blockIdx.x, ncols);
  if (fin_publish(fin, C, tiles, g, tile, blockIdx.x, ncols, mu, m2t))
    fin_merge<false>(fin, C, G, Bg, tiles, TM_STATS, g, blockIdx.x, ncols, pre, MergeFirst{});
}

// ---------------------------------------------------------------------------- host side
constexpr int TM_MIN = 16;  // smallest GEMM row tile: rs_tower_part_floats sizes the partials for it

unsigned long long* g_dbg = nullptr;  // rs_tower_debug_buffer: profiling only

template <typename T, int TM, int TN, int PRO, int EPI, int DCH>
int launch_d(const TwArgs& a, int nblocks, hipStream_t st, const char* name) {
  TwArgs b = a;
  b.dbg = g_dbg;
  b.tiles = cdiv(b.Bg, TM);
  b.nbx = nblocks;
  const int rts = cdiv(b.G * b.tiles, 8) * 8;  // row tiles padded to whole XCD groups
  tower_kernel<T, TM, TN, PRO, EPI, DCH><<<dim3(nblocks * rts), 256, 0, st>>>(b);
  RS_CHECK_LAUNCH(name);
  return 0;
}

// k chunks in flight: the smallest of 2 / 3 / 4 / 5 / 8 / 10 that covers the K extent, so every
// operand load of a workgroup goes out in one round trip, within a register budget for the staged
// chunks set by the residency the grid needs (one or two workgroups per CU: ~160 VGPRs; more:
// ~64). A chunk stages LA (x2 with a second A input) + LW float4 per thread.
template <typename T, int TM, int TN, int PRO, int EPI>
int launch_tm(const TwArgs& a, int nblocks, hipStream_t st, const char* name) {
  constexpr bool TWO = PRO == PRO_BNB || PRO == PRO_L2B;
  constexpr int LA = (TM * (KC / 4) + 255) / 256, LW = (TN * (KC / 4) + 255) / 256;
  constexpr int regs = 4 * (LA * (TWO ? 2 : 1) + LW);
  const int nk = cdiv(a.K, KC);
  const int64_t grid = (int64_t)nblocks * (cdiv(a.G * cdiv(a.Bg, TM), 8) * 8);
  const int per_cu = (int)((grid + 255) / 256);
  const int budget = per_cu > 2 ? 64 : (TN > 64 || TM == 64 ? 160 : 176);
  static const int opts[] = {2, 3, 4, 5, 8, 10};
  int d = 2;
  for (int o : opts) {
    if (o * regs > budget) break;
    d = o;
    if (o >= nk) break;
  }
#define RS_TW_LAUNCH(DV) return launch_d<T, TM, TN, PRO, EPI, DV>(a, nblocks, st, name)
  switch (d) {
    case 2: RS_TW_LAUNCH(2);
    case 3: RS_TW_LAUNCH(3);
    case 4: RS_TW_LAUNCH(4);
    case 5: RS_TW_LAUNCH(5);
    case 8: RS_TW_LAUNCH(8);
    default: RS_TW_LAUNCH(10);
  }
#undef RS_TW_LAUNCH
}

// Row tile per launch (round 4): 64 rows when that grid fills the chip (193..256 workgroups, or
// >= 512), else 32 (B = 4096 gives 64 row tiles: a 128-column Linear was 128 workgroups on 256 CUs); the final
// Linear (whole rows per workgroup for F.normalize, no statistics hand-off) goes to 16 rows when
// 32 still leave CUs idle. Measured (tools/tower_phases.py, C3 user tower): the 128-column
// forward 22 -> 17 us, the final Linear 14 -> 6 us, the 128-column backward 19 -> 17 us; 32-row
// tiles on grids that were already >= 256 workgroups were slower (their last arriver merges twice
// the tiles).
template <typename T, int TN, int PRO, int EPI>
int launch(const TwArgs& a, int nblocks, hipStream_t st, const char* name) {
  auto wgs = [&](int tm) { return (int64_t)nblocks * (cdiv(a.G * cdiv(a.Bg, tm), 8) * 8); };
  // 64 rows fill the chip once (193..256 workgroups) or at two and more per CU; between, a 64-row
  // grid runs a second partial wave of workgroups (C3's 320-workgroup first-layer backward: 40 us
  // at 64 rows, 25 us at 32)
  const int64_t w64 = wgs(64);
  int tm = (w64 > 192 && w64 <= 256) || w64 >= 512 ? 64 : 32;
  if (EPI == EPI_L2 && wgs(32) < 256) tm = 16;
  if constexpr (EPI == EPI_L2) {
    if (tm == 16) return launch_tm<T, 16, TN, PRO, EPI>(a, nblocks, st, name);
  }
  if (tm == 64) return launch_tm<T, 64, TN, PRO, EPI>(a, nblocks, st, name);
  return launch_tm<T, 32, TN, PRO, EPI>(a, nblocks, st, name);
}

template <typename T>
int fwd_dispatch(const TwArgs& a, bool final_l2, hipStream_t st) {
  if (final_l2) {
    if (a.N <= 64) return launch<T, 64, PRO_BN, EPI_L2>(a, 1, st, "rs_tower_fwd l2");
    return launch<T, 128, PRO_BN, EPI_L2>(a, 1, st, "rs_tower_fwd l2");
  }
  return launch<T, 64, PRO_BN, EPI_STATS>(a, cdiv(a.N, 64), st, "rs_tower_fwd");
}

template <typename T, int PRO>
int bwd_dispatch(const TwArgs& a, hipStream_t st) {
  return launch<T, 64, PRO, EPI_BWD>(a, cdiv(a.N, 64), st, "rs_tower_bwd");
}


// ------------------------------------------------------------------------ weight gradients
// dW[N][K] += dz^T h and db[N] += colsum(dz) of every Linear of a tower in ONE launch (a grouped
// GEMM over the layers' tiles), bf16 mode: 64 x 64 dW tiles, the M rows split S ways per tile;
// each workgroup streams 32-row chunks of dz and h (fp32, rounded to bf16 while staged
// row-major in LDS) and reads the MFMA operands with ds_read_b64_tr_b16 (8 consecutive rows of a
// column per lane) into v_mfma_f32_32x32x16_bf16. The S partial tiles meet in a fixed order: the
// workgroup arriving last for a tile (write-through partials, one ticket per workgroup) sums them
// s = 0..S-1 and adds the sum into dW (and db: fp32 column sums of the unrounded dz).
// fp32 mode: the same kernel on v_mfma_f32_32x32x2_f32, chunks staged as fp32 (pitch 96 floats:
// the two rows of a k-step fall in opposite bank halves) and read one element per lane.
typedef short wshortx4 __attribute__((ext_vector_type(4)));
typedef short wshortx8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
constexpr int WG_MAXJ = 4;
constexpr int WCH = 32;         // rows per chunk
constexpr int WPITCH = 96;      // bf16 LDS pitch of a 64-wide image (4 rows of a transposed read in distinct 64-B windows)

struct WgJob {
  const float* dz;  // [M][N]
  const float* h;   // [M][K]
  float* dW;        // [N][K] (+=)
  float* db;        // [N] (+=)
  float* part;      // [tiles][S][16][256] dW partials, then [tiles_n][S][64] db partials
  int* cnt;         // [tiles] tickets (zero on entry and exit)
  int N, K, tn, tk, S, R, wg0;
};
struct WgArgs {
  WgJob j[WG_MAXJ];
  int nj, M;
};

__device__ __forceinline__ bf16x8t wtr_frag(const __bf16* lo, const __bf16* hi) {
  typedef __attribute__((address_space(3))) wshortx4* lptr;
  const wshortx4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lo));
  const wshortx4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(hi));
  const wshortx8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8t, v);
}

template <typename T>
__global__ __launch_bounds__(256) void tower_wgrad_kernel(WgArgs a) {
  constexpr int D = 3;  // chunks of loads in flight per thread
  constexpr bool F32 = sizeof(T) == 4;
  __shared__ __attribute__((aligned(16))) T Ys[2][WCH][WPITCH];
  __shared__ __attribute__((aligned(16))) T Xs[2][WCH][WPITCH];
  __shared__ float csum[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int ji = 0;
  for (int q = 1; q < a.nj; ++q)
    if ((int)blockIdx.x >= a.j[q].wg0) ji = q;
  const WgJob& J = a.j[ji];
  const int local = blockIdx.x - J.wg0;
  const int tile = local / J.S, s = local % J.S;
  const int tn = tile / J.tk, tk = tile % J.tk;
  const int n0 = tn * 64, k0 = tk * 64;
  const int r0 = s * J.R, r1 = min(a.M, r0 + J.R);
  const int N = J.N, K = J.K;
  const bool do_db = tk == 0 && J.db;
  // loads: dz rows [32][64] and h rows [32][64], 2 float4 each per thread
  const int lr = tid >> 4, lc = (tid & 15) * 4;  // rows lr, lr + 16; columns lc..lc+3
  f4 ry[D][2], rx[D][2];
  const int nch = (r1 - r0 + WCH - 1) / WCH;
  auto load = [&](int ch, f4 (&ry)[2], f4 (&rx)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int m = min(r0 + ch * WCH + lr + 16 * u, r1 - 1);
      ry[u] = *reinterpret_cast<const f4*>(J.dz + (size_t)m * N + min(n0 + lc, N - 4));
      rx[u] = *reinterpret_cast<const f4*>(J.h + (size_t)m * K + min(k0 + lc, K - 4));
    }
  };
  float ysum[4] = {0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int ch, int buf, f4 (&ry)[2], f4 (&rx)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = lr + 16 * u;
      const bool rok = r0 + ch * WCH + row < r1;
      const f4 y = rok && n0 + lc < N ? ry[u] : f4{0.f, 0.f, 0.f, 0.f};
      const f4 x = rok && k0 + lc < K ? rx[u] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) ysum[e] += y[e];
      lds_put4<T>(&Ys[buf][row][lc], y);
      lds_put4<T>(&Xs[buf][row][lc], x);
    }
  };
  f16v acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  const int wm = wave >> 1, wn = wave & 1;  // 32 x 32 sub-tile of the wave: n rows wm, k cols wn
  const int gq = lane >> 4, lq = (lane & 15) >> 2, lp = lane & 3;
  const int trow = 8 * (gq >> 1) + lq, tcol = 16 * (gq & 1) + 4 * lp;
#pragma unroll
  for (int st = 0; st < D; ++st) load(min(st, nch - 1), ry[st], rx[st]);
  const int nchp = (nch + D - 1) / D * D;  // padded: padding chunks stage zeros
  for (int c0 = 0; c0 < nchp; c0 += D) {
#pragma unroll
    for (int st = 0; st < D; ++st) {
      const int ch = c0 + st;
      const int buf = ch & 1;
      stage(ch, buf, ry[st], rx[st]);
      lds_barrier();
      load(min(ch + D, nch - 1), ry[st], rx[st]);
      if constexpr (F32) {
        // k-step q: rows 2q (lanes 0-31) and 2q + 1 (lanes 32-63); A = dz[m][n0 + 32 wm + c],
        // B = h[m][k0 + 32 wn + c]
        const int c = lane & 31, hh = lane >> 5;
#pragma unroll
        for (int q = 0; q < WCH / 2; ++q)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ys[buf][2 * q + hh][32 * wm + c], Xs[buf][2 * q + hh][32 * wn + c],
                                                     acc, 0, 0, 0);
      } else {
#pragma unroll
        for (int ks = 0; ks < WCH / 16; ++ks) {
          const __bf16* py = &Ys[buf][16 * ks + trow][32 * wm + tcol];
          const __bf16* px = &Xs[buf][16 * ks + trow][32 * wn + tcol];
          const bf16x8t af = wtr_frag(py, py + 4 * WPITCH);
          const bf16x8t bf = wtr_frag(px, px + 4 * WPITCH);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
        }
      }
    }
  }
  // column sums of dz (db), per thread over its rows, then the 16 row lanes in order
  float dbv = 0.f;
  if (do_db) {
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[lr][lc + e] = ysum[e];
    lds_barrier();
    if (tid < 64)
#pragma unroll
      for (int r = 0; r < 16; ++r) dbv += csum[r][tid];
  }
  // partial -> write-through, ticket; the last arriver of the tile sums the S partials in order
  float* pt = J.part + ((size_t)tile * J.S) * 4096;
#pragma unroll
  for (int e = 0; e < 16; ++e) st_sc1(pt + (size_t)s * 4096 + e * 256 + tid, acc[e]);
  float* pdb = J.part + (size_t)J.tn * J.tk * J.S * 4096 + ((size_t)tn * J.S) * 64;
  if (do_db && tid < 64) st_sc1(pdb + s * 64 + tid, dbv);
  if (!ticket(J.cnt + tile, J.S - 1)) return;
  // the S partials (this workgroup's own included: its sc1 stores are drained) summed in split
  // order, 4 splits' loads in flight at a time: one split per round trip made the last arriver's
  // tail ~S x 1.5 us
  f16v sum;
#pragma unroll
  for (int e = 0; e < 16; ++e) sum[e] = 0.f;
  constexpr int QB = 4;
  for (int q0 = 0; q0 < J.S; q0 += QB) {
    f16v v[QB];
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int q = min(q0 + u, J.S - 1);
#pragma unroll
      for (int e = 0; e < 16; ++e) v[u][e] = ld_sc1(pt + (size_t)q * 4096 + e * 256 + tid);
    }
#pragma unroll
    for (int u = 0; u < QB; ++u)
      if (q0 + u < J.S) sum += v[u];
  }
  // dW += sum: every old value loaded before any is stored (a load after a store to the same
  // array would wait for the store: 16 serial round trips)
  const int kk = k0 + 32 * wn + (lane & 31);
  float* __restrict__ dWp = J.dW;
  float old[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int nn = min(n0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5), N - 1);
    old[e] = dWp[(size_t)nn * K + min(kk, K - 1)];
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int nn = n0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
    if (nn < N && kk < K) dWp[(size_t)nn * K + kk] = old[e] + sum[e];
  }
  if (do_db && tid < 64 && n0 + tid < N) {
    float dv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dv[q] = ld_sc1(pdb + min(q, J.S - 1) * 64 + tid);
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q < J.S) t += dv[q];
    for (int q = 16; q < J.S; ++q) t += ld_sc1(pdb + q * 64 + tid);
    J.db[n0 + tid] += t;
  }
  if (tid == 0) __hip_atomic_store(J.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

bool al16(const void* p) { return !p || aligned16(p); }

}  // namespace
}  // namespace rs

using namespace rs;

// Profiling only (tools/tower_phases.py): GEMM instances record per-workgroup phase timestamps
// (wall_clock64, 100 MHz) into buf [workgroups][8] while it is set; NULL turns it off.
extern "C" int rs_tower_debug_buffer(unsigned long long* buf) {
  g_dbg = buf;
  return 0;
}

extern "C" int64_t rs_tower_part_floats(int G, int Bg, int N, int kind) {
  const int tm = kind == 0 ? TM_STATS : TM_MIN;
  return (int64_t)G * cdiv(Bg, tm) * 2 * N;
}

extern "C" int rs_tower_sync_ints(int G, int N) { return (G + 1) * cdiv(N, 64); }

extern "C" int rs_tower_stats(const float* x, int G, int Bg, int C, float* part, int* sync,
                              double* scratch, float* mean, float* rstd, float* running_mean,
                              float* running_var, int64_t* num_batches, float momentum, float eps,
                              int64_t* rng_state, int64_t* key_out, void* stream) {
  RS_CHECK_ARG(x && part && sync && scratch && mean && rstd, "rs_tower_stats: null pointer");
  RS_CHECK_ARG(!rng_state == !key_out, "rs_tower_stats: rng_state and key_out come together");
  RS_CHECK_ARG(G >= 1 && Bg >= 1 && C >= 1, "rs_tower_stats: bad shape G=%d Bg=%d C=%d", G, Bg, C);
  RS_CHECK_ARG(!running_mean == !running_var, "rs_tower_stats: running stats must come together");
  Fin f{};
  f.part = part; f.cnt = sync; f.scratch = scratch; f.o0 = mean; f.o1 = rstd;
  f.run_mean = running_mean; f.run_var = running_var; f.nbt = num_batches;
  f.momentum = momentum; f.eps = eps; f.bwd = 0; f.nb = cdiv(C, 64);
  const int tiles = cdiv(Bg, TM_STATS);
  tower_stats_kernel<<<dim3(f.nb, G * tiles), 256, 0, as_stream(stream)>>>(x, Bg, C, G, tiles, f, rng_state,
                                                                          key_out);
  RS_CHECK_LAUNCH("rs_tower_stats");
  return 0;
}

extern "C" int rs_tower_fwd(const float* A, int G, int Bg, int K, const float* in_mean,
                            const float* in_rstd, const float* bn_w, const float* bn_b, int relu,
                            float drop_p, const int64_t* key, int site, float* h_out,
                            const float* W, const float* bias, int N, float* z, float* part,
                            int* sync, double* scratch, float* mean, float* rstd,
                            float* running_mean, float* running_var, int64_t* num_batches,
                            float momentum, float eps, float* out, float* norm, float l2_eps,
                            int bf16, void* stream) {
  RS_CHECK_ARG(A && in_mean && in_rstd && bn_w && bn_b && W && bias, "rs_tower_fwd: null pointer");
  RS_CHECK_ARG((z && part && sync && scratch && mean && rstd && !out) || (!z && out && norm),
               "rs_tower_fwd: give z + its statistics hand-off (hidden) or out + norm (final)");
  RS_CHECK_ARG(G >= 1 && Bg >= 1 && K >= 4 && K <= KMAX && K % 4 == 0 && N >= 4 && N % 4 == 0,
               "rs_tower_fwd: bad shape G=%d Bg=%d K=%d N=%d", G, Bg, K, N);
  RS_CHECK_ARG(!out || N <= 128, "rs_tower_fwd: final layer wider than 128 (N=%d)", N);
  RS_CHECK_ARG(drop_p == 0.f || (relu && key && drop_p > 0.f && drop_p < 1.f), "rs_tower_fwd: bad dropout");
  RS_CHECK_ARG(!running_mean == !running_var, "rs_tower_fwd: running stats must come together");
  RS_CHECK_ARG((int64_t)G * Bg * (int64_t)(K > N ? K : N) < (1ll << 32),
               "rs_tower_fwd: too many elements for the dropout index");
  RS_CHECK_ARG(al16(A) && al16(W) && al16(bias) && al16(h_out) && al16(z) && al16(out),
               "rs_tower_fwd: pointers must be 16-byte aligned");
  TwArgs a{};
  a.A = A; a.W = W; a.bias = bias; a.N = N; a.K = K; a.G = G; a.Bg = Bg; a.wt = 0;
  a.in_mean = in_mean; a.in_rstd = in_rstd; a.in_w = bn_w; a.in_b = bn_b;
  a.relu = relu; a.drop_p = drop_p; a.key = key; a.site = site;
  a.h_out = h_out;
  a.C = z ? z : out; a.norm_out = norm; a.l2eps = l2_eps;
  a.fin.part = part; a.fin.cnt = sync; a.fin.scratch = scratch; a.fin.o0 = mean; a.fin.o1 = rstd;
  a.fin.run_mean = running_mean; a.fin.run_var = running_var; a.fin.nbt = num_batches;
  a.fin.momentum = momentum; a.fin.eps = eps; a.fin.bwd = 0; a.fin.nb = cdiv(N, 64);
  hipStream_t st = as_stream(stream);
  return bf16 ? fwd_dispatch<__bf16>(a, out != nullptr, st) : fwd_dispatch<float>(a, out != nullptr, st);
}

extern "C" int rs_tower_bwd(const float* gin, int G, int Bg, int K, const float* y,
                            const float* norm, float l2_eps, const float* z, const float* mean,
                            const float* rstd, const float* bn_w, const float* mg,
                            const float* mgx, float* dz, const float* W, int N, const float* ez,
                            const float* e_mean, const float* e_rstd, const float* e_w,
                            const float* e_b, int e_relu, float e_drop_p, const int64_t* e_key,
                            int e_site, float* g, float* part, int* sync, double* scratch,
                            float* out_mg, float* out_mgx, float* e_dgamma, float* e_dbeta,
                            int bf16, void* stream) {
  const bool l2 = y != nullptr;
  RS_CHECK_ARG(gin && dz, "rs_tower_bwd: null pointer");
  RS_CHECK_ARG(l2 ? (norm != nullptr) : (z && mean && rstd && bn_w && mg && mgx),
               "rs_tower_bwd: prologue inputs missing");
  RS_CHECK_ARG(G >= 1 && Bg >= 1 && K >= 4 && K % 4 == 0 && N >= 0 && N % 4 == 0 && (l2 || K <= KMAX),
               "rs_tower_bwd: bad shape G=%d Bg=%d K=%d N=%d", G, Bg, K, N);
  RS_CHECK_ARG(N == 0 || (W && ez && e_mean && e_rstd && g && part && sync && scratch && out_mg &&
                          out_mgx && e_dgamma && e_dbeta && (!e_relu || (e_w && e_b))),
               "rs_tower_bwd: epilogue inputs missing");
  RS_CHECK_ARG(N > 0 || !l2, "rs_tower_bwd: N = 0 needs the BatchNorm prologue");
  RS_CHECK_ARG(e_drop_p == 0.f || (e_relu && e_key && e_drop_p > 0.f && e_drop_p < 1.f), "rs_tower_bwd: bad dropout");
  RS_CHECK_ARG((int64_t)G * Bg * (int64_t)(N > K ? N : K) < (1ll << 32), "rs_tower_bwd: too many elements");
  RS_CHECK_ARG(al16(gin) && al16(y) && al16(z) && al16(dz) && al16(W) && al16(ez) && al16(e_mean) &&
                   al16(e_rstd) && al16(e_w) && al16(e_b) && al16(g),
               "rs_tower_bwd: pointers must be 16-byte aligned");
  TwArgs a{};
  a.A = gin; a.A2 = l2 ? y : z; a.W = W; a.N = N; a.K = K; a.G = G; a.Bg = Bg; a.wt = 1;
  a.rownorm = norm; a.l2eps = l2_eps;
  a.in_mean = mean; a.in_rstd = rstd; a.in_w = bn_w; a.in_mg = mg; a.in_mgx = mgx;
  a.h_out = dz;
  a.eZ = ez; a.e_mean = e_mean; a.e_rstd = e_rstd; a.e_w = e_w; a.e_b = e_b; a.e_relu = e_relu;
  a.e_drop_p = e_drop_p; a.e_key = e_key; a.e_site = e_site;
  a.C = g;
  a.fin.part = part; a.fin.cnt = sync; a.fin.scratch = scratch; a.fin.o0 = out_mg; a.fin.o1 = out_mgx;
  a.fin.dgamma = e_dgamma; a.fin.dbeta = e_dbeta; a.fin.bwd = 1; a.fin.nb = cdiv(N, 64);
  hipStream_t st = as_stream(stream);
  if (N == 0) {
    a.tiles = cdiv(Bg, 16);
    a.nbx = 1;
    tower_kernel<float, 16, 16, PRO_BNB, EPI_NONE><<<dim3(1, G * a.tiles), 256, 0, st>>>(a);
    RS_CHECK_LAUNCH("rs_tower_bwd dx");
    return 0;
  }
  if (l2) return bf16 ? bwd_dispatch<__bf16, PRO_L2B>(a, st) : bwd_dispatch<float, PRO_L2B>(a, st);
  return bf16 ? bwd_dispatch<__bf16, PRO_BNB>(a, st) : bwd_dispatch<float, PRO_BNB>(a, st);
}

// Weight gradients of up to 4 Linears in one launch (tower_wgrad_kernel). Per layer i: dz_i
// [M][N_i], h_i [M][K_i], dW_i [N_i][K_i] += dz^T h, db_i [N_i] += colsum(dz) (may be NULL);
// ws_i: rs_tower_wgrad_ws_floats(M, N_i, K_i) floats; sync_i: rs_tower_wgrad_sync_ints(N_i, K_i)
// ints, zero on entry (zero again on exit). bf16 != 0: operands rounded to bf16 on
// v_mfma_f32_32x32x16_bf16; 0: exact fp32 products on v_mfma_f32_32x32x2_f32.
extern "C" int rs_tower_wgrad_split(int M, int N, int K) {
  const int tiles = cdiv(N, 64) * cdiv(K, 64);
  int S = (256 + tiles - 1) / tiles;
  const int smax = cdiv(M, 256);  // >= 256 rows per split
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  return S;
}
extern "C" int64_t rs_tower_wgrad_ws_floats(int M, int N, int K) {
  const int S = rs_tower_wgrad_split(M, N, K);
  return (int64_t)cdiv(N, 64) * cdiv(K, 64) * S * 4096 + (int64_t)cdiv(N, 64) * S * 64;
}
extern "C" int rs_tower_wgrad_sync_ints(int N, int K) { return cdiv(N, 64) * cdiv(K, 64); }

extern "C" int rs_tower_wgrad(int nlayers, int M, const int* Ns, const int* Ks,
                              const float* const* dz, const float* const* h, float* const* dW,
                              float* const* db, float* const* ws, int* const* sync, int bf16, void* stream) {
  RS_CHECK_ARG(nlayers >= 1 && nlayers <= WG_MAXJ && M >= 1, "rs_tower_wgrad: bad nlayers %d / M %d", nlayers, M);
  WgArgs a{};
  a.nj = nlayers;
  a.M = M;
  int wg = 0;
  for (int i = 0; i < nlayers; ++i) {
    const int N = Ns[i], K = Ks[i];
    RS_CHECK_ARG(N >= 4 && K >= 4 && N % 4 == 0 && K % 4 == 0, "rs_tower_wgrad: bad shape N=%d K=%d", N, K);
    RS_CHECK_ARG(dz[i] && h[i] && dW[i] && ws[i] && sync[i], "rs_tower_wgrad: null pointer (layer %d)", i);
    RS_CHECK_ARG(al16(dz[i]) && al16(h[i]), "rs_tower_wgrad: operands must be 16-byte aligned");
    WgJob& j = a.j[i];
    j.dz = dz[i]; j.h = h[i]; j.dW = dW[i]; j.db = db[i]; j.part = ws[i]; j.cnt = sync[i];
    j.N = N; j.K = K; j.tn = cdiv(N, 64); j.tk = cdiv(K, 64);
    j.S = rs_tower_wgrad_split(M, N, K);
    j.R = cdiv(cdiv(M, j.S), WCH) * WCH;
    j.S = cdiv(M, j.R);  // splits that hold rows
    j.wg0 = wg;
    wg += j.tn * j.tk * j.S;
  }
  if (bf16) tower_wgrad_kernel<__bf16><<<wg, 256, 0, as_stream(stream)>>>(a);
  else tower_wgrad_kernel<float><<<wg, 256, 0, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_tower_wgrad");
  return 0;
}
