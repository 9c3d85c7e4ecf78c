// Multi-table feature gather / scatter-add for the tower inputs and the per-token sequence
// features (K1, K2, K3, K10, K11 of SURVEY.md §2.2).
//
// One launch covers every feature of a tower: the host turns the config into a list of
// segments (rs_feature_seg_t) and each workgroup owns one segment x a tile of rows, so the
// concat buffer [rows, ldo] is written directly (no torch.cat). A row of D floats is read by
// D/4 consecutive lanes with 16-byte loads (a 128-wide row = 32 lanes = one 512 B burst), a
// bag (pooled feature) is accumulated in registers by the same lanes, so the index and the
// row reads stay coalesced and the HBM traffic is exactly ids + rows + output.
//
// Backward: dense [V, D] table gradients (the reference uses sparse=False embeddings, T16) by
// float atomics, skipping the padding row as embedding_dense_backward does; Linear(1, D) dense
// features by a deterministic column reduction; last-valid rows by a plain copy-add.
//
// Read-through catch-up (rs_gather_fwd_lazy): a large lazy-Adam table's segment (lazy_last set)
// returns each row as rs_sorted_catchup would leave it -- the zero-gradient Adam steps the row
// missed replayed in registers from its exp_avg / exp_avg_sq -- without writing the row, its
// moments or `last`. The optimizer step replays the same steps before its own (lookup.hip
// kAdam), so the stored state is the same bits; the forward's separate catch-up pass (read p, m,
// v and write them back: 6 row transfers per distinct row) becomes 2 extra row reads per lookup.
#include <atomic>

#include "adam.h"
#include "common.h"

namespace rs {
namespace {

std::atomic<int> g_deterministic{0};  // rs_set_deterministic
bool deterministic() { return g_deterministic.load(std::memory_order_relaxed) || getenv_flag("RSYS_DETERMINISTIC"); }

constexpr int kMaxSeg = 20;  // segments travel by value in the kernel arguments (~2.4 KB)
// tables up to this size get their gradient accumulated in LDS first (privatised per workgroup,
// then one global atomic per touched element): a 30-row genre table hit 600k times per step
// would otherwise serialise on a few hundred addresses
constexpr int64_t kSmallTableBytes = 48 * 1024;

constexpr int kRowsPerLane = 4;            // forward sparse rows per lane on token-sized launches
constexpr int kBagBatch = 16;              // bag ids (and rows) loaded per batch
constexpr int kLazyBagBatch = 8;           // the same with exp_avg / exp_avg_sq rows beside them
// forward: a table of at most this size whose workgroup reads at least as many row bytes as the
// table holds is staged whole into LDS first (every row of such a table is hot: the genre / age /
// occupation tables are read thousands of times per step), and its lookups are served from LDS
constexpr int kStageBytes = 16 * 1024;
// forward, pooled (mean / sum) lookups of a large table with its sorted call (seg.hot_keys), opt-in
// (RSYS_HOT_ROWS=1): the hot rows -- runs of >= 2 kHotQ equal sorted keys, found by sampling every
// kHotQ-th key -- are staged once per workgroup into LDS (up to kHotMax rows) and served from there
// through flat loads; the segment runs kHotBlocks persistent workgroups (the staging is paid per
// workgroup). Measured slower (round 5, C3 fp32 in the step, two repetitions): the history
// gather 0.039 -> 0.086 ms per step with uniform ids (the padding row is half the lookups) and
// 0.038 -> 0.087 ms with Zipf(1.05) ids -- 256 persistent workgroups keep far fewer row loads in
// flight than the 2,048 short ones, and the hot rows are already served by L2
constexpr int kHotQ = 256;
constexpr int kHotMax = 64;
constexpr int kHotHash = 256;
constexpr int kHotBlocks = 256;

// read-through catch-up of lazy-Adam segments: the moments sit at fixed element offsets from the
// parameters (one flat buffer each), the step counter and per-step constants are the optimizer's
struct LazyLaunch {
  int64_t moff, voff;     // floats from a table element to its exp_avg / exp_avg_sq element
  const int64_t* step;    // optimizer steps taken: rows are returned as of this step
  const float2* consts;   // {lr / bc1(s), 1 / sqrt(bc2(s))}; consts[0] = {capacity, overflow}
  AdamConst h;
};

struct SegLaunch {
  rs_feature_seg_t segs[kMaxSeg];
  int nseg;
  int rows;
  float* out;  // fwd: concat out; bwd: unused
  const float* dout;
  int ldo;
  int* err;
  int block_start[kMaxSeg + 1];
  int16_t rpb[kMaxSeg];   // rows per block
  int16_t chunks[kMaxSeg];  // lanes per row
  uint8_t vec[kMaxSeg];
  uint8_t small[kMaxSeg];   // bwd: table gradient accumulated in LDS (kernel gather_bwd_small)
  int sblock_start[kMaxSeg + 1];
  int sblocks[kMaxSeg];
  int small_lds;        // bytes of dynamic LDS for the small-table kernel
  int16_t split[kMaxSeg];   // pooled bags: row groups sharing one bag (positions split S ways)
  int stage[kMaxSeg];   // fwd: bytes of the table staged into LDS (0: read from HBM / L2)
  int stage_lds;        // fwd: dynamic LDS bytes (the largest staged table)
  // bwd, hot mid-size tables (gather_bwd_range_kernel): rows per range, ranges, lookup chunks,
  // first block, offset (floats) of the segment's [chunks][vocab][dim] partials in ws
  int rrows[kMaxSeg];
  int16_t rranges[kMaxSeg];
  int16_t rchunks[kMaxSeg];
  int rblock_start[kMaxSeg + 1];
  uint8_t tiny[kMaxSeg];   // bwd: small table by the slot-image kernel (gather_bwd_slot_kernel)
  int16_t slots[kMaxSeg];  // bwd: its row slots per workgroup (private [V][D] LDS images)
  int slot_lds;            // bwd: dynamic LDS bytes of the slot kernel
  uint8_t rpt[kMaxSeg];    // fwd sparse segments: rows per lane (kRowsPerLane on token-sized launches)
  uint8_t hot[kMaxSeg];    // fwd: pooled lookups with their hot rows staged in LDS (gather_pool_hot)
  int16_t tblocks[kMaxSeg];
  int tblock_start[kMaxSeg + 1];
  // bwd partials (small and ranged tables): [pchunks][vocab][dim] floats at ws + pws_off
  int16_t pchunks[kMaxSeg];
  int64_t pws_off[kMaxSeg];
  // bwd, tiny tables by the one-hot MFMA kernel (gather_bwd_onehot_kernel): lookup rows per wave,
  // first block, dynamic LDS bytes
  uint8_t oh[kMaxSeg];
  int oh_rpw[kMaxSeg];
  int oblock_start[kMaxSeg + 1];
  int oh_lds;
  int64_t ws_floats;
  int range_lds;
  float* ws;
  LazyLaunch lz;  // rs_gather_fwd_lazy only
};
static_assert(sizeof(SegLaunch) <= 4096, "SegLaunch must fit the kernel-argument segment");

__device__ __forceinline__ int find_seg(const SegLaunch& a, int bid) {
  int s = 0;
  while (s + 1 < a.nseg && bid >= a.block_start[s + 1]) ++s;
  return s;
}

__device__ __forceinline__ bool id_ok(int64_t id, int64_t vocab, int* err) {
  if (id < 0 || id >= vocab) {
    if (err) atomicOr(err, 1);
    return false;
  }
  return true;
}

template <bool VEC>
__device__ __forceinline__ void load_row(const float* p, float* v) {
  if (VEC) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = p[0];
  }
}

template <bool VEC>
__device__ __forceinline__ void store_row(float* p, const float* v) {
  if (VEC) *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else p[0] = v[0];
}

// The optimizer step a lazy row is returned at (sparse.hip clamp_step: past the constants'
// capacity the last slot is reused and the optimizer raises its overflow flag).
__device__ __forceinline__ int lazy_target(const LazyLaunch& z) {
  const int cap = __float_as_int(z.consts[0].x);
  const int64_t t = *z.step;
  return t < cap ? (int)t : cap - 1;
}

// Row values p (4 columns) with the row's moments mv / vv and `last`: replay the zero-gradient
// steps last + 1 .. t as rs_sorted_catchup does (nothing to replay, or a row never stepped with
// weight_decay == 0 -- its moments are zero and the replay is the identity; per element, zero
// moments likewise).
template <int W = 4>
__device__ __forceinline__ void lazy_replay(const LazyLaunch& z, int2 last, int t, float* p, const float* mv,
                                            const float* vv) {
  if (last.y >= t || (last.x == 0 && z.h.wd == 0.f)) return;
  float m[W], v[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    m[j] = mv[j];
    v[j] = vv[j];
  }
  adam_catch_row<W>(z.h, z.consts, last.x, last.y, t, p, m, v);
}

// Pooled bag: the (un-normalised) sum or max of positions [lbeg, lend) of row `row`'s bag.
// LAZY: the rows read through the catch-up.
template <bool VEC, bool LAZY = false>
__device__ __forceinline__ void pool_acc(const SegLaunch& a, const rs_feature_seg_t& sg, int row,
                                         int c, int lbeg, int lend, float* acc) {
  constexpr int W = VEC ? 4 : 1;
  constexpr int NB = LAZY ? kLazyBagBatch : kBagBatch;
  const int64_t* ids = sg.idx + (int64_t)row * sg.idx_stride;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = sg.pool_mode == RS_POOL_MAX ? -INFINITY : 0.f;
  // Straight-line code only (no per-row branch or error atomic inside the batch): a branch
  // around each load makes the compiler wait for it before issuing the next.
  const bool is_max = sg.pool_mode == RS_POOL_MAX;
  const int t = LAZY ? lazy_target(a.lz) : 0;
  bool bad = false;
  int64_t raw[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) raw[u] = lbeg + u < lend ? ids[lbeg + u] : 0;
  for (int l0 = lbeg; l0 < lend; l0 += NB) {
    const int nb = lend - l0 < NB ? lend - l0 : NB;
    bool ok[NB];
    float v[NB][4];
    float mv[LAZY ? NB : 1][4], vv[LAZY ? NB : 1][4];
    int2 lst[LAZY ? NB : 1];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const bool valid = raw[u] >= 0 && raw[u] < sg.vocab;
      bad |= u < nb && !valid;
      ok[u] = u < nb && valid;
      const int64_t r = ok[u] ? raw[u] : 0;
      load_row<VEC>(sg.table + r * sg.dim + c, v[u]);
      if constexpr (LAZY) {
        lst[u] = reinterpret_cast<const int2*>(sg.lazy_last)[r];
        load_row<VEC>(sg.table + r * sg.dim + c + a.lz.moff, mv[u]);
        load_row<VEC>(sg.table + r * sg.dim + c + a.lz.voff, vv[u]);
      }
    }
    const int n2 = l0 + NB;
#pragma unroll
    for (int u = 0; u < NB; ++u) raw[u] = n2 + u < lend ? ids[n2 + u] : 0;
    if constexpr (LAZY) {
#pragma unroll
      for (int u = 0; u < NB; ++u)
        if (ok[u]) lazy_replay<W>(a.lz, lst[u], t, v[u], mv[u], vv[u]);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const float x = ok[u] ? v[u][j] : 0.f;
        const float y = is_max ? fmaxf(acc[j], x) : acc[j] + x;
        acc[j] = u < nb ? y : acc[j];
      }
    }
  }
  if (bad && a.err) atomicOr(a.err, 1);
}

template <bool VEC, bool LAZY = false>
__device__ void gather_seg(const SegLaunch& a, const rs_feature_seg_t& sg, int row, int chunk) {
  constexpr int W = VEC ? 4 : 1;
  const int c = chunk * W;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float* o = a.out + (int64_t)row * a.ldo + sg.out_col + c;
  if (sg.kind == RS_SEG_SPARSE) {
    const int64_t id = sg.idx[(int64_t)row * sg.idx_stride];
    if (id_ok(id, sg.vocab, a.err)) {
      const float* pr = sg.table + id * sg.dim + c;
      load_row<VEC>(pr, acc);
      if constexpr (LAZY) {
        float mv[4], vv[4];
        const int2 l = reinterpret_cast<const int2*>(sg.lazy_last)[id];
        load_row<VEC>(pr + a.lz.moff, mv);
        load_row<VEC>(pr + a.lz.voff, vv);
        lazy_replay<W>(a.lz, l, lazy_target(a.lz), acc, mv, vv);
      }
    }
  } else if (sg.kind == RS_SEG_POOL) {
    pool_acc<VEC, LAZY>(a, sg, row, c, 0, sg.bag, acc);
    if (sg.pool_mode == RS_POOL_MEAN) {
      const float n = (float)sg.bag;
#pragma unroll
      for (int j = 0; j < W; ++j) acc[j] = acc[j] / n;
    }
  } else if (sg.kind == RS_SEG_DENSE) {
    const float x = sg.x[(int64_t)row * sg.idx_stride];
#pragma unroll
    for (int j = 0; j < W; ++j) acc[j] = sg.bias[c + j] + x * sg.table[c + j];
  } else if (sg.kind == RS_SEG_LASTVALID) {
    const int64_t l = sg.idx[row];
    load_row<VEC>(sg.table + ((int64_t)row * sg.bag + l) * sg.dim + c, acc);
  } else {  // RS_SEG_COPY
    load_row<VEC>(sg.table + (int64_t)row * sg.dim + c, acc);
  }
  if (VEC) {
    *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  } else {
    o[0] = acc[0];
  }
}

// Sparse lookups, R rows per lane (token-sized launches: C2's 204,800-row sequence gather was 6,400
// workgroups of one float4 per lane, each a serial id -> row -> store chain). The workgroup owns
// rows [lb R rpb, (lb + 1) R rpb); all R ids are loaded, then all R rows, then the R stores, so a
// lane has R independent chains in flight. Same values as gather_seg (bad ids: zeros + err flag).
template <int R, bool LAZY = false>
__device__ void gather_sparse_rows(const SegLaunch& a, const rs_feature_seg_t& sg, int rpb, int lb,
                                   int r, int chunk) {
  const int c = chunk * 4;
  int64_t id[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int row = (lb * R + k) * rpb + r;
    id[k] = row < a.rows ? sg.idx[(int64_t)row * sg.idx_stride] : 0;
  }
  float v[R][4];
  float mv[LAZY ? R : 1][4], vv[LAZY ? R : 1][4];
  int2 lst[LAZY ? R : 1];
  bool okk[R];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int row = (lb * R + k) * rpb + r;
    const bool ok = id[k] >= 0 && id[k] < sg.vocab;
    okk[k] = ok;
    bad |= row < a.rows && !ok;
    const float* pr = sg.table + (ok ? id[k] : 0) * sg.dim + c;
    load_row<true>(pr, v[k]);
    if constexpr (LAZY) {
      lst[k] = reinterpret_cast<const int2*>(sg.lazy_last)[ok ? id[k] : 0];
      load_row<true>(pr + a.lz.moff, mv[k]);
      load_row<true>(pr + a.lz.voff, vv[k]);
    }
  }
  if constexpr (LAZY) {
    const int t = lazy_target(a.lz);
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (okk[k]) lazy_replay(a.lz, lst[k], t, v[k], mv[k], vv[k]);
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[k][j] = okk[k] ? v[k][j] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int row = (lb * R + k) * rpb + r;
    if (row < a.rows) store_row<true>(a.out + (int64_t)row * a.ldo + sg.out_col + c, v[k]);
  }
  if (bad && a.err) atomicOr(a.err, 1);
}

// Pooled bag split over S row groups (small batches: more loads in flight per bag). Row group
// g = r * S + p sums positions [p * per, (p + 1) * per) of bag r; the S partial sums are added
// in p order through LDS by group p = 0.
template <bool VEC, bool LAZY = false>
__device__ void gather_pool_split(const SegLaunch& a, const rs_feature_seg_t& sg, int s, int lb) {
  constexpr int W = VEC ? 4 : 1;
  __shared__ float4 red[256];
  const int C = a.chunks[s], S = a.split[s];
  const int grp = threadIdx.x / C, chunk = threadIdx.x % C;
  const int r = grp / S, p = grp % S;
  const int row = lb * a.rpb[s] + r;
  const bool active = r < a.rpb[s] && row < a.rows;
  const int per = (sg.bag + S - 1) / S;
  const int lbeg = p * per < sg.bag ? p * per : sg.bag;
  const int lend = lbeg + per < sg.bag ? lbeg + per : sg.bag;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (active) pool_acc<VEC, LAZY>(a, sg, row, chunk * W, lbeg, lend, acc);
  red[threadIdx.x] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  if (!active || p != 0) return;
  for (int q = 1; q < S; ++q) {
    const float4 t = red[threadIdx.x + q * C];
    acc[0] += t.x; acc[1] += t.y; acc[2] += t.z; acc[3] += t.w;
  }
  if (sg.pool_mode == RS_POOL_MEAN) {
    const float n = (float)sg.bag;
#pragma unroll
    for (int j = 0; j < W; ++j) acc[j] = acc[j] / n;
  }
  float* o = a.out + (int64_t)row * a.ldo + sg.out_col + chunk * W;
  store_row<VEC>(o, acc);
}

// The hot rows of a pooled call (seg.hot_keys: its ids sorted by row): sample every kHotQ-th
// sorted position p; p starts the first sample of a run of at least kHotQ keys when key[p] ==
// key[p + kHotQ - 1] and key[p - kHotQ] differs, so every run of >= 2 kHotQ - 1 lookups (and some
// shorter ones) is listed once. Up to kHotMax rows are staged into `rows` (LDS) and entered into an
// open-addressing table id -> slot. Returns the number staged. Which rows make the list (LDS
// atomics) does not change any value: a staged row is a copy of the table row.
struct HotLds {
  int count;
  int ids[kHotMax];
  int tab[kHotHash];
  uint8_t slot[kHotHash];
};

__device__ __forceinline__ int hot_hash(uint32_t id) { return (int)((id * 2654435761u) >> 24); }

__device__ int hot_stage(const rs_feature_seg_t& sg, HotLds& h, float4* rows) {
  if (threadIdx.x == 0) h.count = 0;
  for (int i = threadIdx.x; i < kHotHash; i += 256) h.tab[i] = -1;
  __syncthreads();
  const uint32_t* keys = sg.hot_keys;
  const int64_t n = sg.hot_n;
  for (int64_t p = (int64_t)threadIdx.x * kHotQ; p + kHotQ - 1 < n; p += (int64_t)256 * kHotQ) {
    const uint32_t k = keys[p];
    if (k == 0xFFFFFFFFu || keys[p + kHotQ - 1] != k || (p >= kHotQ && keys[p - kHotQ] == k)) continue;
    const int i = atomicAdd(&h.count, 1);
    if (i < kHotMax) h.ids[i] = (int)k;
  }
  __syncthreads();
  const int cnt = h.count < kHotMax ? h.count : kHotMax;
  if ((int)threadIdx.x < cnt) {
    const int id = h.ids[threadIdx.x];
    int b = hot_hash((uint32_t)id);
    while (atomicCAS(&h.tab[b], -1, id) != -1) b = (b + 1) & (kHotHash - 1);
    h.slot[b] = (uint8_t)threadIdx.x;
  }
  const int q = sg.dim / 4;
  for (int i = threadIdx.x; i < cnt * q; i += 256) {
    const int r = i / q;
    rows[i] = reinterpret_cast<const float4*>(sg.table + (int64_t)h.ids[r] * sg.dim)[i - r * q];
  }
  __syncthreads();
  return cnt;
}

// slot of row id among the staged hot rows, or -1
__device__ __forceinline__ int hot_find(const HotLds& h, int64_t id) {
  int b = hot_hash((uint32_t)id);
  for (;;) {
    const int t = h.tab[b];
    if (t == (int)id) return h.slot[b];
    if (t < 0) return -1;
    b = (b + 1) & (kHotHash - 1);
  }
}

// pool_acc (VEC, plain rows) with the staged hot rows: a lookup of a hot row reads its LDS copy
// through the same flat load (no branch around the load), in the same order -- the same sums
__device__ __forceinline__ void pool_acc_hot(const rs_feature_seg_t& sg, const HotLds& h, int cnt,
                                             const float4* hrows, int row, int c, int lbeg, int lend,
                                             float* acc, bool& bad) {
  constexpr int NB = kBagBatch;
  const int64_t* ids = sg.idx + (int64_t)row * sg.idx_stride;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = 0.f;
  int64_t raw[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) raw[u] = lbeg + u < lend ? ids[lbeg + u] : 0;
  for (int l0 = lbeg; l0 < lend; l0 += NB) {
    const int nb = lend - l0 < NB ? lend - l0 : NB;
    bool ok[NB];
    float v[NB][4];
    int sl[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const bool valid = raw[u] >= 0 && raw[u] < sg.vocab;
      bad |= u < nb && !valid;
      ok[u] = u < nb && valid;
      sl[u] = cnt ? hot_find(h, ok[u] ? raw[u] : 0) : -1;
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int64_t r = ok[u] ? raw[u] : 0;
      const float* src = sl[u] >= 0 ? reinterpret_cast<const float*>(hrows + sl[u] * (sg.dim / 4)) + c
                                    : sg.table + r * sg.dim + c;
      load_row<true>(src, v[u]);
    }
    const int n2 = l0 + NB;
#pragma unroll
    for (int u = 0; u < NB; ++u) raw[u] = n2 + u < lend ? ids[n2 + u] : 0;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = ok[u] ? v[u][j] : 0.f;
        const float y = acc[j] + x;
        acc[j] = u < nb ? y : acc[j];
      }
    }
  }
}

// gather_pool_split over persistent workgroups with the hot rows in LDS: workgroup lb of nblk
// takes row groups lb, lb + nblk, ...
__device__ void gather_pool_hot(const SegLaunch& a, const rs_feature_seg_t& sg, int s, int lb, int nblk,
                                float4* dyn) {
  __shared__ float4 red[256];
  __shared__ HotLds h;
  const int cnt = hot_stage(sg, h, dyn);
  const int C = a.chunks[s], S = a.split[s];
  const int grp = threadIdx.x / C, chunk = threadIdx.x % C;
  const int r = grp / S, p = grp % S;
  const int per = (sg.bag + S - 1) / S;
  const int lbeg = p * per < sg.bag ? p * per : sg.bag;
  const int lend = lbeg + per < sg.bag ? lbeg + per : sg.bag;
  const int ngroups = (a.rows + a.rpb[s] - 1) / a.rpb[s];
  bool bad = false;
  for (int g = lb; g < ngroups; g += nblk) {
    const int row = g * a.rpb[s] + r;
    const bool active = r < a.rpb[s] && row < a.rows;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (active) pool_acc_hot(sg, h, cnt, dyn, row, chunk * 4, lbeg, lend, acc, bad);
    red[threadIdx.x] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (active && p == 0) {
      for (int q = 1; q < S; ++q) {
        const float4 t = red[threadIdx.x + q * C];
        acc[0] += t.x; acc[1] += t.y; acc[2] += t.z; acc[3] += t.w;
      }
      if (sg.pool_mode == RS_POOL_MEAN) {
        const float n = (float)sg.bag;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = acc[j] / n;
      }
      store_row<true>(a.out + (int64_t)row * a.ldo + sg.out_col + chunk * 4, acc);
    }
    __syncthreads();
  }
  if (bad && a.err) atomicOr(a.err, 1);
}

// LAZY launches (rs_gather_fwd_lazy): segments with lazy_last read through the catch-up (float4
// rows, never staged: the plan checks); the others as in a plain launch
template <bool LAZY>
__global__ __launch_bounds__(256) void gather_fwd_kernel(SegLaunch a) {
  extern __shared__ float4 stage_lds[];
  const int s = find_seg(a, blockIdx.x);
  rs_feature_seg_t sg = a.segs[s];
  const int lb = blockIdx.x - a.block_start[s];
  if (LAZY && sg.lazy_last) {  // uniform per workgroup
    if (a.split[s] > 1) {
      if (a.vec[s]) gather_pool_split<true, true>(a, sg, s, lb);
      else gather_pool_split<false, true>(a, sg, s, lb);
      return;
    }
    const int C = a.chunks[s];
    const int r = threadIdx.x / C, chunk = threadIdx.x % C;
    if (r >= a.rpb[s]) return;
    if (a.rpt[s] == kRowsPerLane) {
      gather_sparse_rows<kRowsPerLane, true>(a, sg, a.rpb[s], lb, r, chunk);
      return;
    }
    const int row = lb * a.rpb[s] + r;
    if (row >= a.rows) return;
    if (a.vec[s]) gather_seg<true, true>(a, sg, row, chunk);
    else gather_seg<false, true>(a, sg, row, chunk);
    return;
  }
  if (a.hot[s]) {  // uniform per workgroup: persistent workgroups with the hot rows in LDS
    gather_pool_hot(a, sg, s, lb, a.block_start[s + 1] - a.block_start[s], stage_lds);
    return;
  }
  if (a.stage[s]) {  // uniform per workgroup: the whole table into LDS, then read it from there
    const float4* src = reinterpret_cast<const float4*>(sg.table);
    for (int i = threadIdx.x; i < a.stage[s] / 16; i += 256) stage_lds[i] = src[i];
    __syncthreads();
    sg.table = reinterpret_cast<const float*>(stage_lds);
  }
  if (a.split[s] > 1) {  // uniform per workgroup: the barrier inside is reached by every thread
    if (a.vec[s]) gather_pool_split<true>(a, sg, s, lb);
    else gather_pool_split<false>(a, sg, s, lb);
    return;
  }
  const int C = a.chunks[s];
  const int r = threadIdx.x / C, chunk = threadIdx.x % C;
  if (r >= a.rpb[s]) return;
  if (a.rpt[s] == kRowsPerLane) {  // plan: sparse, vec only
    gather_sparse_rows<kRowsPerLane>(a, sg, a.rpb[s], lb, r, chunk);
    return;
  }
  const int row = lb * a.rpb[s] + r;
  if (row >= a.rows) return;
  if (a.vec[s]) gather_seg<true>(a, sg, row, chunk);
  else gather_seg<false>(a, sg, row, chunk);
}

// LDS_ACC: accumulate into the workgroup-private LDS copy `lds` of the table gradient
// [lbeg, lend): the bag positions this lane scatters (a split bag, see gather_pool_split)
template <bool VEC, bool LDS_ACC = false>
__device__ void scatter_seg(const SegLaunch& a, const rs_feature_seg_t& sg, int row, int chunk,
                            float* lds = nullptr, int lbeg = 0, int lend = -1) {
  constexpr int W = VEC ? 4 : 1;
  const int c = chunk * W;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  load_row<VEC>(a.dout + (int64_t)row * a.ldo + sg.out_col + c, g);
  if (sg.kind == RS_SEG_SPARSE) {
    const int64_t id = sg.idx[(int64_t)row * sg.idx_stride];
    if (id == sg.pad_idx || id < 0 || id >= sg.vocab) return;
    float* d = (LDS_ACC ? lds : sg.grad) + id * sg.dim + c;
    if (!LDS_ACC && sg.touch_count && sg.touch_count[id] == 1) {
      store_row<VEC>(d, g);  // the row's only lookup this step: its gradient row is still zero
      return;
    }
#pragma unroll
    for (int j = 0; j < W; ++j) atomicAdd(d + j, g[j]);
  } else if (sg.kind == RS_SEG_POOL) {
    const int64_t* ids = sg.idx + (int64_t)row * sg.idx_stride;
    if (sg.pool_mode == RS_POOL_MAX) {
      // gradient goes to the (first) arg-max row of each column (torch.max(dim) backward)
      float best[4];
      int64_t arg[4];
#pragma unroll
      for (int j = 0; j < W; ++j) { best[j] = -INFINITY; arg[j] = -1; }
      for (int l = 0; l < sg.bag; ++l) {
        const int64_t id = ids[l];
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (id >= 0 && id < sg.vocab) load_row<VEC>(sg.table + id * sg.dim + c, v);
#pragma unroll
        for (int j = 0; j < W; ++j)
          if (v[j] > best[j] || arg[j] < 0) { best[j] = v[j]; arg[j] = id; }
      }
#pragma unroll
      for (int j = 0; j < W; ++j)
        if (arg[j] >= 0 && arg[j] != sg.pad_idx && arg[j] < sg.vocab)
          atomicAdd((LDS_ACC ? lds : sg.grad) + arg[j] * sg.dim + c + j, g[j]);
      return;
    }
    if (sg.pool_mode == RS_POOL_MEAN) {
      const float n = (float)sg.bag;
#pragma unroll
      for (int j = 0; j < W; ++j) g[j] = g[j] / n;
    }
    // per batch: the touch counts of this batch's rows are loaded together with the next
    // batch's ids, so each batch costs one dependent round trip before its stores/atomics
    if (lend < 0) lend = sg.bag;
    int64_t raw[kBagBatch];
#pragma unroll
    for (int u = 0; u < kBagBatch; ++u) raw[u] = lbeg + u < lend ? ids[lbeg + u] : 0;
    for (int l0 = lbeg; l0 < lend; l0 += kBagBatch) {
      const int nb = lend - l0 < kBagBatch ? lend - l0 : kBagBatch;
      int64_t id[kBagBatch];
      bool use[kBagBatch];
#pragma unroll
      for (int u = 0; u < kBagBatch; ++u) {
        id[u] = raw[u];
        use[u] = u < nb && id[u] != sg.pad_idx && id[u] >= 0 && id[u] < sg.vocab;
      }
      // the touch counts are folded into one bit mask before the first store: otherwise the
      // compiler sinks each load into its branch and waits for them one at a time
      unsigned once = 0;
      if (!LDS_ACC && sg.touch_count) {
        int t[kBagBatch];
#pragma unroll
        for (int u = 0; u < kBagBatch; ++u) t[u] = sg.touch_count[use[u] ? id[u] : 0];
#pragma unroll
        for (int u = 0; u < kBagBatch; ++u) once |= (unsigned)(t[u] == 1) << u;
      }
      const int n2 = l0 + kBagBatch;
#pragma unroll
      for (int u = 0; u < kBagBatch; ++u) raw[u] = n2 + u < lend ? ids[n2 + u] : 0;
#pragma unroll
      for (int u = 0; u < kBagBatch; ++u) {
        if (!use[u]) continue;
        float* d = (LDS_ACC ? lds : sg.grad) + id[u] * sg.dim + c;
        if ((once >> u) & 1u) {
          store_row<VEC>(d, g);
        } else {
#pragma unroll
          for (int j = 0; j < W; ++j) atomicAdd(d + j, g[j]);
        }
      }
    }
  } else if (sg.kind == RS_SEG_LASTVALID) {
    const int64_t l = sg.idx[row];
    float* d = sg.grad + ((int64_t)row * sg.bag + l) * sg.dim + c;
#pragma unroll
    for (int j = 0; j < W; ++j) d[j] += g[j];
  } else {  // RS_SEG_COPY: plain store of the slice gradient
    float* d = sg.grad + (int64_t)row * sg.dim + c;
#pragma unroll
    for (int j = 0; j < W; ++j) d[j] = g[j];
  }
}

__device__ __forceinline__ void gather_bwd_body(const SegLaunch& a, int bid) {
  const int s = find_seg(a, bid);
  const rs_feature_seg_t& sg = a.segs[s];
  if (sg.kind == RS_SEG_DENSE || a.small[s]) return;
  const int lb = bid - a.block_start[s];
  const int C = a.chunks[s], S = a.split[s];
  const int grp = threadIdx.x / C, chunk = threadIdx.x % C;
  const int r = grp / S, p = grp % S;
  if (r >= a.rpb[s]) return;
  const int row = lb * a.rpb[s] + r;
  if (row >= a.rows) return;
  int lbeg = 0, lend = -1;
  if (S > 1) {
    const int per = (sg.bag + S - 1) / S;
    lbeg = p * per < sg.bag ? p * per : sg.bag;
    lend = lbeg + per < sg.bag ? lbeg + per : sg.bag;
  }
  if (a.vec[s]) scatter_seg<true>(a, sg, row, chunk, nullptr, lbeg, lend);
  else scatter_seg<false>(a, sg, row, chunk, nullptr, lbeg, lend);
}

__device__ __forceinline__ void gather_bwd_small_body(const SegLaunch& a, int bid, float* lds) {
  int s = 0;
  while (s + 1 < a.nseg && bid >= a.sblock_start[s + 1]) ++s;
  const rs_feature_seg_t& sg = a.segs[s];
  const int lb = bid - a.sblock_start[s];
  const int nblk = a.sblocks[s];
  const int n = (int)(sg.vocab * sg.dim);
  for (int e = threadIdx.x; e < n; e += 256) lds[e] = 0.f;
  __syncthreads();
  const int C = a.chunks[s];
  const int r = threadIdx.x / C, chunk = threadIdx.x % C;
  if (r < a.rpb[s]) {
    for (int row = lb * a.rpb[s] + r; row < a.rows; row += nblk * a.rpb[s]) {
      if (a.vec[s]) scatter_seg<true, true>(a, sg, row, chunk, lds);
      else scatter_seg<false, true>(a, sg, row, chunk, lds);
    }
  }
  __syncthreads();
  // one global atomic per touched element
  for (int e = threadIdx.x; e < n; e += 256) {
    const float v = lds[e];
    if (v != 0.f) atomicAdd(sg.grad + e, v);
  }
}

// dense segment s (Linear(1, D) of one input column) by one 256-thread workgroup: dW[c] +=
// sum_r dout[r][c] x[r], db[c] += sum_r dout[r][c]; row-lanes with 16 rows' loads in flight, the
// row-lanes of a column summed by wave shuffles and then in wave order (deterministic). red: 512
// floats of LDS
__device__ __forceinline__ void dense_bwd_body(const SegLaunch& a, int s, float* red) {
  const rs_feature_seg_t& sg = a.segs[s];
  const int D = sg.dim;
  const int lanes = 256 / D;  // D <= 256
  const int c = threadIdx.x % D, rl = threadIdx.x / D;
  constexpr int U = 16;
  float aw = 0.f, ab = 0.f;
  if (rl < lanes) {
    int row = rl;
    for (; row + (U - 1) * lanes < a.rows; row += U * lanes) {
      float gv[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        gv[u] = a.dout[(int64_t)(row + u * lanes) * a.ldo + sg.out_col + c];
        xv[u] = sg.x[(int64_t)(row + u * lanes) * sg.idx_stride];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        aw += gv[u] * xv[u];
        ab += gv[u];
      }
    }
    for (; row < a.rows; row += lanes) {
      const float gv = a.dout[(int64_t)row * a.ldo + sg.out_col + c];
      aw += gv * sg.x[(int64_t)row * sg.idx_stride];
      ab += gv;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int np;  // partials per column at red[i * D + c] (weights) and red[256 + i * D + c] (bias)
  if (D < 64 && 64 % D == 0) {
    for (int off = D; off < 64; off <<= 1) {
      aw += __shfl_xor(aw, off, 64);
      ab += __shfl_xor(ab, off, 64);
    }
    if (lane < D) {
      red[w * D + c] = aw;
      red[256 + w * D + c] = ab;
    }
    np = 4;
  } else {
    red[threadIdx.x] = aw;
    red[256 + threadIdx.x] = ab;
    np = lanes;
  }
  __syncthreads();
  if (threadIdx.x < D) {
    float sw = 0.f, sb = 0.f;
    for (int i = 0; i < np; ++i) { sw += red[i * D + c]; sb += red[256 + i * D + c]; }
    sg.grad[c] += sw;
    sg.grad_bias[c] += sb;
  }
}

// the backward's scatter, small-table and dense work in ONE launch (round 5): blocks [0, nsmall)
// the small-table kernel's, then one per dense segment, then the scatter's (C2's user tower: three
// launches on the critical chain, 8.7 + 13.3 + 12.2 us)
__global__ __launch_bounds__(256) void gather_bwd_fused_kernel(SegLaunch a, int nsmall, int ndense) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  int b = blockIdx.x;
  if (b < nsmall) {
    gather_bwd_small_body(a, b, lds);
    return;
  }
  b -= nsmall;
  if (b < ndense) {
    int s = 0, k = 0;
    for (; s < a.nseg; ++s)
      if (a.segs[s].kind == RS_SEG_DENSE && k++ == b) break;
    dense_bwd_body(a, s, lds);
    return;
  }
  gather_bwd_body(a, b - ndense);
}

// Small tables in deterministic mode (rs_set_deterministic; <= 16 KB, or up to 48 KB when the
// ranged kernel cannot take them: C2 / C3's gender, age, occupation, genre, release-year tables,
// and the per-token genre bags of the history: 614,400 bag ids per step into a 30 x 8 table):
// slot-private LDS images, no atomics, bitwise reproducible. A workgroup owns a contiguous run of
// lookup rows; its lanes form `slots` groups of D (lane = slot * D + column) and slot k takes
// rows k, k + slots, ... of the run, adding each bag id's dout column into ITS OWN [V][D] image
// by a plain LDS read-modify-write (no two lanes ever touch one word, so no atomics and one fixed
// order per word). The slot images are then summed in slot order into the workgroup's partial,
// and reduce_partials_kernel adds the workgroup partials in order. Per bag id that is two LDS
// operations per column lane -- the earlier kernels compared every id with every table row
// (register accumulators: V compare-selects per id and column, 46 us at C2's genre table) or
// used LDS / global float atomics (33 us, order-dependent bits).
constexpr int kSlotRows = 8;  // rows per slot per batch: their dout columns and ids load together
constexpr int kSlotBag = 8;   // bags up to this long load all their ids at once

__global__ __launch_bounds__(256) void gather_bwd_slot_kernel(SegLaunch a) {
  extern __shared__ __attribute__((aligned(16))) float img[];  // [slots][V][D]
  int s = 0;
  while (s + 1 < a.nseg && (int)blockIdx.x >= a.tblock_start[s + 1]) ++s;
  const rs_feature_seg_t& sg = a.segs[s];
  const int lb = blockIdx.x - a.tblock_start[s];
  const int nblk = a.tblocks[s], nsl = a.slots[s];
  const int D = sg.dim;
  const int E = (int)(sg.vocab * D);
  for (int e = threadIdx.x; e < nsl * E; e += 256) img[e] = 0.f;
  __syncthreads();
  const int sl = threadIdx.x / D, c = threadIdx.x - sl * D;
  const int per = (a.rows + nblk - 1) / nblk;
  const int r0 = lb * per, r1 = r0 + per < a.rows ? r0 + per : a.rows;
  if (sl < nsl) {
    const bool pool = sg.kind == RS_SEG_POOL;
    const int bag = pool ? sg.bag : 1;
    const float sc = pool && sg.pool_mode == RS_POOL_MEAN ? 1.f / (float)bag : 1.f;
    const int64_t pad = sg.pad_idx, V = sg.vocab;
    float* my = img + sl * E + c;
    for (int r = r0 + sl; r < r1; r += kSlotRows * nsl) {
      float g[kSlotRows];
      int64_t row[kSlotRows];
#pragma unroll
      for (int u = 0; u < kSlotRows; ++u) {
        row[u] = r + u * nsl;
        g[u] = row[u] < r1 ? a.dout[row[u] * a.ldo + sg.out_col + c] * sc : 0.f;
      }
      if (bag <= kSlotBag) {
        // every id of the batch in flight with the dout columns: one round trip per batch
        int id[kSlotRows][kSlotBag];  // table row, or -1 (no contribution)
#pragma unroll
        for (int u = 0; u < kSlotRows; ++u)
#pragma unroll
          for (int l = 0; l < kSlotBag; ++l) {
            const int64_t x = (row[u] < r1 && l < bag) ? sg.idx[row[u] * sg.idx_stride + l] : -1;
            id[u][l] = (x >= 0 && x < V && x != pad) ? (int)x : -1;
          }
#pragma unroll
        for (int u = 0; u < kSlotRows; ++u)
#pragma unroll
          for (int l = 0; l < kSlotBag; ++l)
            if (id[u][l] >= 0) my[id[u][l] * D] += g[u];
      } else {
        for (int l = 0; l < bag; ++l) {
          int64_t id[kSlotRows];
#pragma unroll
          for (int u = 0; u < kSlotRows; ++u) id[u] = row[u] < r1 ? sg.idx[row[u] * sg.idx_stride + l] : -1;
#pragma unroll
          for (int u = 0; u < kSlotRows; ++u)
            if (id[u] >= 0 && id[u] < V && id[u] != pad) my[id[u] * D] += g[u];
        }
      }
    }
  }
  __syncthreads();
  float* dst = a.ws + a.pws_off[s] + (int64_t)lb * E;
  for (int e = threadIdx.x; e < E; e += 256) {
    float t = img[e];
    for (int k = 1; k < nsl; ++k) t += img[k * E + e];
    dst[e] = t;
  }
}

// One-hot MFMA table gradient of tiny, heavily hit tables (round 5; V <= 64 rows, D <= 16 columns,
// >= 65,536 lookups a call): grad[V][D] += sum over lookup rows r of count_r[V] (x) dout[r][D], a [V x rows] x
// [rows x D] product on v_mfma_f32_16x16x4_f32 whose A operand -- the row's bag-id counts, scaled by
// 1 / bag for mean pooling -- is built in registers from the ids: in k-step t, lane (i = l & 15,
// k = l >> 4) holds A[v = 16 m + i][row 4 t + k] = sc * #{ids of the row == v} (four bag
// positions per pass) and B[row 4 t + k][c = i] = dout[row][c]. The per-token genre bags of C2's
// history (204,800 rows x 3 ids into a 30 x 8 table) were 25.7 us of LDS float atomics on 240
// words in the C2 step (gather_bwd_small_kernel), 19.6 here; every row is one MFMA column whatever
// its ids. The towers' tables (4,096 lookups) stay on the atomic kernel (see kOhMinLookups). Each wave sums a contiguous run
// of rows in a fixed order, the 8 waves meet in a fixed LDS order, and the workgroup partials are
// reduced in order (reduce_partials_kernel or the deferred flush): deterministic, in both modes.
constexpr int kOhWaves = 8;   // 512 threads: 256 registers a lane (64 accumulators, 8 k-steps of ids)
constexpr int kOhSteps = 8;   // k-steps (4 rows each) per batch: 32 rows' loads in flight per wave
constexpr int kOhMaxM = 4;    // M tiles: V <= 64 (the MFMA chains grow with the tiles: at C2's
                              // 152-row year table, 16 tiles, the atomic kernel was 2x faster)
constexpr int kOhMaxE = 1024; // V x D: 4 LDS slices of 4 KB
constexpr int64_t kOhMinLookups = 65536;  // below: the atomic kernel (one 4,096-row batch of the
                                          // towers' tables: 12 us atomic, 16 us one-hot incl. launch)

// MT: M tiles computed for every segment of the launch (the largest segment's, rounded up to a
// power of two): tiles past a table's rows only ever add zeros, and no per-tile branch breaks the
// MFMA chains
template <int MT>
__global__ __launch_bounds__(kOhWaves * 64) void gather_bwd_onehot_kernel(SegLaunch a) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][V * D]
  int s = 0;
  while (s + 1 < a.nseg && (int)blockIdx.x >= a.oblock_start[s + 1]) ++s;
  const rs_feature_seg_t& sg = a.segs[s];
  const int lb = blockIdx.x - a.oblock_start[s];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = lane & 15, k = lane >> 4;
  const int D = sg.dim;
  const int V = (int)sg.vocab;
  const int E = V * D;
  const bool pool = sg.kind == RS_SEG_POOL;
  const int bag = pool ? sg.bag : 1;
  const float sc = pool && sg.pool_mode == RS_POOL_MEAN ? 1.f / (float)bag : 1.f;
  const int64_t pad = sg.pad_idx;
  const int64_t rpw = a.oh_rpw[s];
  const int64_t r0 = ((int64_t)lb * kOhWaves + w) * rpw;
  const int64_t r1 = r0 + rpw < (int64_t)a.rows ? r0 + rpw : (int64_t)a.rows;
  f4v acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f4v{0.f, 0.f, 0.f, 0.f};
  for (int64_t rb = r0; rb < r1; rb += 4 * kOhSteps) {
    float bv[kOhSteps];
    int64_t row[kOhSteps];
#pragma unroll
    for (int t = 0; t < kOhSteps; ++t) {
      row[t] = rb + 4 * t + k;
      bv[t] = (row[t] < r1 && i < D) ? a.dout[row[t] * a.ldo + sg.out_col + i] : 0.f;
    }
    for (int l0 = 0; l0 < bag; l0 += 4) {
      int id[kOhSteps][4];  // table row, or -1 (no contribution)
#pragma unroll
      for (int t = 0; t < kOhSteps; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t x = (row[t] < r1 && l0 + u < bag) ? sg.idx[row[t] * sg.idx_stride + l0 + u] : -1;
          id[t][u] = (x >= 0 && x < V && x != pad) ? (int)x : -1;
        }
#pragma unroll
      for (int t = 0; t < kOhSteps; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int v = 16 * m + i;
          const float cnt = (float)((id[t][0] == v) + (id[t][1] == v) + (id[t][2] == v) + (id[t][3] == v));
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(cnt * sc, bv[t], acc[m], 0, 0, 0);
        }
    }
  }
  // acc[m][j]: table row v = 16 m + 4 k + j, column c = i. Waves 4..7 hand theirs to waves 0..3,
  // then each element is the fixed-order sum of the 4 slices
  const int c = i;
  if (w >= 4) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int v = 16 * m + 4 * k + j;
        if (v < V && c < D) red[(w - 4) * E + v * D + c] = acc[m][j];
      }
    }
  }
  __syncthreads();
  if (w < 4) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int v = 16 * m + 4 * k + j;
        if (v < V && c < D) {
          float* r = red + w * E + v * D + c;
          *r = acc[m][j] + *r;
        }
      }
    }
  }
  __syncthreads();
  float* dst = a.ws + a.pws_off[s] + (int64_t)lb * E;
  for (int e = threadIdx.x; e < E; e += kOhWaves * 64) {
    float t = red[e];
#pragma unroll
    for (int q = 1; q < 4; ++q) t += red[q * E + e];
    dst[e] = t;
  }
}

// LDS-image table gradient of hot mid-size tables: no atomics, deterministic. C2's 3,500 x 32
// hist_movie_ids table gets 204,800 token lookups per step (~58 per row); the atomic scatter
// serialises on the hot rows' L2 lines (90 us per step). A workgroup owns one RANGE of table rows
// (rrows[s] rows = 64 KB of LDS) x one CHUNK of the lookups:
//  1. the chunk's ids are staged into LDS 8,192 at a time as int16 local rows (-1 outside the
//     range or padding);
//  2. wave w owns the rows with local row % 16 == w: it scans the staged ids (8 per lane per LDS
//     read) in a fixed order and queues its hits (ballot + mbcnt);
//  3. D/4 lanes per queued lookup read its dout row (float4 slices, 4 steps of G = 64 / (D/4)
//     lookups in flight) and add it into the image by plain LDS read-modify-write: a row belongs
//     to one wave, and lookups of the same row inside one step are applied one group at a time in
//     queue order, so every row is summed in the same order every time;
//  4. the image is written whole to ws[chunk] and reduce_partials_kernel adds the chunks in order.
// Every dout row is read once and the gradient is bitwise reproducible. LDS float atomics were
// measured first (the same plan with ds_add_f32): ~0.5 lane-adds per clock per CU whatever the bank
// pattern, 61 us at C2's shape. Block order is XCD-aware: the ranges of one chunk (which read the
// same ids) share an XCD.
constexpr int kRangeBytes = 64 * 1024;
constexpr int kRangeThreads = 1024;
constexpr int kRangeWaves = kRangeThreads / 64;
constexpr int kRangeIds = 8192;    // ids staged per pass (LDS, int16 local rows)
constexpr int kRangeQueue = 1024;  // per-wave queue entries

__device__ __forceinline__ int64_t lookup_id(const rs_feature_seg_t& sg, int64_t e) {
  if (sg.kind == RS_SEG_POOL) {
    const int64_t r = e / sg.bag;
    return sg.idx[r * sg.idx_stride + (e - r * sg.bag)];
  }
  return sg.idx[e * sg.idx_stride];
}

__device__ __forceinline__ void range_rmw(float* lds, int loc, int D, int c4, float4 v, float scale) {
  float4* d = reinterpret_cast<float4*>(lds + loc * D + c4);
  float4 x = *d;
  x.x += v.x * scale; x.y += v.y * scale; x.z += v.z * scale; x.w += v.w * scale;
  *d = x;
}

__global__ __launch_bounds__(kRangeThreads) void gather_bwd_range_kernel(SegLaunch a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // the range image [R][D]
  __shared__ __attribute__((aligned(16))) short sid[kRangeIds];
  __shared__ int queue[kRangeWaves][kRangeQueue];
  int s = 0;
  while (s + 1 < a.nseg && (int)blockIdx.x >= a.rblock_start[s + 1]) ++s;
  const rs_feature_seg_t& sg = a.segs[s];
  const int lb = blockIdx.x - a.rblock_start[s];
  const int nr = a.rranges[s], nch = a.rchunks[s];
  // lb -> (range, chunk): xcd = lb % 8 is the chunk's residue, so the ranges of a chunk share it
  const int xcd = lb & 7, slot = lb >> 3;
  const int range = slot % nr, chunk = (slot / nr) * 8 + xcd;
  const int R = a.rrows[s], D = sg.dim;
  const int64_t v0 = (int64_t)range * R;
  const int nrow = (int)(sg.vocab - v0 < R ? sg.vocab - v0 : R);
  const int nel = nrow * D;  // a multiple of 4
  for (int i = threadIdx.x * 4; i < nel; i += 4 * kRangeThreads)
    *reinterpret_cast<float4*>(lds + i) = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t n = (int64_t)a.rows * (sg.kind == RS_SEG_POOL ? sg.bag : 1);
  const int64_t per = (n + nch - 1) / nch;
  const int64_t e0 = (int64_t)chunk * per, e1 = e0 + per < n ? e0 + per : n;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int C = D / 4, G = 64 / C;  // lanes per lookup (a float4 of columns each), lookups per step
  const int g = lane / C, c4 = (lane % C) * 4;
  const float scale = sg.kind == RS_SEG_POOL && sg.pool_mode == RS_POOL_MEAN ? 1.f / (float)sg.bag : 1.f;
  const int bag = sg.kind == RS_SEG_POOL ? sg.bag : 1;
  const int64_t pad = sg.pad_idx;
  int* q = queue[w];
  for (int64_t p0 = e0; p0 < e1; p0 += kRangeIds) {
    const int np = (int)(e1 - p0 < kRangeIds ? e1 - p0 : kRangeIds);
    __syncthreads();  // the image is zeroed / the previous pass's scans are done with sid
#pragma unroll
    for (int u = 0; u < kRangeIds / kRangeThreads; ++u) {
      const int i = u * kRangeThreads + threadIdx.x;
      const int64_t id = i < np ? lookup_id(sg, p0 + i) : -1;
      const int64_t loc = id - v0;
      sid[i] = (short)((i < np && loc >= 0 && loc < nrow && id != pad) ? (int)loc : -1);
    }
    __syncthreads();
    int nq = 0;
    // 8 staged ids per lane per LDS read (ids b + 8 lane + u): the queue order is fixed, so each
    // row's lookups are always summed in the same order
    for (int b = 0; b < np; b += 512) {
      const int4 raw = *reinterpret_cast<const int4*>(&sid[b + 8 * lane]);  // sid is -1 past np
      const int packed[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int loc = (int)(short)(packed[u >> 1] >> (16 * (u & 1)));
        const bool hit = loc >= 0 && (loc & (kRangeWaves - 1)) == w;
        const uint64_t m = __ballot(hit);
        const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (hit) q[nq + pos] = ((b + 8 * lane + u) << 14) | loc;  // i < 8192, loc < 16384
        nq += __popcll(m);
      }
      if (nq <= kRangeQueue - 512 && b + 512 < np) continue;  // wave-uniform
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      for (int j = 0; j < nq; j += 4 * G) {
        float4 v[4];
        int lk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int qi = j + k * G + g;
          const bool ok = qi < nq;
          const int ent = q[ok ? qi : 0];
          lk[k] = ok ? (ent & 0x3fff) : -1;
          const int64_t row = (p0 + (ent >> 14)) / bag;
          v[k] = *reinterpret_cast<const float4*>(a.dout + (ok ? row : 0) * a.ldo + sg.out_col + c4);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          // another group earlier in this step on the same row: apply the step group by group
          bool dup = false;
          for (int gg = 0; gg < G; ++gg) {
            const int o = __shfl(lk[k], gg * C);
            dup |= gg < g && o == lk[k] && o >= 0;
          }
          if (__ballot(dup) == 0) {
            if (lk[k] >= 0) range_rmw(lds, lk[k], D, c4, v[k], scale);
          } else {
            for (int gg = 0; gg < G; ++gg) {
              if (g == gg && lk[k] >= 0) range_rmw(lds, lk[k], D, c4, v[k], scale);
              __builtin_amdgcn_wave_barrier();
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      nq = 0;
    }
  }
  __syncthreads();
  float* dst = a.ws + a.pws_off[s] + (int64_t)chunk * sg.vocab * D + v0 * D;
  for (int i = threadIdx.x * 4; i < nel; i += 4 * kRangeThreads)
    *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(lds + i);
}

// grad[e] += sum of the partials ws[k][e] over k (small and ranged tables), in a fixed order:
// a 1024-thread workgroup takes 64 float4 elements of every partial segment; wave w sums the
// partials k = w, w + 16, ... in k order, the 16 wave sums are added in wave order through LDS.
constexpr int kReduceWaves = 16;
__global__ __launch_bounds__(kReduceWaves * 64) void reduce_partials_kernel(SegLaunch a) {
  __shared__ float4 red[kReduceWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int s = 0; s < a.nseg; ++s) {
    const int nch = a.pchunks[s];
    if (!nch) continue;
    const rs_feature_seg_t& sg = a.segs[s];
    const int64_t n = sg.vocab * sg.dim;
    const int64_t n4 = n / 4;
    const float* src = a.ws + a.pws_off[s];
    const bool v4 = (n & 3) == 0;
    const int64_t nel = v4 ? n4 : n;  // float4 elements (scalar when vocab * dim % 4 != 0)
    for (int64_t base = (int64_t)blockIdx.x * 64; base < nel; base += (int64_t)gridDim.x * 64) {
      const int64_t i = base + lane;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < nel) {
        for (int k0 = w; k0 < nch; k0 += 8 * kReduceWaves) {
          float4 t[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int k = k0 + u * kReduceWaves;
            if (k >= nch) { t[u] = make_float4(0.f, 0.f, 0.f, 0.f); continue; }
            if (v4) t[u] = reinterpret_cast<const float4*>(src + (int64_t)k * n)[i];
            else t[u] = make_float4(src[(int64_t)k * n + i], 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            acc.x += t[u].x; acc.y += t[u].y; acc.z += t[u].z; acc.w += t[u].w;
          }
        }
      }
      red[w][lane] = acc;
      __syncthreads();
      if (w == 0 && i < nel) {
        float4 r = red[0][lane];
        for (int q = 1; q < kReduceWaves; ++q) {
          const float4 t = red[q][lane];
          r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
        }
        if (v4) {
          float4* g = reinterpret_cast<float4*>(sg.grad) + i;
          float4 o = *g;
          o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
          *g = o;
        } else {
          sg.grad[i] += r.x;
        }
      }
      __syncthreads();
    }
  }
}

// Ranged table-gradient plan of one segment (0 ranges: the atomic scatter). Sparse ids and sum /
// mean bags of a table of 48 KB - 4 MB (smaller ones: the slot kernel), D in {16, 32, 64, 128,
// 256} (D/4 lanes per lookup divide a wave into <= 16 groups); ranges of 64 KB; chunks of >= 2 x
// vocab lookups (the [vocab, dim] partial of a chunk costs no more than its dout rows), a multiple
// of 8 (XCD mapping), at most 1024 / ranges. Deterministic mode (round 4) also takes the tables hit
// < 8 times per row (C2's 6,060-row user and 3,500-row item tables at 4,096 lookups) and the
// small ones the slot kernel leaves to it: measured at C2 (tools/gather_bwd_time.py) the user
// tower's table gradients 25 -> 53-65 us, so the atomic scatter stays the default for them.
struct RangePlan { int rows, ranges, chunks; };

RangePlan range_plan(const rs_feature_seg_t& g, int rows, bool vec) {
  RangePlan r{0, 0, 0};
  const bool table_kind = g.kind == RS_SEG_SPARSE || (g.kind == RS_SEG_POOL && g.pool_mode != RS_POOL_MAX);
  const bool dim_ok = g.dim >= 16 && g.dim <= 256 && 256 % g.dim == 0;
  const int64_t tbytes = g.vocab * g.dim * 4;
  const int64_t n = (int64_t)rows * (g.kind == RS_SEG_POOL ? g.bag : 1);
  // default: tables hit >= 8 times per row on average (the atomic scatter is faster below that);
  // deterministic mode: every table of 4 MB or less that the kernel takes, small ones included
  const bool det = deterministic();
  if (!table_kind || !vec || !dim_ok || (tbytes <= kSmallTableBytes && !det) || tbytes > (4 << 20) || n == 0 ||
      (n < 8 * g.vocab && !det) || getenv_flag("RSYS_NO_RANGE_GRAD"))
    return r;
  int R = kRangeBytes / (g.dim * 4);
  const int nr = (int)((g.vocab + R - 1) / R);
  R = (int)((g.vocab + nr - 1) / nr);  // balanced ranges
  int nch = (int)(n / (2 * g.vocab)) / 8 * 8;
  const int one_pass = (cdiv(n, kRangeIds) + 7) / 8 * 8;  // every chunk staged in one pass
  if (nch < one_pass) nch = one_pass;
  const int cap = (1024 / nr) / 8 * 8;
  if (nch > cap) nch = cap;
  if (nch < 8) nch = 8;
  r.rows = R;
  r.ranges = nr;
  r.chunks = nch;
  return r;
}

int plan(SegLaunch& a, const rs_feature_seg_t* segs_host, int nseg, int rows, int ldo,
         const float* out_ptr_for_align, bool bwd = false) {
  RS_CHECK_ARG(nseg >= 1 && nseg <= kMaxSeg, "gather: nseg %d out of [1,%d]", nseg, kMaxSeg);
  int blocks = 0;
  a.stage_lds = 0;
  for (int s = 0; s < nseg; ++s) {
    const rs_feature_seg_t& g = segs_host[s];
    RS_CHECK_ARG(g.dim >= 1 && g.dim <= 1024, "gather: seg %d dim %d", s, g.dim);
    RS_CHECK_ARG(g.out_col >= 0 && g.out_col + g.dim <= ldo, "gather: seg %d columns exceed ldo", s);
    RS_CHECK_ARG(g.kind >= 0 && g.kind <= 4, "gather: seg %d bad kind %d", s, g.kind);
    RS_CHECK_ARG(g.kind != RS_SEG_POOL || g.bag >= 1, "gather: seg %d empty bag", s);
    RS_CHECK_ARG(g.kind != RS_SEG_DENSE || g.dim <= 256, "gather: dense seg %d dim > 256", s);
    bool vec = (g.dim % 4 == 0) && (g.out_col % 4 == 0) && (ldo % 4 == 0) &&
               aligned16(out_ptr_for_align) && aligned16(g.table) && g.kind != RS_SEG_DENSE;
    int C = vec ? g.dim / 4 : g.dim;
    if (C > 256) { vec = false; C = g.dim; }
    RS_CHECK_ARG(C <= 256, "gather: seg %d too wide", s);
    a.vec[s] = vec;
    a.chunks[s] = C;
    const bool table_kind = g.kind == RS_SEG_SPARSE || g.kind == RS_SEG_POOL;
    // small tables: the float-atomic small-table kernel by default; deterministic mode
    // (rs_set_deterministic): the slot-image kernel where >= 4 slots fit (images <= 16 KB), the
    // ranged kernel for the larger ones it takes (D >= 16, float4 rows: C2 / C3's zip table),
    // else slots anyway. A max-pooled table (its arg-max needs the table rows) keeps the atomics.
    const bool det = bwd && deterministic();
    const int64_t tb = g.vocab * g.dim * 4;
    const bool rangeable = vec && g.dim >= 16 && g.dim <= 256 && 256 % g.dim == 0;
    // tiny tables (both modes): the one-hot MFMA kernel (RSYS_NO_ONEHOT_GRAD=1: the kernels below)
    a.oh[s] = bwd && table_kind && !(g.kind == RS_SEG_POOL && g.pool_mode == RS_POOL_MAX) && g.vocab <= 16 * kOhMaxM &&
              g.dim <= 16 && g.vocab * g.dim <= kOhMaxE &&
              (int64_t)rows * (g.kind == RS_SEG_POOL ? g.bag : 1) >= kOhMinLookups && !getenv_flag("RSYS_NO_ONEHOT_GRAD");
    a.tiny[s] = det && table_kind && !(g.kind == RS_SEG_POOL && g.pool_mode == RS_POOL_MAX) && !a.oh[s] &&
               tb <= kSmallTableBytes && g.dim <= 64 && (tb <= 16 * 1024 || !rangeable);
    a.small[s] = bwd && table_kind && tb <= kSmallTableBytes && !a.tiny[s] && !a.oh[s] && !(det && rangeable &&
               !(g.kind == RS_SEG_POOL && g.pool_mode == RS_POOL_MAX));
    // Split long sum/mean bags over S row groups while the launch is short of ~8 waves per SIMD
    // and every group keeps >= 8 positions (C3: B = 4096, L = 50, D = 128 -> S = 4).
    int S = 1;
    // (round 5 measured non-temporal row loads for large tables slower in the step, C3 fp32 0.037
    // -> 0.043 ms: the catch-up has just brought the rows on chip)
    if (g.kind == RS_SEG_POOL && g.pool_mode != RS_POOL_MAX && !a.small[s]) {
      while (2 * S * C <= 256 && (g.bag + 2 * S - 1) / (2 * S) >= 8 &&
             (int64_t)rows * C * S < 8192 * 64)
        S *= 2;
    }
    a.split[s] = S;
    // token-sized sparse forward launches: kRowsPerLane rows per lane (>= 2048 workgroups otherwise)
    a.rpt[s] = (!bwd && vec && g.kind == RS_SEG_SPARSE && (int64_t)rows * C >= (int64_t)2048 * 256)
                   ? kRowsPerLane : 1;
    a.rpb[s] = 256 / (C * S);
    a.hot[s] = !bwd && vec && g.kind == RS_SEG_POOL && g.pool_mode != RS_POOL_MAX && g.hot_keys &&
               g.hot_n >= 2 * kHotQ && !g.lazy_last && g.dim <= 256 && getenv_flag("RSYS_HOT_ROWS");
    if (a.hot[s]) {
      const int hb = kHotMax * g.dim * 4;
      if (hb > a.stage_lds) a.stage_lds = hb;
    }
    a.stage[s] = 0;
    if (!bwd && table_kind && vec && !a.hot[s]) {
      const int64_t tbytes = g.vocab * g.dim * 4;
      const int64_t read = (int64_t)a.rpb[s] * (g.kind == RS_SEG_POOL ? g.bag : 1) * g.dim * 4;
      if (tbytes <= kStageBytes && tbytes <= read && !g.lazy_last && !getenv_flag("RSYS_NO_LDS_STAGE")) {
        a.stage[s] = (int)tbytes;
        if (a.stage[s] > a.stage_lds) a.stage_lds = a.stage[s];
      }
    }
    a.rranges[s] = 0;
    a.rchunks[s] = 0;
    a.rrows[s] = 0;
    if (bwd && !a.small[s] && !a.tiny[s] && !a.oh[s]) {
      const RangePlan rp = range_plan(g, rows, vec);
      a.rrows[s] = rp.rows;
      a.rranges[s] = rp.ranges;
      a.rchunks[s] = rp.chunks;
    }
    a.block_start[s] = blocks;
    if (a.hot[s]) {
      const int ng = cdiv(rows, a.rpb[s]);
      blocks += ng < kHotBlocks ? ng : kHotBlocks;
    } else if (!a.small[s] && !a.rranges[s] && !a.tiny[s] && !a.oh[s] && !(bwd && g.kind == RS_SEG_DENSE)) {
      blocks += cdiv(rows, a.rpb[s] * a.rpt[s]);
    }
  }
  a.block_start[nseg] = blocks;
  int rb = 0;
  a.range_lds = 0;
  for (int s = 0; s < nseg; ++s) {
    a.rblock_start[s] = rb;
    if (a.rranges[s]) {
      rb += a.rranges[s] * a.rchunks[s];
      const int bytes = a.rrows[s] * segs_host[s].dim * 4;
      if (bytes > a.range_lds) a.range_lds = bytes;
    }
  }
  a.rblock_start[nseg] = rb;
  int ob = 0;
  a.slot_lds = 0;
  for (int s = 0; s < nseg; ++s) {
    a.tblock_start[s] = ob;
    a.tblocks[s] = 0;
    a.slots[s] = 0;
    if (a.tiny[s]) {
      // slots: as many D-lane groups as a workgroup holds, within 64 KB of images; workgroups:
      // >= kSlotRowsInFlight rows per slot, <= 256, and <= 4 MB of partials in all
      const int64_t E = segs_host[s].vocab * segs_host[s].dim;
      int nsl = 256 / segs_host[s].dim;
      const int fit = (int)((64 * 1024) / (E * 4));
      nsl = nsl < fit ? nsl : fit;
      nsl = nsl < 1 ? 1 : nsl;
      // one batch of kSlotRows rows per slot where the grid allows (<= 2048 workgroups, <= 8 MB
      // of partials): the kernel is a single round trip of loads per workgroup
      int64_t nb = cdiv(rows, nsl * kSlotRows);
      const int64_t cap = std::max<int64_t>(8, (8ll << 20) / (E * 4));
      nb = std::min<int64_t>(std::min<int64_t>(nb, 2048), cap);
      a.slots[s] = (int16_t)nsl;
      a.tblocks[s] = (int16_t)(nb < 1 ? 1 : nb);
      ob += a.tblocks[s];
      a.slot_lds = std::max<int>(a.slot_lds, (int)(nsl * E * 4));
    }
  }
  a.tblock_start[nseg] = ob;
  // one-hot tables: workgroups of 8 waves, each wave a run of whole 32-row batches (C2's
  // genre tokens: 200 workgroups of 4 batches a wave, 26.2 us a call against 27.3 at 400 x 2 and
  // 35.0 at 800 x 1 -- the partials and workgroup launches cost more than the batch round trips)
  int hb = 0;
  a.oh_lds = 0;
  for (int s = 0; s < nseg; ++s) {
    a.oblock_start[s] = hb;
    a.oh_rpw[s] = 0;
    if (!a.oh[s]) continue;
    const int64_t per_wave_min = 4 * kOhSteps;
    // <= 128 rows (4 batches) a wave once the grid is past 256 workgroups (C5's 819,200 history
    // tokens: 800 workgroups rather than 13 serial batches a wave)
    int64_t nb = std::max<int64_t>(std::min<int64_t>(256, cdiv(rows, kOhWaves * per_wave_min)),
                                   std::min<int64_t>(1024, cdiv(rows, kOhWaves * 128)));
    nb = std::max<int64_t>(1, nb);
    int64_t rpw = cdiv(cdiv(rows, nb * kOhWaves), per_wave_min) * per_wave_min;
    nb = std::max<int64_t>(1, cdiv(rows, rpw * kOhWaves));
    a.oh_rpw[s] = (int)rpw;
    a.tblocks[s] = (int16_t)nb;  // the partial count (pchunks)
    hb += (int)nb;
    a.oh_lds = std::max<int>(a.oh_lds, (int)(4 * segs_host[s].vocab * segs_host[s].dim * 4));
  }
  a.oblock_start[nseg] = hb;
  a.ws = nullptr;

  int sb = 0;
  a.small_lds = 0;
  for (int s = 0; s < nseg; ++s) {
    a.sblock_start[s] = sb;
    a.sblocks[s] = 0;
    if (a.small[s]) {
      const int64_t work = (int64_t)rows * (segs_host[s].kind == RS_SEG_POOL ? segs_host[s].bag : 1);
      // ~256 lookups per workgroup: enough workgroups that the LDS accumulation is not one
      // long serial chain; each flushes only its non-zero table entries
      int nb = (int)(work / 256);
      nb = nb < 1 ? 1 : (nb > 512 ? 512 : nb);
      const int maxnb = cdiv(rows, a.rpb[s]);
      a.sblocks[s] = nb < maxnb ? nb : maxnb;
      sb += a.sblocks[s];
      const int bytes = (int)(segs_host[s].vocab * segs_host[s].dim * 4);
      if (bytes > a.small_lds) a.small_lds = bytes;
    }
  }
  a.sblock_start[nseg] = sb;
  int64_t off = 0;
  for (int s = 0; s < nseg; ++s) {
    a.pchunks[s] = a.rranges[s] ? a.rchunks[s] : ((a.tiny[s] || a.oh[s]) ? a.tblocks[s] : 0);
    a.pws_off[s] = off;
    off += (int64_t)a.pchunks[s] * segs_host[s].vocab * segs_host[s].dim;
    off = (off + 3) / 4 * 4;  // float4-aligned partials
  }
  a.ws_floats = off;
  a.nseg = nseg;
  a.rows = rows;
  a.ldo = ldo;
  return 0;
}

// one wave per sequence row: lane l tests position c0 + l, the valid count is a ballot popcount
// (one thread per row looping over L positions was a serial latency chain: 18.6 us at B = 4096)
__global__ __launch_bounds__(256) void seq_mask_kernel(const int64_t* __restrict__ seq, int64_t ld,
                                                       int B, int L, int64_t pad,
                                                       uint8_t* __restrict__ key_pad,
                                                       int64_t* __restrict__ last) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  int valid = 0;
  for (int c0 = 0; c0 < L; c0 += 64) {
    const int l = c0 + lane;
    const bool in = l < L;
    const bool m = in && seq[(int64_t)b * ld + l] == pad;
    valid += __popcll(__ballot(in && !m));
    if (in) key_pad[(int64_t)b * L + l] = m ? 1 : 0;
  }
  if (valid == 0 && lane == (L - 1) % 64) key_pad[(int64_t)b * L + L - 1] = 0;  // all padding: unmask the last position (T6), same thread as the store above
  if (lane == 0) last[b] = valid - 1 > 0 ? valid - 1 : 0;  // clamp(sum(valid) - 1, 0)  (T7)
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_gather_fwd(const rs_feature_seg_t* segs, int nseg, int rows, float* out, int ldo,
                             int* err_flag, void* stream) {
  RS_CHECK_ARG(segs && out, "rs_gather_fwd: null pointer");
  const rs_feature_seg_t* segs_host = segs;
  if (rows == 0) return 0;
  SegLaunch a;
  RS_RET_IF(plan(a, segs_host, nseg, rows, ldo, out));
  for (int i = 0; i < nseg; ++i) a.segs[i] = segs[i];
  a.out = out; a.dout = nullptr; a.err = err_flag;
  gather_fwd_kernel<false><<<a.block_start[nseg], 256, a.stage_lds, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_gather_fwd");
  return 0;
}

extern "C" int rs_gather_fwd_lazy(const rs_feature_seg_t* segs, int nseg, int rows, float* out, int ldo,
                                  int* err_flag, int64_t m_off, int64_t v_off, const int64_t* step,
                                  const float* consts, float beta1, float beta2, float eps, float weight_decay,
                                  void* stream) {
  RS_CHECK_ARG(segs && out && step && consts, "rs_gather_fwd_lazy: null pointer");
  if (rows == 0) return 0;
  SegLaunch a;
  RS_RET_IF(plan(a, segs, nseg, rows, ldo, out));
  for (int i = 0; i < nseg; ++i) {
    const rs_feature_seg_t& g = segs[i];
    if (!g.lazy_last) continue;
    RS_CHECK_ARG(g.kind == RS_SEG_SPARSE || (g.kind == RS_SEG_POOL && g.pool_mode != RS_POOL_MAX),
                 "rs_gather_fwd_lazy: seg %d: read-through needs a sparse or sum / mean pooled lookup", i);
    RS_CHECK_ARG(!a.stage[i], "rs_gather_fwd_lazy: seg %d: a read-through table cannot be staged", i);
  }
  for (int i = 0; i < nseg; ++i) a.segs[i] = segs[i];
  a.out = out; a.dout = nullptr; a.err = err_flag;
  a.lz.moff = m_off; a.lz.voff = v_off; a.lz.step = step;
  a.lz.consts = reinterpret_cast<const float2*>(consts);
  a.lz.h.one_m_b1 = 1.f - beta1; a.lz.h.b2 = beta2; a.lz.h.one_m_b2 = 1.f - beta2;
  a.lz.h.eps = eps; a.lz.h.wd = weight_decay;
  gather_fwd_kernel<true><<<a.block_start[nseg], 256, a.stage_lds, as_stream(stream)>>>(a);
  RS_CHECK_LAUNCH("rs_gather_fwd_lazy");
  return 0;
}

// rs_gather_bwd's workspace: the small and ranged tables' partials. Planned with float4-aligned
// dout rows (the condition under which a segment is ranged at all): an upper bound.
extern "C" int rs_set_deterministic(int on) {
  return g_deterministic.exchange(on ? 1 : 0);
}

extern "C" int64_t rs_gather_ws_bytes(const rs_feature_seg_t* segs_host, int nseg, int rows) {
  if (!segs_host || nseg < 1 || nseg > kMaxSeg || rows <= 0) return 0;
  int ldo = 4;
  for (int s = 0; s < nseg; ++s) ldo = std::max(ldo, segs_host[s].out_col + segs_host[s].dim);
  ldo = (ldo + 3) / 4 * 4;
  SegLaunch a;
  alignas(16) static const float dummy[4] = {0.f, 0.f, 0.f, 0.f};
  if (plan(a, segs_host, nseg, rows, ldo, dummy, true) != 0) return 0;
  return a.ws_floats * 4;
}

extern "C" int rs_gather_bwd(const rs_feature_seg_t* segs, int nseg, int rows, const float* dout,
                             int ldo, float* ws, void* stream) {
  RS_CHECK_ARG(segs && dout, "rs_gather_bwd: null pointer");
  const rs_feature_seg_t* segs_host = segs;
  if (rows == 0) return 0;
  SegLaunch a;
  RS_RET_IF(plan(a, segs_host, nseg, rows, ldo, dout, true));
  for (int s = 0; s < nseg; ++s) {
    const rs_feature_seg_t& g = segs_host[s];
    RS_CHECK_ARG(g.grad, "rs_gather_bwd: seg %d has no grad destination", s);
    RS_CHECK_ARG(g.kind != RS_SEG_DENSE || g.grad_bias, "rs_gather_bwd: seg %d has no bias grad", s);
  }
  for (int i = 0; i < nseg; ++i) a.segs[i] = segs[i];
  a.out = nullptr; a.dout = dout; a.err = nullptr;
  a.ws = ws;
  RS_CHECK_ARG(ws || a.ws_floats == 0,
               "rs_gather_bwd: small / ranged table gradients need ws (rs_gather_ws_bytes)");
  hipStream_t st = as_stream(stream);
  int ndense = 0;
  for (int s = 0; s < nseg; ++s) ndense += segs_host[s].kind == RS_SEG_DENSE;
  if (a.block_start[nseg] + a.sblock_start[nseg] + ndense > 0) {
    gather_bwd_fused_kernel<<<a.sblock_start[nseg] + ndense + a.block_start[nseg], 256,
                              std::max(a.small_lds, 512 * 4), st>>>(a, a.sblock_start[nseg], ndense);
    RS_CHECK_LAUNCH("rs_gather_bwd");
  }
  if (a.rblock_start[nseg] > 0) {
    gather_bwd_range_kernel<<<a.rblock_start[nseg], kRangeThreads, a.range_lds, st>>>(a);
    RS_CHECK_LAUNCH("rs_gather_bwd range");
  }
  if (a.tblock_start[nseg] > 0) {
    gather_bwd_slot_kernel<<<a.tblock_start[nseg], 256, a.slot_lds, st>>>(a);
    RS_CHECK_LAUNCH("rs_gather_bwd slot");
  }
  if (a.oblock_start[nseg] > 0) {
    int mt = 1;
    for (int s = 0; s < nseg; ++s)
      while (a.oh[s] && 16 * mt < segs_host[s].vocab) mt *= 2;
    const int nb = a.oblock_start[nseg];
    switch (mt) {
      case 1: gather_bwd_onehot_kernel<1><<<nb, kOhWaves * 64, a.oh_lds, st>>>(a); break;
      case 2: gather_bwd_onehot_kernel<2><<<nb, kOhWaves * 64, a.oh_lds, st>>>(a); break;
      default: gather_bwd_onehot_kernel<4><<<nb, kOhWaves * 64, a.oh_lds, st>>>(a); break;
    }
    RS_CHECK_LAUNCH("rs_gather_bwd onehot");
  }
  if (a.ws_floats > 0 && reduce_deferring()) {
    // queued for rs_reduce_flush (reduce.hip): the same per-element order as reduce_partials_kernel
    // (16 strided lanes over the chunks, then lanes 0..15), grad += the sum
    for (int s = 0; s < nseg; ++s) {
      if (!a.pchunks[s]) continue;
      float* outs[1] = {segs_host[s].grad};
      const int b0[1] = {0};
      const float one[1] = {1.f};
      reduce_defer_job(a.ws + a.pws_off[s], a.pchunks[s], (int)(segs_host[s].vocab * segs_host[s].dim), 1, outs, b0,
                       one, one);
    }
  } else if (a.ws_floats > 0) {
    int64_t nel = 0;
    for (int s = 0; s < nseg; ++s)
      if (a.pchunks[s]) nel = std::max<int64_t>(nel, segs_host[s].vocab * segs_host[s].dim / 4 + 1);
    reduce_partials_kernel<<<(int)std::min<int64_t>(cdiv(nel, 64), 1024), kReduceWaves * 64, 0, st>>>(a);
    RS_CHECK_LAUNCH("rs_gather_bwd partials");
  }
  return 0;
}

extern "C" int rs_seq_mask(const int64_t* seq, int64_t ld_seq, int B, int L, int64_t pad_value,
                           uint8_t* key_pad, int64_t* last, void* stream) {
  RS_CHECK_ARG(seq && key_pad && last && B >= 0 && L >= 1 && ld_seq >= L, "rs_seq_mask: bad args");
  if (B == 0) return 0;
  seq_mask_kernel<<<cdiv(B, 4), 256, 0, as_stream(stream)>>>(seq, ld_seq, B, L, pad_value, key_pad,
                                                              last);
  RS_CHECK_LAUNCH("rs_seq_mask");
  return 0;
}

// ---------------------------------------------------------------- hard-negative catalog gather
namespace rs {
namespace {
template <typename TI, typename TO>
__global__ void catalog_gather_kernel(const TI* __restrict__ cat, int64_t V, int F, int64_t ld_cat,
                                      const int64_t* __restrict__ ids, int B, int N,
                                      int64_t ld_ids, TO* __restrict__ out, int64_t ld_out,
                                      int* err) {
  const int64_t total = (int64_t)N * B * F;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / F;  // n*B + b
    const int f = (int)(e - row * F);
    const int n = (int)(row / B), b = (int)(row - (int64_t)n * B);
    const int64_t id = ids[(int64_t)b * ld_ids + n];
    TO v = 0;
    if (id >= 0 && id < V) v = (TO)cat[id * ld_cat + f];
    else if (err && f == 0) atomicOr(err, 1);
    out[row * ld_out + f] = v;
  }
}
}  // namespace
}  // namespace rs

extern "C" int rs_catalog_gather(const void* cat, int elem, int widen, int64_t V, int F,
                                 int64_t ld_cat, const int64_t* ids, int B, int N, int64_t ld_ids,
                                 void* out, int64_t ld_out, int* err_flag, void* stream) {
  RS_CHECK_ARG(cat && ids && out && V >= 1 && F >= 1 && B >= 0 && N >= 0 && ld_cat >= F &&
                   ld_out >= F && ld_ids >= N,
               "rs_catalog_gather: bad args");
  RS_CHECK_ARG(elem == 4 || elem == 8, "rs_catalog_gather: elem must be 4 or 8 bytes");
  RS_CHECK_ARG(!widen || elem == 4, "rs_catalog_gather: widen needs int32 input");
  const int64_t total = (int64_t)N * B * F;
  if (total == 0) return 0;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipStream_t st = as_stream(stream);
  if (widen)
    catalog_gather_kernel<int32_t, int64_t><<<blocks, 256, 0, st>>>(
        static_cast<const int32_t*>(cat), V, F, ld_cat, ids, B, N, ld_ids, static_cast<int64_t*>(out), ld_out, err_flag);
  else if (elem == 8)
    catalog_gather_kernel<int64_t, int64_t><<<blocks, 256, 0, st>>>(
        static_cast<const int64_t*>(cat), V, F, ld_cat, ids, B, N, ld_ids, static_cast<int64_t*>(out), ld_out, err_flag);
  else
    catalog_gather_kernel<uint32_t, uint32_t><<<blocks, 256, 0, st>>>(
        static_cast<const uint32_t*>(cat), V, F, ld_cat, ids, B, N, ld_ids, static_cast<uint32_t*>(out), ld_out, err_flag);
  RS_CHECK_LAUNCH("rs_catalog_gather");
  return 0;
}
