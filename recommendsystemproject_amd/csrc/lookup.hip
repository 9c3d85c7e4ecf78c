// Sorted lookups of the large embedding tables: a deterministic, atomic-free replacement of the
// table-gradient scatter-add (GenericTower.py:182 nn.Embedding -> embedding_dense_backward) and
// the row bookkeeping of lazy-exact Adam (sparse.hip).
//
// One "call" = one lookup of a table in the forward (a [rows, bag] id matrix read in place).
//   rs_lookup_sort : stable LSD radix sort of the call's ids -> keys[n] (row ids ascending,
//                    out-of-range ids last as 0xFFFFFFFF) and vals[n] (the lookup index
//                    e = r * bag + l; ascending within a row because the sort is stable).
//   rs_sorted_catchup / _adam / _sqnorm / _zero_grad / _owner : per distinct row (run head of
//                    keys): lazy-Adam catch-up before the gather, the Adam step, the clip-norm
//                    partials, gradient zeroing, and the lowest call index holding a row (a row
//                    looked up by several calls in one step is stepped once).
//   rs_segsum      : the table gradient. Fixed chunks of 64 sorted positions per wave; a run
//                    (one row's lookups) that lies inside a chunk is summed in lookup order and
//                    stored with a plain store; a run crossing chunk boundaries leaves per-chunk
//                    partials that a fixup pass adds in chunk order. Work per wave is the same
//                    whatever the id skew (a Zipf hot row with 10^4 lookups spreads over 10^2
//                    chunks), there are no float atomics, and the result is bitwise
//                    reproducible -- which is what lets every data-parallel rank rebuild the same
//                    gradient from all-gathered bag gradients (dist.py).
//
// Radix sort (multi-tile): per pass, hist (per-tile digit counts) -> scan (one workgroup per
// digit over the tiles) -> scatter (stable in-tile ranking by wave ballots, cross-wave prefix in
// LDS). Digits of up to 9 bits; passes = ceil(bits(vocab) / 9): 3 for 1M-100M-row tables.
// A call of at most 4096 lookups is sorted by one workgroup in one launch (keys in registers,
// exchanged through LDS between passes).
#include "common.h"
#include "adam.h"

#pragma clang fp contract(off)  // the Adam here must round exactly like adam_kernel / sparse.hip

namespace rs {
namespace {

// multi-tile radix sort: 1,024-lookup tiles of 256 threads (a 204,800-lookup call is 200 tiles:
// 4,096-lookup tiles of 1,024 threads gave 50 workgroups and a 16-wave prefix per ranking round)
constexpr int kSortThreads = 256;
constexpr int kSortRounds = 4;
constexpr int kSortTile = kSortThreads * kSortRounds;  // 1,024 lookups per tile
// one-workgroup sort of calls of at most kTileMax lookups (4 keys per thread)
constexpr int kTileThreads = 1024;
constexpr int kTileMax = 4096;
constexpr int kMaxDigitBits = 9;
constexpr int kMaxRadix = 1 << kMaxDigitBits;
constexpr uint32_t kSentinel = 0xFFFFFFFFu;

struct SortPlan {
  int bits;    // key bits (sentinel's low `bits` bits exceed every valid id)
  int passes;
  int dbits[4];
  int shift[4];
  int ntiles;
};

SortPlan make_plan(int64_t n, int64_t vocab) {
  SortPlan p;
  int bits = 1;
  while (bits < 32 && ((int64_t)1 << bits) - 1 < vocab) ++bits;
  p.bits = bits;
  p.passes = (bits + kMaxDigitBits - 1) / kMaxDigitBits;
  int sh = 0;
  for (int i = 0; i < p.passes; ++i) {
    const int left = bits - sh, passes_left = p.passes - i;
    p.dbits[i] = (left + passes_left - 1) / passes_left;
    p.shift[i] = sh;
    sh += p.dbits[i];
  }
  p.ntiles = cdiv(n, kSortTile);
  return p;
}

// pass-0 key of lookup e: the row id read in place from the [rows, bag] id matrix (row stride
// `stride`, int64 or int32 ids); out-of-range ids sort last as the sentinel
__device__ __forceinline__ uint32_t raw_key(const void* ids, int id_bytes, int bag, int64_t stride,
                                            int64_t vocab, int64_t e) {
  const int64_t r = e / bag, l = e - r * bag;
  const int64_t id = id_bytes == 8 ? static_cast<const int64_t*>(ids)[r * stride + l]
                                   : (int64_t) static_cast<const int32_t*>(ids)[r * stride + l];
  return id >= 0 && id < vocab ? (uint32_t)id : kSentinel;
}

template <int NT>
struct RankLds {
  static constexpr int NW = NT / 64;
  uint16_t wc[NW][kMaxRadix];   // per-wave digit counts of the current round (leaders)
  uint16_t pre[NW][kMaxRadix];  // tile-local start of each wave's group of a digit
  int run[kMaxRadix];           // tile-local count of each digit before this round
};

// Stable rank of this lane's digit within the tile, for one round of kSortThreads keys (key
// order = round, wave, lane). Returns the tile-local position among keys of the same digit
// (counting earlier rounds through lds.run). Two barriers.
template <int NT>
__device__ __forceinline__ int rank_round(RankLds<NT>& lds, uint32_t d, bool valid, int dbits,
                                          int radix) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t peers = __ballot(valid);
  for (int b = 0; b < dbits; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  if (!valid) peers = 0;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int lrank = __popcll(peers & lt);
  if (valid && lrank == 0) lds.wc[w][d] = (uint16_t)__popcll(peers);
  __syncthreads();
  for (int t = threadIdx.x; t < radix; t += NT) {
    int r = lds.run[t];
#pragma unroll
    for (int ww = 0; ww < RankLds<NT>::NW; ++ww) {
      const int c = lds.wc[ww][t];
      lds.wc[ww][t] = 0;
      lds.pre[ww][t] = (uint16_t)r;
      r += c;
    }
    lds.run[t] = r;
  }
  __syncthreads();
  return valid ? (int)lds.pre[w][d] + lrank : 0;
}

template <int NT>
__device__ __forceinline__ void rank_reset(RankLds<NT>& lds, int radix) {
  for (int t = threadIdx.x; t < radix; t += NT) lds.run[t] = 0;
  for (int i = threadIdx.x; i < RankLds<NT>::NW * kMaxRadix; i += NT)
    (&lds.wc[0][0])[i] = 0;
}

// ---------------------------------------------------------------- multi-tile radix sort
__global__ __launch_bounds__(kSortThreads) void sort_hist_kernel(
    const void* __restrict__ ids, int id_bytes, int bag, int64_t stride, int64_t vocab,
    const uint32_t* __restrict__ src, int64_t n, int shift, int dbits, int* __restrict__ hist) {
  __shared__ int h[kMaxRadix];
  const int radix = 1 << dbits;
  for (int t = threadIdx.x; t < radix; t += kSortThreads) h[t] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t e = base + r * kSortThreads + threadIdx.x;
    if (e < n) {
      const uint32_t k = src ? src[e] : raw_key(ids, id_bytes, bag, stride, vocab, e);
      atomicAdd(&h[(k >> shift) & (radix - 1)], 1);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < radix; t += kSortThreads) hist[(int64_t)t * gridDim.x + blockIdx.x] = h[t];
}

// one workgroup per digit: exclusive scan of hist[d][0 .. ntiles) in place, total -> tot[d]
__global__ __launch_bounds__(256) void sort_scan_kernel(int* __restrict__ hist, int ntiles,
                                                        int* __restrict__ tot) {
  __shared__ int wsum[4];
  __shared__ int carry;
  int* row = hist + (int64_t)blockIdx.x * ntiles;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int b0 = 0; b0 < ntiles; b0 += 256) {
    const int i = b0 + threadIdx.x;
    const int x = i < ntiles ? row[i] : 0;
    int y = x;
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(y, o, 64);
      if (lane >= o) y += t;
    }
    if (lane == 63) wsum[w] = y;
    __syncthreads();
    int pre = carry;
    for (int k = 0; k < w; ++k) pre += wsum[k];
    if (i < ntiles) row[i] = pre + y - x;
    __syncthreads();
    if (threadIdx.x == 255) carry = pre + y;
    __syncthreads();
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = carry;
}

__global__ __launch_bounds__(kSortThreads) void sort_scatter_kernel(
    const void* __restrict__ ids, int id_bytes, int bag, int64_t stride, int64_t vocab,
    const uint32_t* __restrict__ ksrc, const uint32_t* __restrict__ vsrc, int64_t n, int shift,
    int dbits, const int* __restrict__ hist, const int* __restrict__ tot,
    uint32_t* __restrict__ kdst, uint32_t* __restrict__ vdst) {
  __shared__ RankLds<kSortThreads> lds;
  __shared__ int gbase[kMaxRadix];
  const int radix = 1 << dbits;
  rank_reset(lds, radix);
  // global base of digit d for this tile: (keys of smaller digits) + (digit d in earlier tiles)
  if (threadIdx.x < 64) {
    int carry = 0;
    const int lane = threadIdx.x;
    for (int d0 = 0; d0 < radix; d0 += 64) {
      const int x = d0 + lane < radix ? tot[d0 + lane] : 0;
      int y = x;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(y, o, 64);
        if (lane >= o) y += t;
      }
      if (d0 + lane < radix)
        gbase[d0 + lane] = carry + y - x + hist[(int64_t)(d0 + lane) * gridDim.x + blockIdx.x];
      carry += __shfl(y, 63, 64);
    }
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  uint32_t key[kSortRounds], val[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t e = base + r * kSortThreads + threadIdx.x;
    key[r] = kSentinel;
    val[r] = 0;
    if (e < n) {
      key[r] = ksrc ? ksrc[e] : raw_key(ids, id_bytes, bag, stride, vocab, e);
      val[r] = vsrc ? vsrc[e] : (uint32_t)e;
    }
  }
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int64_t e = base + r * kSortThreads + threadIdx.x;
    const bool valid = e < n;
    const uint32_t d = (key[r] >> shift) & (radix - 1);
    const int lp = rank_round(lds, d, valid, dbits, radix);
    if (valid) {
      const int64_t pos = (int64_t)gbase[d] + lp;
      kdst[pos] = key[r];
      vdst[pos] = val[r];
    }
  }
}

// ---------------------------------------------------------------- one-tile sort (n <= 4096)
// One workgroup, the keys in registers (4 per thread) and exchanged through LDS between the
// radix passes. (Measured and rejected: a bitonic sort of key/index pairs -- 39 us with an LDS
// barrier per step, 47 us with the short distances in registers and shuffles: 78 steps of 4,096
// compare-exchanges on one CU are VALU-bound.)
// Wave-major ranking (round 3): wave w holds keys w*256 .. w*256+255 (4 rounds of 64 lanes), so a
// key's rank among equal digits is (digit base) + (that digit's count in earlier waves) + (its
// count in this wave's earlier rounds) + (its lane rank): each wave keeps running per-digit counts
// in its own LDS row with no workgroup barrier inside the rounds, and one prefix over the 16
// waves per digit replaces the per-round 16-wave prefix and its two barriers (4 per pass before:
// the user_id sort, 4,096 keys, 3 passes, took ~23 us).
constexpr int kTileWaves = kTileThreads / 64;
constexpr int kTileKeys = kTileMax / kTileWaves;  // keys per wave (4 rounds of 64)
static_assert(kTileKeys == kSortRounds * 64, "one-tile sort: 4 rounds of 64 keys per wave");

__global__ __launch_bounds__(kTileThreads) void sort_tile_kernel(
    const void* __restrict__ ids, int id_bytes, int bag, int64_t stride, int64_t vocab, int n,
    SortPlan plan, uint32_t* __restrict__ kout, uint32_t* __restrict__ vout) {
  __shared__ uint16_t cnt[kTileWaves][kMaxRadix];  // per wave: running, then exclusive, digit counts
  __shared__ int dbase[kMaxRadix];                  // exclusive scan of the digit totals
  __shared__ int wsum[kTileWaves];
  __shared__ uint32_t xchg[kTileMax];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  uint32_t key[kSortRounds], val[kSortRounds];
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int e = w * kTileKeys + r * 64 + lane;
    key[r] = e < n ? raw_key(ids, id_bytes, bag, stride, vocab, e) : kSentinel;
    val[r] = (uint32_t)e;
  }
  for (int p = 0; p < plan.passes; ++p) {
    const int radix = 1 << plan.dbits[p], shift = plan.shift[p], dbits = plan.dbits[p];
    for (int t = threadIdx.x; t < kTileWaves * radix; t += kTileThreads) cnt[t / radix][t % radix] = 0;
    __syncthreads();
    int pin[kSortRounds];  // rank among this wave's keys of the same digit
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      const bool valid = w * kTileKeys + r * 64 + lane < n;
      const uint32_t d = (key[r] >> shift) & (radix - 1);
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < dbits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
      }
      const int lrank = __popcll(peers & lt);
      // every lane reads its digit's count, then the group's first lane adds the group (the
      // wave's LDS operations complete in program order; the store is after the load)
      const int old = valid ? (int)cnt[w][d] : 0;
      __builtin_amdgcn_wave_barrier();
      if (valid && lrank == 0) cnt[w][d] = (uint16_t)(old + __popcll(peers));
      __builtin_amdgcn_wave_barrier();
      pin[r] = old + lrank;
    }
    __syncthreads();
    // per digit: exclusive offsets over the waves, then the digit totals scanned
    int tot = 0;
    if ((int)threadIdx.x < radix) {
#pragma unroll
      for (int ww = 0; ww < kTileWaves; ++ww) {
        const int c = cnt[ww][threadIdx.x];
        cnt[ww][threadIdx.x] = (uint16_t)tot;
        tot += c;
      }
    }
    int y = tot;  // inclusive scan over the digits: lanes, then the waves' sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(y, o, 64);
      if (lane >= o) y += t;
    }
    if (lane == 63) wsum[w] = y;
    __syncthreads();
    if ((int)threadIdx.x < radix) {
      int pre = 0;
      for (int ww = 0; ww < w; ++ww) pre += wsum[ww];
      dbase[threadIdx.x] = pre + y - tot;
    }
    __syncthreads();
    int pos[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      const bool valid = w * kTileKeys + r * 64 + lane < n;
      const uint32_t d = (key[r] >> shift) & (radix - 1);
      pos[r] = valid ? dbase[d] + (int)cnt[w][d] + pin[r] : -1;
    }
    // exchange keys, then values, through LDS into the new order
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) if (pos[r] >= 0) xchg[pos[r]] = key[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      const int e = w * kTileKeys + r * 64 + lane;
      if (e < n) key[r] = xchg[e];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) if (pos[r] >= 0) xchg[pos[r]] = val[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
      const int e = w * kTileKeys + r * 64 + lane;
      if (e < n) val[r] = xchg[e];
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const int e = w * kTileKeys + r * 64 + lane;
    if (e < n) {
      kout[e] = key[r];
      vout[e] = val[r];
    }
  }
}

// ---------------------------------------------------------------- counting sort (n <= kRankMax)
// A small call (C3's user-id and item-id calls: 4,096 ids) sorted by counting ranks spread over
// the whole chip instead of one workgroup's radix passes (sort_tile_kernel: 3 passes of 4,096 keys
// on one CU, ~19 us). The stable rank of lookup i is
//   rank(i) = #{j : key_j < key_i} + #{j < i : key_j == key_i},
// a permutation of 0 .. n-1. Pass 1: workgroup (ib, jb) counts, for the 256 keys of block ib, the
// keys of block jb that precede them (j < i is decided per block: every j of a lower block
// precedes i on a tie, no j of a higher block does; the diagonal block compares indices) -- 256 x
// 256 compares, one broadcast LDS read per 4 keys; the partial counts go to the workspace. Pass 2:
// one thread per lookup sums its nb partials and stores its key and lookup index at its rank.
// n = 4,096: 256 workgroups of ~2 x 256 VALU operations per lane, then 16 workgroups.
constexpr int kRankBlock = 256;
constexpr int kRankMax = 8192;

__global__ __launch_bounds__(kRankBlock) void rank_partial_kernel(const void* __restrict__ ids, int id_bytes,
                                                                  int bag, int64_t stride, int64_t vocab, int n,
                                                                  int* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint32_t kj[kRankBlock];
  const int ib = blockIdx.x, jb = blockIdx.y, t = threadIdx.x;
  const int i = ib * kRankBlock + t, j = jb * kRankBlock + t;
  const uint32_t ki = i < n ? raw_key(ids, id_bytes, bag, stride, vocab, i) : kSentinel;
  // past n: the sentinel, which precedes no key (never <, and == only on the diagonal block at
  // an index above every valid one)
  kj[t] = j < n ? raw_key(ids, id_bytes, bag, stride, vocab, j) : kSentinel;
  __syncthreads();
  int cnt = 0;
  const uint4* q = reinterpret_cast<const uint4*>(kj);
  if (jb < ib) {
#pragma unroll 16
    for (int c = 0; c < kRankBlock / 4; ++c) {
      const uint4 k4 = q[c];
      cnt += (k4.x <= ki) + (k4.y <= ki) + (k4.z <= ki) + (k4.w <= ki);
    }
  } else if (jb > ib) {
#pragma unroll 16
    for (int c = 0; c < kRankBlock / 4; ++c) {
      const uint4 k4 = q[c];
      cnt += (k4.x < ki) + (k4.y < ki) + (k4.z < ki) + (k4.w < ki);
    }
  } else {
#pragma unroll 16
    for (int c = 0; c < kRankBlock / 4; ++c) {
      const uint4 k4 = q[c];
      const int b = 4 * c;
      cnt += (k4.x < ki || (k4.x == ki && b < t)) + (k4.y < ki || (k4.y == ki && b + 1 < t)) +
             (k4.z < ki || (k4.z == ki && b + 2 < t)) + (k4.w < ki || (k4.w == ki && b + 3 < t));
    }
  }
  if (i < n) part[(int64_t)jb * n + i] = cnt;
}

__global__ __launch_bounds__(256) void rank_scatter_kernel(const void* __restrict__ ids, int id_bytes, int bag,
                                                           int64_t stride, int64_t vocab, int n, int nb,
                                                           const int* __restrict__ part,
                                                           uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int r = 0;
  for (int b = 0; b < nb; ++b) r += part[(int64_t)b * n + i];
  keys[r] = raw_key(ids, id_bytes, bag, stride, vocab, i);
  vals[r] = (uint32_t)i;
}

// ---------------------------------------------------------------- per distinct row

__device__ __forceinline__ int clamp_step(const float2* consts, int64_t t) {
  const int cap = __float_as_int(consts[0].x);
  return t < cap ? (int)t : cap - 1;
}

enum RowOp { kCatchup = 0, kAdam = 1, kSqnorm = 2, kOwner = 3, kZero = 4 };

struct RowArgs {
  const uint32_t* keys;
  int64_t n;
  int D;
  float* p;
  float* g;
  float* m;
  float* v;
  int* last;
  int* owner;   // null: the call is the only one of its step
  int call;
  const int64_t* step;
  const float2* consts;
  AdamConst h;
  float scale;
  const float* coef;
  double* ws;   // kSqnorm: one partial per workgroup
};

// One group of G lanes per sorted position (G = the lanes that cover a row 4 columns each:
// D = 128 -> 32 lanes, two rows per wave; D <= 4 G); a group whose position is a run head (a
// distinct row) processes that row with float4 loads (a whole wave walking its 64 positions' heads
// one at a time was a chain of dependent row round trips: 3-4x slower). U > 1 takes U positions
// per group iteration with their loads issued together; measured slower at U = 4 (168 VGPRs, fewer
// resident waves: tools/lazy_bench.py), so U = 1.
constexpr int kRowUnroll = 1;
// The clip partials (kSqnorm) read one gradient row per position: 4 positions per group iteration
// with their loads issued together (16 VGPRs of rows; the per-lane accumulation order is that of
// U = 1: positions i0, i0 + ngroups, ...). Their grid is fixed at kRowGrid workgroups (one partial
// each), so a group walks ~13 positions at C3 -- one key and one row round trip each at U = 1.
constexpr int kSqUnroll = 4;

// bid / nblocks: this workgroup's index and count among the workgroups working on `a` (a batched
// launch deals one contiguous block range to each call)
template <int OP, int G, int U>
__device__ __forceinline__ void sorted_rows_body(const RowArgs& a, int bid, int nblocks) {
  __shared__ double red[4];
  __shared__ float2 cwin[(OP == kCatchup || OP == kAdam) ? kConstWin : 1];
  const int gl = threadIdx.x & (G - 1);
  double acc = 0.0;
  int t = 0;
  float2 ct = make_float2(0.f, 0.f);
  float s = 1.f;
  ConstWin cw{a.consts, cwin, 0};
  if (OP == kCatchup || OP == kAdam) {
    t = clamp_step(a.consts, *a.step);
    cw.lo = t - kConstWin + 1;
    if (threadIdx.x < kConstWin) {
      const int st = cw.lo + (int)threadIdx.x;
      cwin[threadIdx.x] = a.consts[st > 0 ? st : 0];
    }
    __syncthreads();
  }
  if (OP == kAdam) {
    ct = cwin[kConstWin - 1];
    s = a.scale * (a.coef ? *a.coef : 1.f);
  }
  const int64_t ngroups = (int64_t)nblocks * (256 / G);
  const int c0 = gl * 4;
  const int w = c0 < a.D ? (a.D - c0 < 4 ? a.D - c0 : 4) : 0;  // columns of this lane
  const bool vec = (a.D & 3) == 0;
  for (int64_t i0 = (int64_t)bid * (256 / G) + threadIdx.x / G; i0 < a.n; i0 += ngroups * U) {
    int64_t row[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * ngroups;
      const uint32_t k = i < a.n ? a.keys[i] : kSentinel;
      const uint32_t kp = i > 0 && i < a.n ? a.keys[i - 1] : kSentinel;
      act[u] = k != kSentinel && (i == 0 || kp != k);
      row[u] = k;
    }
    if (OP == kOwner) {
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (act[u] && gl == 0) atomicMin(&a.owner[row[u]], a.call);
      continue;
    }
    // a row's state steps: lm = its moments', lp = its parameters' (lp > lm after a forward
    // catch-up that wrote p alone, weight_decay == 0; equal otherwise)
    int lm[U], lp[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      lm[u] = lp[u] = 0;
      if (act[u] && OP != kCatchup && a.owner && a.owner[row[u]] != a.call) act[u] = false;
      if (act[u] && (OP == kCatchup || OP == kAdam)) {
        const int2 l2 = reinterpret_cast<const int2*>(a.last)[row[u]];
        lm[u] = l2.x;
        lp[u] = l2.y;
      }
      // catch-up: p already current, or a row never stepped (its m = v = 0 from the start: with
      // weight_decay == 0 the replay is the identity, exactly)
      if (OP == kCatchup && act[u] && (lp[u] >= t || (lm[u] == 0 && a.h.wd == 0.f))) act[u] = false;
    }
    float pp[U][4], mm[U][4], vv[U][4], gg[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!act[u] || w == 0) continue;
      const int64_t o = row[u] * a.D + c0;
      if (OP == kCatchup || OP == kAdam) {
        if (vec) {
          const float4 p4 = *reinterpret_cast<const float4*>(a.p + o);
          pp[u][0] = p4.x; pp[u][1] = p4.y; pp[u][2] = p4.z; pp[u][3] = p4.w;
          if (lm[u] == 0 && a.h.wd == 0.f && OP == kAdam) {  // never stepped: m = v = 0
#pragma unroll
            for (int j = 0; j < 4; ++j) { mm[u][j] = 0.f; vv[u][j] = 0.f; }
          } else {
            const float4 m4 = *reinterpret_cast<const float4*>(a.m + o);
            const float4 v4 = *reinterpret_cast<const float4*>(a.v + o);
            mm[u][0] = m4.x; mm[u][1] = m4.y; mm[u][2] = m4.z; mm[u][3] = m4.w;
            vv[u][0] = v4.x; vv[u][1] = v4.y; vv[u][2] = v4.z; vv[u][3] = v4.w;
          }
        } else {  // D % 4 != 0: the lane's columns past w are zeros (m = v = 0: they stay put)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pp[u][j] = j < w ? a.p[o + j] : 0.f;
            mm[u][j] = j < w ? a.m[o + j] : 0.f;
            vv[u][j] = j < w ? a.v[o + j] : 0.f;
          }
        }
      }
      if (OP == kAdam || OP == kSqnorm) {
        if (vec) {
          const float4 g4 = *reinterpret_cast<const float4*>(a.g + o);
          gg[u][0] = g4.x; gg[u][1] = g4.y; gg[u][2] = g4.z; gg[u][3] = g4.w;
        } else {
          for (int j = 0; j < w; ++j) gg[u][j] = a.g[o + j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!act[u]) continue;
      if (w > 0) {
        const int64_t o = row[u] * a.D + c0;
        if (OP == kCatchup || OP == kAdam)
          adam_catch_row_f<4>(a.h, cw, lm[u], lp[u], OP == kCatchup ? t : t - 1, pp[u], mm[u], vv[u]);
        if (OP == kAdam) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < w) adam_update(a.h, ct.x, ct.y, gg[u][j] * s, pp[u][j], mm[u][j], vv[u][j]);
        } else if (OP == kSqnorm) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < w) {
              const float x = gg[u][j] * a.scale;
              acc += (double)(x * x);
            }
        }
        if (OP == kCatchup || OP == kAdam) {
          // the forward catch-up writes p alone when weight_decay == 0 (the moments stay at their
          // step and are replayed again by the optimizer step: two row writes per row saved)
          const bool mv = OP == kAdam || a.h.wd != 0.f;
          if (vec) {
            *reinterpret_cast<float4*>(a.p + o) = make_float4(pp[u][0], pp[u][1], pp[u][2], pp[u][3]);
            if (mv) {
              *reinterpret_cast<float4*>(a.m + o) = make_float4(mm[u][0], mm[u][1], mm[u][2], mm[u][3]);
              *reinterpret_cast<float4*>(a.v + o) = make_float4(vv[u][0], vv[u][1], vv[u][2], vv[u][3]);
            }
          } else {
            for (int j = 0; j < w; ++j) {
              a.p[o + j] = pp[u][j];
              if (mv) { a.m[o + j] = mm[u][j]; a.v[o + j] = vv[u][j]; }
            }
          }
        }
        if (OP == kAdam || OP == kZero) {
          if (vec) *reinterpret_cast<float4*>(a.g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
          else for (int j = 0; j < w; ++j) a.g[o + j] = 0.f;
        }
      }
      if ((OP == kCatchup || OP == kAdam) && gl == 0) {
        const bool p_only = OP == kCatchup && a.h.wd == 0.f;
        reinterpret_cast<int2*>(a.last)[row[u]] = make_int2(p_only ? lm[u] : t, t);
        if (OP == kAdam && a.owner) a.owner[row[u]] = 0x7fffffff;
      }
    }
  }
  if (OP == kSqnorm) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) a.ws[bid] = red[0] + red[1] + red[2] + red[3];
  }
}

template <int OP, int G, int U>
__global__ __launch_bounds__(256) void sorted_rows_kernel(RowArgs a) {
  sorted_rows_body<OP, G, U>(a, blockIdx.x, gridDim.x);
}

// several calls in one launch (the optimizer's per-call Adam steps / clip partials: one dispatch
// instead of one per call); call c owns workgroups [first[c], first[c + 1])
constexpr int kRowBatchMax = 8;

// The dense region of the flat buffer riding in the same launch (round 5: one launch less each for
// the clip partials and the Adam step of a step with lazy tables -- ~4.5 us of launch floor each on
// this box): workgroups [0, blocks) do what rs_grad_sqnorm / rs_adam_step do, with the same
// partition (the same partials, the same bits), the sorted calls the rest.
struct DensePart {
  float* p; float* g; float* m; float* v;  // Adam: all four; sqnorm: g
  int64_t n;
  int blocks;                              // 0: no dense part
  float lr, b1, b2;                        // Adam: the step constants come from *step (as rs_adam_step)
  AdamConst h;
  double* ws;                              // sqnorm: one partial per dense workgroup
};

struct RowBatch {
  RowArgs a[kRowBatchMax];
  int first[kRowBatchMax + 1];
  int n;
  DensePart d;
};

// rs_grad_sqnorm's and rs_adam_step's grids (optim.hip sq_blocks / adam blocks)
static int dense_sq_blocks(int64_t n) {
  int64_t b = (n + 256 * 16 - 1) / (256 * 16);
  return (int)(b > 1024 ? 1024 : (b < 1 ? 1 : b));
}
static int dense_adam_blocks(int64_t n) {
  int64_t b = (n / 4 + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

template <int OP>
__device__ __forceinline__ void dense_part(const DensePart& d, const int64_t* step, float scale, const float* coef,
                                           int bid) {
#pragma clang fp contract(off)
  const int64_t stride = (int64_t)d.blocks * 256;
  if constexpr (OP == kSqnorm) {
    __shared__ double red[4];
    double acc = 0.0;
    const int64_t n4 = d.n / 4;
    if ((reinterpret_cast<uintptr_t>(d.g) & 15) == 0) {
      const float4* g4 = reinterpret_cast<const float4*>(d.g);
      for (int64_t i = bid * 256 + threadIdx.x; i < n4; i += stride) {
        const float4 v = g4[i];
        const float a = v.x * scale, b = v.y * scale, c = v.z * scale, e = v.w * scale;
        acc += (double)(a * a) + (double)(b * b) + (double)(c * c) + (double)(e * e);
      }
      for (int64_t i = n4 * 4 + bid * 256 + threadIdx.x; i < d.n; i += stride) {
        const float a = d.g[i] * scale;
        acc += (double)(a * a);
      }
    } else {
      for (int64_t i = bid * 256 + threadIdx.x; i < d.n; i += stride) {
        const float a = d.g[i] * scale;
        acc += (double)(a * a);
      }
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) d.ws[bid] = red[0] + red[1] + red[2] + red[3];
  } else if constexpr (OP == kAdam) {
    const float s = scale * (coef ? *coef : 1.f);
    float step_size, inv_bc2;
    adam_step_consts((double)d.lr, (double)d.b1, (double)d.b2, (double)*step, &step_size, &inv_bc2);
    const bool vec = ((reinterpret_cast<uintptr_t>(d.p) | reinterpret_cast<uintptr_t>(d.g) |
                       reinterpret_cast<uintptr_t>(d.m) | reinterpret_cast<uintptr_t>(d.v)) & 15) == 0;
    int64_t done = 0;
    if (vec) {
      const int64_t n4 = d.n / 4;
      float4* p4 = reinterpret_cast<float4*>(d.p);
      float4* g4 = reinterpret_cast<float4*>(d.g);
      float4* m4 = reinterpret_cast<float4*>(d.m);
      float4* v4 = reinterpret_cast<float4*>(d.v);
      for (int64_t i = bid * 256 + threadIdx.x; i < n4; i += stride) {
        float4 p = p4[i], g = g4[i], m = m4[i], v = v4[i];
        adam_update(d.h, step_size, inv_bc2, g.x * s, p.x, m.x, v.x);
        adam_update(d.h, step_size, inv_bc2, g.y * s, p.y, m.y, v.y);
        adam_update(d.h, step_size, inv_bc2, g.z * s, p.z, m.z, v.z);
        adam_update(d.h, step_size, inv_bc2, g.w * s, p.w, m.w, v.w);
        p4[i] = p; m4[i] = m; v4[i] = v;
      }
      done = n4 * 4;
    }
    for (int64_t i = done + bid * 256 + threadIdx.x; i < d.n; i += stride) {
      float p = d.p[i], m = d.m[i], v = d.v[i];
      adam_update(d.h, step_size, inv_bc2, d.g[i] * s, p, m, v);
      d.p[i] = p; d.m[i] = m; d.v[i] = v;
    }
  }
}

template <int OP, int G, int U>
__global__ __launch_bounds__(256) void sorted_rows_batch_kernel(RowBatch b) {
  if ((int)blockIdx.x < b.d.blocks) {  // uniform per workgroup
    dense_part<OP>(b.d, b.a[0].step, b.a[0].scale, b.a[0].coef, blockIdx.x);
    return;
  }
  const int bid = (int)blockIdx.x - b.d.blocks;
  int c = 0;
  while (c + 1 < b.n && bid >= b.first[c + 1]) ++c;
  sorted_rows_body<OP, G, U>(b.a[c], bid - b.first[c], b.first[c + 1] - b.first[c]);
}

constexpr int kRowGrid = 2048;

// ---------------------------------------------------------------- catch-up in lookup order
// The forward catch-up without the sort: one group of G lanes per lookup e of the [rows, bag] id
// matrix. The group whose compare-and-swap moves last[row] from its stale value to t is the one
// that replays the row (any one of the row's lookups: the replay only depends on the row's
// state, so the result is the same bits as the sorted catch-up's); every other lookup of the row
// sees last == t, or loses the swap, and does nothing. The gather is the next kernel, so every
// row it reads is current. This takes the sort off the forward path: it only feeds the backward
// (segment sums) and the optimizer, and runs on a side stream (flat.py).
struct IdCatchArgs {
  const void* ids;
  int id_bytes;
  int bag;
  int64_t stride;
  int64_t vocab;
  int64_t n;
  int D;
  float* p;
  float* m;
  float* v;
  int* last;
  const int64_t* step;
  const float2* consts;
  AdamConst h;
};

template <int G>
__global__ __launch_bounds__(256) void lookup_catchup_kernel(IdCatchArgs a) {
  const int gl = threadIdx.x & (G - 1);
  const int t = clamp_step(a.consts, *a.step);
  __shared__ float2 cwin[kConstWin];  // the recent steps' constants (ConstWin)
  const ConstWin cw{a.consts, cwin, t - kConstWin + 1};
  if (threadIdx.x < kConstWin) {
    const int st = cw.lo + (int)threadIdx.x;
    cwin[threadIdx.x] = a.consts[st > 0 ? st : 0];
  }
  __syncthreads();
  const int64_t ngroups = (int64_t)gridDim.x * (256 / G);
  const int c0 = gl * 4;
  const int w = c0 < a.D ? (a.D - c0 < 4 ? a.D - c0 : 4) : 0;
  const bool vec = (a.D & 3) == 0;
  for (int64_t e = (int64_t)blockIdx.x * (256 / G) + threadIdx.x / G; e < a.n; e += ngroups) {
    const uint32_t k = raw_key(a.ids, a.id_bytes, a.bag, a.stride, a.vocab, e);
    if (k == kSentinel) continue;  // the gather flags it
    // the row's state steps (moments, parameters) as one 64-bit word: the compare-and-swap moves
    // both together
    unsigned long long* lw = reinterpret_cast<unsigned long long*>(a.last) + k;
    const unsigned long long old = *lw;
    const int lm = (int)(uint32_t)old, lp = (int)(uint32_t)(old >> 32);
    // p already current, or a row never stepped (m = v = 0: with weight_decay == 0 the replay is
    // the identity, exactly)
    if (lp >= t || (lm == 0 && a.h.wd == 0.f)) continue;
    const bool p_only = a.h.wd == 0.f;  // as sorted_rows_body's catch-up: p written alone
    const unsigned long long nw = ((unsigned long long)(uint32_t)t << 32) | (uint32_t)(p_only ? lm : t);
    int won = 0;
    if (gl == 0) won = atomicCAS(lw, old, nw) == old;
    won = __shfl(won, 0, G);
    if (!won || w == 0) continue;
    const int64_t o = (int64_t)k * a.D + c0;
    float pp[4], mm[4], vv[4];
    if (vec) {
      const float4 p4 = *reinterpret_cast<const float4*>(a.p + o);
      const float4 m4 = *reinterpret_cast<const float4*>(a.m + o);
      const float4 v4 = *reinterpret_cast<const float4*>(a.v + o);
      pp[0] = p4.x; pp[1] = p4.y; pp[2] = p4.z; pp[3] = p4.w;
      mm[0] = m4.x; mm[1] = m4.y; mm[2] = m4.z; mm[3] = m4.w;
      vv[0] = v4.x; vv[1] = v4.y; vv[2] = v4.z; vv[3] = v4.w;
    } else {  // D % 4 != 0: columns past w are zeros (they stay put)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pp[j] = j < w ? a.p[o + j] : 0.f;
        mm[j] = j < w ? a.m[o + j] : 0.f;
        vv[j] = j < w ? a.v[o + j] : 0.f;
      }
    }
    adam_catch_row_f<4>(a.h, cw, lm, lp, t, pp, mm, vv);
    if (vec) {
      *reinterpret_cast<float4*>(a.p + o) = make_float4(pp[0], pp[1], pp[2], pp[3]);
      if (!p_only) {
        *reinterpret_cast<float4*>(a.m + o) = make_float4(mm[0], mm[1], mm[2], mm[3]);
        *reinterpret_cast<float4*>(a.v + o) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      }
    } else {
      for (int j = 0; j < w; ++j) {
        a.p[o + j] = pp[j];
        if (!p_only) { a.m[o + j] = mm[j]; a.v[o + j] = vv[j]; }
      }
    }
  }
}

// ---------------------------------------------------------------- segment sum (table gradient)
constexpr int kChunk = 64;
constexpr int kSegBatch = 16;  // positions whose contributions are loaded together
// partial flags (per chunk, then per block of 64 chunks): a run comes in over the left border
// (head partial), goes on over the right border too (through), or starts here and goes on
// (tail partial)
constexpr int kTail = 1, kHead = 2, kThrough = 4;

struct SegArgs {
  const uint32_t* keys;
  const uint32_t* vals;
  int64_t n;
  int bag;
  int mode;       // 0 one id per dout row, 1 mean bag, 2 sum bag
  int64_t pad;    // skipped row (no gradient), -1 none
  const float* dout;
  int64_t ldo;
  int D;
  float* grad;
  int accumulate;
  float* part;    // [nchunks][2][D]: head / tail partial of runs crossing chunk borders
  int* flags;     // [nchunks]: 1 = a run starts in this chunk and continues past it
  int nchunks;
  int* cnt;       // the fix kernel's ticket (after the flags; zeroed by segsum_kernel)
};

// agent-scope (sc1) accesses for the fix kernel's hand-off to its last workgroup (the fence-free
// form of MI355X_MICROARCH.md: sc1 stores, every storing wave drained, one agent-scope add per
// workgroup after a barrier, sc1 loads by the last adder -- no L2 write-back fence)
__device__ __forceinline__ float seg_ld(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int seg_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void seg_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void seg_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NV>  // columns per lane (D <= 64 * NV)
__device__ __forceinline__ void load_contrib(const SegArgs& a, uint32_t e, float inv, float* x) {
  const int64_t b = a.mode == 0 ? (int64_t)e : (int64_t)(e / (uint32_t)a.bag);
  const float* src = a.dout + b * a.ldo;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = lane + 64 * j;
    x[j] = c < a.D ? src[c] : 0.f;
  }
  if (a.mode == 1) {
#pragma unroll
    for (int j = 0; j < NV; ++j) x[j] = x[j] / inv;  // mean backward: grad / bag, per lookup
  }
}

template <int NV>
__device__ __forceinline__ void put_row(const SegArgs& a, int64_t row, const float* acc) {
  const int lane = threadIdx.x & 63;
  float* dst = a.grad + row * a.D;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = lane + 64 * j;
    if (c < a.D) dst[c] = a.accumulate ? dst[c] + acc[j] : acc[j];
  }
}

template <int NV, bool SC1 = false>
__device__ __forceinline__ void put_part(const SegArgs& a, int chunk, int which, const float* acc) {
  const int lane = threadIdx.x & 63;
  float* dst = a.part + ((int64_t)chunk * 2 + which) * a.D;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = lane + 64 * j;
    if (c < a.D) {
      if (SC1) seg_st(dst + c, acc[j]);
      else dst[c] = acc[j];
    }
  }
}

// Row of dout feeding lookup e (mode 0: one id per dout row; 1 / 2: a bag of `bag` ids).
__device__ __forceinline__ int64_t contrib_row(const SegArgs& a, uint32_t e) {
  return a.mode == 0 ? (int64_t)e : (int64_t)(e / (uint32_t)a.bag);
}

// One wave per chunk of 64 sorted positions.
//  * Singletons -- a row looked up exactly once (its run is one position; under uniform ids
//    nearly every position) -- are compacted through LDS and written in parallel: G lanes per
//    row with float4 loads of the dout row and a float4 store of the gradient row, 8 rows in
//    flight per lane group (the previous walk over positions one at a time was bound by its
//    per-position scalar instructions, 3,300 SALU + 2,300 VALU per wave).
//  * Longer runs (repeated rows, hot Zipf rows) are walked in position order as before, their
//    contributions loaded kSegBatch at a time; a run crossing the chunk border leaves a head or
//    tail partial for the fixup pass.
template <int NV, int G>
__device__ __forceinline__ void segsum_chunk(const SegArgs& a, int chunk, int2* slot) {
  const int lane = threadIdx.x & 63;
  const int64_t c0 = (int64_t)chunk * kChunk;
  const int cn = (int)(a.n - c0 < kChunk ? a.n - c0 : kChunk);
  const int64_t pi = c0 + lane;
  const uint32_t k = lane < cn ? a.keys[pi] : kSentinel;
  const uint32_t e = lane < cn ? a.vals[pi] : 0u;
  const uint32_t kp = pi > 0 && lane < cn ? a.keys[pi - 1] : kSentinel;
  const uint32_t kn = lane < cn && pi + 1 < a.n ? a.keys[pi + 1] : kSentinel;
  const bool valid = k != kSentinel && (int64_t)k != a.pad;
  const bool single = valid && kp != k && kn != k;
  const int brow = lane < cn ? (int)contrib_row(a, e) : 0;  // dout row of this lane's position
  const uint64_t smask = __ballot(single);
  const uint64_t mmask = __ballot(valid && !single);
  const float nbag = (float)a.bag;
  // ---- singletons
  if (smask) {
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    if (single) slot[__popcll(smask & lt)] = make_int2(brow, (int)k);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int ns = __popcll(smask);
    constexpr int R = 64 / G;  // rows per wave per round
    constexpr int U = 8;       // rounds in flight
    const int g = lane / G, gl = lane % G;
    const int c = gl * 4;
    for (int r0 = 0; r0 < ns; r0 += R * U) {
      float4 x[U];
      int2 sl[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = r0 + u * R + g;
        sl[u] = j < ns ? slot[j] : make_int2(-1, 0);
        x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (sl[u].x >= 0 && c < a.D)
          x[u] = *reinterpret_cast<const float4*>(a.dout + (int64_t)sl[u].x * a.ldo + c);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (sl[u].x < 0 || c >= a.D) continue;
        float4 v = x[u];
        if (a.mode == 1) { v.x = v.x / nbag; v.y = v.y / nbag; v.z = v.z / nbag; v.w = v.w / nbag; }
        float4* dst = reinterpret_cast<float4*>(a.grad + (int64_t)(uint32_t)sl[u].y * a.D + c);
        if (a.accumulate) {
          const float4 o = *dst;
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *dst = v;
      }
    }
  }
  int flag = 0;
  // ---- runs of two or more positions, in position order
  if (mmask) {
    const uint32_t kprev = c0 > 0 ? a.keys[c0 - 1] : kSentinel;
    const uint32_t knext = c0 + kChunk < a.n ? a.keys[c0 + kChunk] : kSentinel;
    float acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = 0.f;
    int first = -1;  // first position of the current run in this chunk
    uint64_t m = mmask;
    while (m) {
      int pos[kSegBatch];
      float x[kSegBatch][NV];
#pragma unroll
      for (int u = 0; u < kSegBatch; ++u) {
        pos[u] = m ? __ffsll((long long)m) - 1 : -1;
        if (m) m &= m - 1;
        // loaded unconditionally (position 0's row stands in past the end of the mask): a load
        // under a branch is waited for at the join
        const int64_t row = (int64_t)__builtin_amdgcn_readlane((int)brow, pos[u] >= 0 ? pos[u] : 0);
        const float* src = a.dout + row * a.ldo;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int cc = lane + 64 * j;
          x[u][j] = cc < a.D ? src[cc] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kSegBatch; ++u) {
        const int i = pos[u];
        if (i < 0) break;
        if (first < 0) first = i;
#pragma unroll
        for (int j = 0; j < NV; ++j) acc[j] += a.mode == 1 ? x[u][j] / nbag : x[u][j];
        const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)k, i);
        const uint32_t nk = (uint32_t)__builtin_amdgcn_readlane((int)kn, i);  // key after position i
        if (nk == key && i + 1 < cn) continue;  // the run goes on inside this chunk
        const bool head = first == 0 && kprev == key;   // began in an earlier chunk
        const bool tail = i + 1 == cn && knext == key;  // continues into the next chunk
        if (!head && !tail) put_row<NV>(a, key, acc);
        else if (head) {
          put_part<NV>(a, chunk, 0, acc);  // (also when it continues: "through")
          flag |= tail ? (kHead | kThrough) : kHead;
        } else {
          put_part<NV>(a, chunk, 1, acc);
          flag |= kTail;
        }
#pragma unroll
        for (int j = 0; j < NV; ++j) acc[j] = 0.f;
        first = -1;
      }
    }
  }
  if (lane == 0) a.flags[chunk] = flag;
}

// Runs crossing chunk borders, in two levels of fixed-order partial sums (a Zipf hot row spans
// hundreds to thousands of chunks; one wave walking them all was the longest step of the
// backward). Level 1: one wave per block of kFixBlock chunks walks their partials in order,
// stores the runs that start and end inside the block, and leaves a head / tail partial for the
// runs crossing the block's borders. Level 2: the block where such a run starts adds its tail
// partial and the following blocks' head partials. Both levels load their partials 16 at a time.
constexpr int kFixBatch = 16;
constexpr int kFixBlock = 16;  // chunks per level-1 block: one batch of loads per block wave

template <int NV, bool SC1 = false>
__device__ __forceinline__ void load_vec(const float* src, int D, float* v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < D ? (SC1 ? seg_ld(src + c) : src[c]) : 0.f;
  }
}

// SC1: the block partials and flags go out as agent-scope stores (the fused fix kernel's last
// workgroup reads them)
template <int NV, bool SC1 = false>
__device__ __forceinline__ void fix_block(const SegArgs& a, int blk) {
  const int nblk = (a.nchunks + kFixBlock - 1) / kFixBlock;
  if (blk >= nblk) return;
  const int lane = threadIdx.x & 63;
  const int j0 = blk * kFixBlock;
  const int nc = a.nchunks - j0 < kFixBlock ? a.nchunks - j0 : kFixBlock;
  const int fl = lane < nc ? a.flags[j0 + lane] : 0;
  // first / last key of every chunk of the block, loaded up front (not inside the ordered walk)
  const int64_t p0 = (int64_t)(j0 + lane) * kChunk;
  const uint32_t kfirst = fl ? a.keys[p0] : kSentinel;
  const uint32_t klast = fl ? a.keys[p0 + kChunk - 1 < a.n ? p0 + kChunk - 1 : a.n - 1] : kSentinel;
  const uint64_t any = __ballot(fl != 0);
  int bflag = 0;
  if (any) {
    float acc[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) acc[j] = 0.f;
    bool open = false, from_left = false;
    uint32_t key = kSentinel;
    uint64_t m = any;
    while (m) {
      int cj[kFixBatch];
      float hv[kFixBatch][NV], tv[kFixBatch][NV];
#pragma unroll
      for (int u = 0; u < kFixBatch; ++u) {
        cj[u] = m ? __ffsll((long long)m) - 1 : -1;
        if (m) m &= m - 1;
        // both partials of every chunk of the batch, unconditionally (a load under a branch
        // made the compiler wait for it at the join: one round trip per chunk)
        const int64_t c = j0 + (cj[u] >= 0 ? cj[u] : 0);
        load_vec<NV>(a.part + (c * 2) * a.D, a.D, hv[u]);
        load_vec<NV>(a.part + (c * 2 + 1) * a.D, a.D, tv[u]);
      }
#pragma unroll
      for (int u = 0; u < kFixBatch; ++u) {
        if (cj[u] < 0) break;
        const int f = __builtin_amdgcn_readlane(fl, cj[u]);
        if (f & kHead) {
          if (!open) {  // the run came in over the block's left border
            open = true;
            from_left = true;
            key = (uint32_t)__builtin_amdgcn_readlane((int)kfirst, cj[u]);
#pragma unroll
            for (int j = 0; j < NV; ++j) acc[j] = 0.f;
          }
#pragma unroll
          for (int j = 0; j < NV; ++j) acc[j] += hv[u][j];
          if (!(f & kThrough)) {  // ends in chunk c
            if (from_left) {
              put_part<NV, SC1>(a, a.nchunks + blk, 0, acc);
              bflag |= kHead;
            } else {
              put_row<NV>(a, key, acc);
            }
            open = false;
          }
        }
        if (f & kTail) {
          open = true;
          from_left = false;
          key = (uint32_t)__builtin_amdgcn_readlane((int)klast, cj[u]);
#pragma unroll
          for (int j = 0; j < NV; ++j) acc[j] = tv[u][j];
        }
      }
    }
    if (open) {  // continues over the block's right border
      if (from_left) {
        put_part<NV, SC1>(a, a.nchunks + blk, 0, acc);
        bflag |= kHead | kThrough;
      } else {
        put_part<NV, SC1>(a, a.nchunks + blk, 1, acc);
        bflag |= kTail;
      }
    }
  }
  if (lane == 0) {
    if (SC1) seg_st(a.flags + a.nchunks + blk, bflag);
    else a.flags[a.nchunks + blk] = bflag;
  }
}

template <int NV, bool SC1 = false>
__device__ __forceinline__ void fix_run(const SegArgs& a, int blk) {
  const int nblk = (a.nchunks + kFixBlock - 1) / kFixBlock;
  if (blk >= nblk) return;
  const int bf = SC1 ? seg_ld(a.flags + a.nchunks + blk) : a.flags[a.nchunks + blk];
  if (!(bf & kTail)) return;
  const int64_t lastpos = (int64_t)(blk * kFixBlock + kFixBlock - 1) * kChunk + kChunk - 1;
  const uint32_t key = a.keys[lastpos < a.n ? lastpos : a.n - 1];
  float acc[NV];
  load_vec<NV, SC1>(a.part + ((int64_t)(a.nchunks + blk) * 2 + 1) * a.D, a.D, acc);
  bool done = false;
  for (int b = blk + 1; b < nblk && !done; b += kFixBatch) {
    float h[kFixBatch][NV];
    int f[kFixBatch];
#pragma unroll
    for (int u = 0; u < kFixBatch; ++u) {
      const int bb = b + u < nblk ? b + u : nblk - 1;
      f[u] = SC1 ? seg_ld(a.flags + a.nchunks + bb) : a.flags[a.nchunks + bb];
      load_vec<NV, SC1>(a.part + ((int64_t)(a.nchunks + bb) * 2) * a.D, a.D, h[u]);
    }
#pragma unroll
    for (int u = 0; u < kFixBatch; ++u) {
      if (done || b + u >= nblk) { done = true; continue; }
#pragma unroll
      for (int j = 0; j < NV; ++j) acc[j] += h[u][j];
      if (!(f[u] & kThrough)) done = true;  // the run ends in block b + u
    }
  }
  put_row<NV>(a, key, acc);
}

template <int NV, int G>
__device__ __forceinline__ void segsum_body(const SegArgs& a, int bid, int2 (*slot)[64]) {
  if (bid == 0 && threadIdx.x == 0) *a.cnt = 0;  // the fix kernel's ticket
  const int chunk = bid * 4 + (threadIdx.x >> 6);
  if (chunk < a.nchunks) segsum_chunk<NV, G>(a, chunk, slot[threadIdx.x >> 6]);
}

template <int NV, int G>
__global__ __launch_bounds__(256) void segsum_kernel(SegArgs a) {
  __shared__ int2 slot[4][64];
  segsum_body<NV, G>(a, blockIdx.x, slot);
}

// Both fix levels in one launch (round 5): every wave runs level 1 for its block, the workgroups
// hand their block partials and flags to the last one to finish (agent-scope stores, one ticket),
// which runs level 2 for every block. Saves a launch per call (~4.5 us each on this box, three
// calls on C3's critical path).
struct FixLds {
  int s_last;
  int tails[256];
  int ntails;
};

// block bid of nb of one call's fix launch
template <int NV>
__device__ __forceinline__ void segsum_fix_body(const SegArgs& a, int bid, int nb, FixLds& L) {
  int& s_last = L.s_last;
  int* tails = L.tails;
  int& ntails = L.ntails;
  fix_block<NV, true>(a, bid * 4 + (threadIdx.x >> 6));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(a.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
  __syncthreads();
  if (!s_last) return;
  // level 2 in the last workgroup: only blocks whose run continues past their right border have
  // work. Their flags are read 256 at a time and the tail blocks listed in LDS first -- the waves
  // walking every block (fix_run's flag load, then its early return) was ~50 dependent round
  // trips per wave at C3's 200 history blocks. Each listed block writes its own run's row, so the
  // order the waves take them in does not matter.
  const int nblk = (a.nchunks + kFixBlock - 1) / kFixBlock;
  for (int b0 = 0; b0 < nblk; b0 += 256) {
    if (threadIdx.x == 0) ntails = 0;
    __syncthreads();
    const int b = b0 + (int)threadIdx.x;
    const int bf = b < nblk ? seg_ld(a.flags + a.nchunks + b) : 0;
    if (bf & kTail) tails[atomicAdd(&ntails, 1)] = b;
    __syncthreads();
    for (int i = threadIdx.x >> 6; i < ntails; i += 4) fix_run<NV, true>(a, tails[i]);
    __syncthreads();
  }
}

template <int NV>
__global__ __launch_bounds__(256) void segsum_fix_kernel(SegArgs a) {
  __shared__ FixLds L;
  segsum_fix_body<NV>(a, blockIdx.x, gridDim.x, L);
}

// several calls (different tables) in one segment-sum launch and one fix launch (round 5: C3's
// user tower, the 1M-row user-id table and the 10M-row history table, were two launch pairs back
// to back on the chain); each call's blocks, ticket and summation order are its own
constexpr int kSegCalls = 4;
struct SegBatch {
  SegArgs c[kSegCalls];
  int blk0[kSegCalls + 1];   // segsum blocks
  int fblk0[kSegCalls + 1];  // fix blocks
  int n;
};

template <int NV, int G>
__global__ __launch_bounds__(256) void segsum_batch_kernel(SegBatch b) {
  __shared__ int2 slot[4][64];
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.blk0[k + 1]) ++k;
  segsum_body<NV, G>(b.c[k], blockIdx.x - b.blk0[k], slot);
}

template <int NV>
__global__ __launch_bounds__(256) void segsum_fix_batch_kernel(SegBatch b) {
  __shared__ FixLds L;
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.fblk0[k + 1]) ++k;
  segsum_fix_body<NV>(b.c[k], blockIdx.x - b.fblk0[k], b.fblk0[k + 1] - b.fblk0[k], L);
}

AdamConst make_hyper(float b1, float b2, float eps, float wd) {
  AdamConst h;
  h.one_m_b1 = 1.f - b1; h.b2 = b2; h.one_m_b2 = 1.f - b2; h.eps = eps; h.wd = wd;
  return h;
}

// workspace: ping-pong keys + vals, then the [radix][tiles] histogram and digit totals
int64_t sort_ws_bytes(int64_t n, int64_t vocab) {
  if (n <= kRankMax) return (int64_t)cdiv(n, kRankBlock) * n * 4 + 256;  // the counting sort's partials
  const SortPlan p = make_plan(n, vocab);
  return 2 * n * 4 + ((int64_t)kMaxRadix * p.ntiles + kMaxRadix) * 4 + 256;
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int64_t rs_lookup_sort_ws_bytes(int64_t n, int64_t vocab) { return sort_ws_bytes(n, vocab); }

extern "C" int rs_lookup_sort(const void* ids, int id_bytes, int rows, int bag, int64_t row_stride,
                              int64_t vocab, uint32_t* keys, uint32_t* vals, void* ws, void* stream) {
  RS_CHECK_ARG(ids && keys && vals && rows >= 0 && bag >= 1 && row_stride >= bag &&
                   (id_bytes == 4 || id_bytes == 8) && vocab >= 1 && vocab < ((int64_t)1 << 31),
               "rs_lookup_sort: bad args");
  const int64_t n = (int64_t)rows * bag;
  RS_CHECK_ARG(n < ((int64_t)1 << 31), "rs_lookup_sort: %lld lookups exceed 2^31", (long long)n);
  if (n == 0) return 0;
  hipStream_t st = as_stream(stream);
  const SortPlan p = make_plan(n, vocab);
  // past one tile's keys, up to kRankMax: the counting sort (its partials in ws); round 5 measured it
  // no faster than the one-tile radix sort below kTileMax (10.4 + 6.6 us against ~18 us)
  if (n <= kRankMax && ws && n > kTileMax) {
    const int nb = (int)cdiv(n, kRankBlock);
    rank_partial_kernel<<<dim3(nb, nb), kRankBlock, 0, st>>>(ids, id_bytes, bag, row_stride, vocab, (int)n,
                                                              static_cast<int*>(ws));
    RS_CHECK_LAUNCH("rs_lookup_sort rank");
    rank_scatter_kernel<<<nb, 256, 0, st>>>(ids, id_bytes, bag, row_stride, vocab, (int)n, nb,
                                            static_cast<const int*>(ws), keys, vals);
    RS_CHECK_LAUNCH("rs_lookup_sort rank scatter");
    return 0;
  }
  if (n <= kTileMax) {  // without a workspace: one workgroup's radix passes
    sort_tile_kernel<<<1, kTileThreads, 0, st>>>(ids, id_bytes, bag, row_stride, vocab, (int)n, p, keys, vals);
    RS_CHECK_LAUNCH("rs_lookup_sort tile");
    return 0;
  }
  RS_CHECK_ARG(ws, "rs_lookup_sort: workspace needed for %lld lookups", (long long)n);
  uint32_t* tk = static_cast<uint32_t*>(ws);
  uint32_t* tv = tk + n;
  int* hist = reinterpret_cast<int*>(tv + n);
  int* tot = hist + (int64_t)kMaxRadix * p.ntiles;
  // ping-pong so that the last pass lands in (keys, vals)
  for (int q = 0; q < p.passes; ++q) {
    const bool to_out = ((p.passes - 1 - q) & 1) == 0;
    uint32_t* kd = to_out ? keys : tk;
    uint32_t* vd = to_out ? vals : tv;
    const uint32_t* ks = q == 0 ? nullptr : (to_out ? tk : keys);
    const uint32_t* vs = q == 0 ? nullptr : (to_out ? tv : vals);
    sort_hist_kernel<<<p.ntiles, kSortThreads, 0, st>>>(ids, id_bytes, bag, row_stride, vocab, ks, n,
                                                        p.shift[q], p.dbits[q], hist);
    RS_CHECK_LAUNCH("rs_lookup_sort hist");
    sort_scan_kernel<<<1 << p.dbits[q], 256, 0, st>>>(hist, p.ntiles, tot);
    RS_CHECK_LAUNCH("rs_lookup_sort scan");
    sort_scatter_kernel<<<p.ntiles, kSortThreads, 0, st>>>(ids, id_bytes, bag, row_stride, vocab, ks,
                                                           vs, n, p.shift[q], p.dbits[q], hist, tot,
                                                           kd, vd);
    RS_CHECK_LAUNCH("rs_lookup_sort scatter");
  }
  return 0;
}

static int sorted_rows(int op, const uint32_t* keys, int64_t n, int D, float* p, float* g, float* m,
                       float* v, int* last, int* owner, int call, const int64_t* step,
                       const float* consts, float b1, float b2, float eps, float wd, float scale,
                       const float* coef, double* ws, hipStream_t st) {
  if (n == 0 && op != kSqnorm) return 0;
  RowArgs a;
  a.keys = keys; a.n = n; a.D = D; a.p = p; a.g = g; a.m = m; a.v = v; a.last = last;
  a.owner = owner; a.call = call; a.step = step;
  a.consts = reinterpret_cast<const float2*>(consts); a.h = make_hyper(b1, b2, eps, wd);
  a.scale = scale; a.coef = coef; a.ws = ws;
  // lanes per row: 4 columns each, a power of two in [4, 64]
  const int G = D <= 16 ? 4 : D <= 32 ? 8 : D <= 64 ? 16 : D <= 128 ? 32 : 64;
  const int grid = op == kSqnorm ? kRowGrid
                                 : std::max<int64_t>(1, std::min<int64_t>(kRowGrid * 4, cdiv(n, 256 / G * kRowUnroll)));
#define RS_ROWS_U(OPV, UV)                                                        \
  switch (G) {                                                                    \
    case 4: sorted_rows_kernel<OPV, 4, UV><<<grid, 256, 0, st>>>(a); break;        \
    case 8: sorted_rows_kernel<OPV, 8, UV><<<grid, 256, 0, st>>>(a); break;        \
    case 16: sorted_rows_kernel<OPV, 16, UV><<<grid, 256, 0, st>>>(a); break;      \
    case 32: sorted_rows_kernel<OPV, 32, UV><<<grid, 256, 0, st>>>(a); break;      \
    default: sorted_rows_kernel<OPV, 64, UV><<<grid, 256, 0, st>>>(a); break;      \
  }
#define RS_ROWS(OPV) RS_ROWS_U(OPV, kRowUnroll)
  switch (op) {
    case kCatchup: RS_ROWS(kCatchup) break;
    case kAdam: RS_ROWS(kAdam) break;
    case kSqnorm: RS_ROWS_U(kSqnorm, kSqUnroll) break;
    case kOwner: RS_ROWS(kOwner) break;
    default: RS_ROWS(kZero) break;
  }
#undef RS_ROWS_U
#undef RS_ROWS
  RS_CHECK_LAUNCH("rs_sorted_rows");
  return 0;
}

extern "C" int rs_sorted_catchup(const uint32_t* keys, int64_t n, int D, float* p, float* m, float* v,
                                 int* last, const int64_t* step, const float* consts, float beta1,
                                 float beta2, float eps, float weight_decay, void* stream) {
  RS_CHECK_ARG(keys && p && m && v && last && step && consts && D >= 1 && n >= 0,
               "rs_sorted_catchup: bad args");
  return sorted_rows(kCatchup, keys, n, D, p, nullptr, m, v, last, nullptr, 0, step, consts, beta1,
                     beta2, eps, weight_decay, 1.f, nullptr, nullptr, as_stream(stream));
}

extern "C" int rs_lookup_catchup(const void* ids, int id_bytes, int rows, int bag, int64_t row_stride,
                                 int64_t vocab, int D, float* p, float* m, float* v, int* last,
                                 const int64_t* step, const float* consts, float beta1, float beta2,
                                 float eps, float weight_decay, void* stream) {
  RS_CHECK_ARG(ids && p && m && v && last && step && consts && D >= 1 && rows >= 0 && bag >= 1 &&
                   row_stride >= bag && (id_bytes == 4 || id_bytes == 8) && vocab >= 1 &&
                   vocab < ((int64_t)1 << 31),
               "rs_lookup_catchup: bad args");
  const int64_t n = (int64_t)rows * bag;
  if (n == 0) return 0;
  IdCatchArgs a;
  a.ids = ids; a.id_bytes = id_bytes; a.bag = bag; a.stride = row_stride; a.vocab = vocab; a.n = n;
  a.D = D; a.p = p; a.m = m; a.v = v; a.last = last; a.step = step;
  a.consts = reinterpret_cast<const float2*>(consts);
  a.h = make_hyper(beta1, beta2, eps, weight_decay);
  const int G = D <= 16 ? 4 : D <= 32 ? 8 : D <= 64 ? 16 : D <= 128 ? 32 : 64;
  RS_CHECK_ARG(D <= 4 * G, "rs_lookup_catchup: D %d > 256", D);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(kRowGrid * 4, cdiv(n, 256 / G)));
  hipStream_t st = as_stream(stream);
  switch (G) {
    case 4: lookup_catchup_kernel<4><<<grid, 256, 0, st>>>(a); break;
    case 8: lookup_catchup_kernel<8><<<grid, 256, 0, st>>>(a); break;
    case 16: lookup_catchup_kernel<16><<<grid, 256, 0, st>>>(a); break;
    case 32: lookup_catchup_kernel<32><<<grid, 256, 0, st>>>(a); break;
    default: lookup_catchup_kernel<64><<<grid, 256, 0, st>>>(a); break;
  }
  RS_CHECK_LAUNCH("rs_lookup_catchup");
  return 0;
}

extern "C" int rs_sorted_adam(const uint32_t* keys, int64_t n, int D, float* p, float* g, float* m,
                              float* v, int* last, int* owner, int call, const int64_t* step,
                              const float* consts, float beta1, float beta2, float eps,
                              float weight_decay, float scale, const float* coef, void* stream) {
  RS_CHECK_ARG(keys && p && g && m && v && last && step && consts && D >= 1 && n >= 0,
               "rs_sorted_adam: bad args");
  return sorted_rows(kAdam, keys, n, D, p, g, m, v, last, owner, call, step, consts, beta1, beta2,
                     eps, weight_decay, scale, coef, nullptr, as_stream(stream));
}

static int lanes_per_row(int D) { return D <= 16 ? 4 : D <= 32 ? 8 : D <= 64 ? 16 : D <= 128 ? 32 : 64; }

static int sorted_rows_batch(int op, const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                             const float* consts, float b1, float b2, float eps, float wd, float scale,
                             const float* coef, double* ws, hipStream_t st, const DensePart* dense = nullptr) {
  RS_CHECK_ARG(calls && ncalls >= 1 && ncalls <= kRowBatchMax, "rs_sorted_*_batch: 1 .. %d calls (got %d)",
               kRowBatchMax, ncalls);
  RowBatch b{};
  b.n = ncalls;
  if (dense && dense->n > 0) {
    b.d = *dense;
    b.d.blocks = op == kSqnorm ? dense_sq_blocks(dense->n) : dense_adam_blocks(dense->n);
  }
  const int G = lanes_per_row(calls[0].D);
  int wg = 0;
  for (int c = 0; c < ncalls; ++c) {
    const rs_sorted_call_t& k = calls[c];
    RS_CHECK_ARG(k.keys && (k.g || op == kCatchup) && k.D >= 1 && k.n >= 0 && lanes_per_row(k.D) == G,
                 "rs_sorted_*_batch: call %d: bad args or another row width class than call 0", c);
    RS_CHECK_ARG((op != kAdam && op != kCatchup) || (k.p && k.m && k.v && k.last),
                 "rs_sorted_adam_batch / rs_sorted_catchup_batch: call %d: null state", c);
    RowArgs& a = b.a[c];
    a.keys = k.keys; a.n = k.n; a.D = k.D; a.p = k.p; a.g = k.g; a.m = k.m; a.v = k.v; a.last = k.last;
    a.owner = k.owner; a.call = k.call; a.step = step;
    a.consts = reinterpret_cast<const float2*>(consts); a.h = make_hyper(b1, b2, eps, wd);
    a.scale = scale; a.coef = coef; a.ws = ws ? ws + (int64_t)c * kRowGrid : nullptr;
    b.first[c] = wg;
    wg += op == kSqnorm ? kRowGrid : (int)std::max<int64_t>(1, std::min<int64_t>(kRowGrid * 4, cdiv(k.n, 256 / G)));
  }
  b.first[ncalls] = wg;
  wg += b.d.blocks;
#define RS_BATCH(OPV)                                                                        \
  switch (G) {                                                                               \
    case 4: sorted_rows_batch_kernel<OPV, 4, OPV == kSqnorm ? kSqUnroll : 1><<<wg, 256, 0, st>>>(b); break;               \
    case 8: sorted_rows_batch_kernel<OPV, 8, OPV == kSqnorm ? kSqUnroll : 1><<<wg, 256, 0, st>>>(b); break;               \
    case 16: sorted_rows_batch_kernel<OPV, 16, OPV == kSqnorm ? kSqUnroll : 1><<<wg, 256, 0, st>>>(b); break;             \
    case 32: sorted_rows_batch_kernel<OPV, 32, OPV == kSqnorm ? kSqUnroll : 1><<<wg, 256, 0, st>>>(b); break;             \
    default: sorted_rows_batch_kernel<OPV, 64, OPV == kSqnorm ? kSqUnroll : 1><<<wg, 256, 0, st>>>(b); break;             \
  }
  if (op == kAdam) {
    RS_BATCH(kAdam)
  } else if (op == kCatchup) {
    RS_BATCH(kCatchup)
  } else {
    RS_BATCH(kSqnorm)
  }
#undef RS_BATCH
  RS_CHECK_LAUNCH("rs_sorted_rows_batch");
  return 0;
}

// The forward catch-up of several sorted calls (tables) in one launch (round 6: C3's user side ran the
// history table's and the user-id table's catch-ups as two launches back to back on one queue)
extern "C" int rs_sorted_catchup_batch(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                                       const float* consts, float beta1, float beta2, float eps,
                                       float weight_decay, void* stream) {
  RS_CHECK_ARG(step && consts, "rs_sorted_catchup_batch: null pointer");
  return sorted_rows_batch(kCatchup, calls, ncalls, step, consts, beta1, beta2, eps, weight_decay, 1.f, nullptr,
                           nullptr, as_stream(stream));
}

extern "C" int rs_sorted_adam_batch(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                                    const float* consts, float beta1, float beta2, float eps, float weight_decay,
                                    float scale, const float* coef, void* stream) {
  RS_CHECK_ARG(step && consts, "rs_sorted_adam_batch: null pointer");
  return sorted_rows_batch(kAdam, calls, ncalls, step, consts, beta1, beta2, eps, weight_decay, scale, coef,
                           nullptr, as_stream(stream));
}

extern "C" int rs_sorted_adam_batch_dense(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                                          const float* consts, float beta1, float beta2, float eps,
                                          float weight_decay, float scale, const float* coef, float* p, float* g,
                                          float* m, float* v, int64_t n, float lr, void* stream) {
  RS_CHECK_ARG(step && consts && n >= 0 && (n == 0 || (p && g && m && v)), "rs_sorted_adam_batch_dense: bad args");
  DensePart d{};
  d.p = p; d.g = g; d.m = m; d.v = v; d.n = n; d.lr = lr; d.b1 = beta1; d.b2 = beta2;
  d.h = make_hyper(beta1, beta2, eps, weight_decay);
  return sorted_rows_batch(kAdam, calls, ncalls, step, consts, beta1, beta2, eps, weight_decay, scale, coef,
                           nullptr, as_stream(stream), &d);
}

extern "C" int rs_sorted_sqnorm_batch_dense(const rs_sorted_call_t* calls, int ncalls, float scale, double* ws,
                                            const float* g, int64_t n, double* ws_dense, void* stream) {
  RS_CHECK_ARG(ws && n >= 0 && (n == 0 || (g && ws_dense)), "rs_sorted_sqnorm_batch_dense: bad args");
  DensePart d{};
  d.g = const_cast<float*>(g); d.n = n; d.ws = ws_dense;
  return sorted_rows_batch(kSqnorm, calls, ncalls, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, scale, nullptr, ws,
                           as_stream(stream), &d);
}

extern "C" int rs_sorted_sqnorm_batch(const rs_sorted_call_t* calls, int ncalls, float scale, double* ws,
                                      void* stream) {
  RS_CHECK_ARG(ws, "rs_sorted_sqnorm_batch: null ws");
  return sorted_rows_batch(kSqnorm, calls, ncalls, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, scale, nullptr, ws,
                           as_stream(stream));
}

extern "C" int rs_sorted_sqnorm_parts(void) { return kRowGrid; }

extern "C" int rs_sorted_sqnorm(const uint32_t* keys, int64_t n, int D, const float* g, int* owner,
                                int call, float scale, double* ws, void* stream) {
  RS_CHECK_ARG(keys && g && ws && D >= 1 && n >= 0, "rs_sorted_sqnorm: bad args");
  return sorted_rows(kSqnorm, keys, n, D, nullptr, const_cast<float*>(g), nullptr, nullptr, nullptr,
                     owner, call, nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, scale, nullptr, ws,
                     as_stream(stream));
}

extern "C" int rs_sorted_owner(const uint32_t* keys, int64_t n, int* owner, int call, void* stream) {
  RS_CHECK_ARG(keys && owner && n >= 0, "rs_sorted_owner: bad args");
  return sorted_rows(kOwner, keys, n, 1, nullptr, nullptr, nullptr, nullptr, nullptr, owner, call,
                     nullptr, nullptr, 0.f, 0.f, 0.f, 0.f, 1.f, nullptr, nullptr, as_stream(stream));
}

extern "C" int rs_sorted_zero_grad(const uint32_t* keys, int64_t n, int D, float* g, void* stream) {
  RS_CHECK_ARG(keys && g && D >= 1 && n >= 0, "rs_sorted_zero_grad: bad args");
  return sorted_rows(kZero, keys, n, D, nullptr, g, nullptr, nullptr, nullptr, nullptr, 0, nullptr,
                     nullptr, 0.f, 0.f, 0.f, 0.f, 1.f, nullptr, nullptr, as_stream(stream));
}

extern "C" int64_t rs_segsum_ws_bytes(int64_t n, int D) {
  const int64_t nc = (n + kChunk - 1) / kChunk;
  const int64_t np = nc + (nc + kFixBlock - 1) / kFixBlock;  // chunk partials, then block partials
  return np * 2 * D * 4 + np * 4 + 256;
}

extern "C" int rs_segsum(const uint32_t* keys, const uint32_t* vals, int64_t n, int bag, int mode,
                         int64_t pad, const float* dout, int64_t ldo, int D, float* grad,
                         int accumulate, void* ws, void* stream) {
  RS_CHECK_ARG(keys && vals && dout && grad && ws && n >= 0 && bag >= 1 && mode >= 0 && mode <= 2 &&
                   D >= 1 && D <= 256 && ldo >= D,
               "rs_segsum: bad args");
  if (n == 0) return 0;
  RS_CHECK_ARG(n < ((int64_t)1 << 31), "rs_segsum: n too large");
  SegArgs a;
  a.keys = keys; a.vals = vals; a.n = n; a.bag = bag; a.mode = mode; a.pad = pad; a.dout = dout;
  a.ldo = ldo; a.D = D; a.grad = grad; a.accumulate = accumulate;
  a.nchunks = cdiv(n, kChunk);
  a.part = static_cast<float*>(ws);
  const int64_t np = a.nchunks + (a.nchunks + kFixBlock - 1) / kFixBlock;
  a.flags = reinterpret_cast<int*>(a.part + np * 2 * D);
  a.cnt = a.flags + np;  // inside rs_segsum_ws_bytes' 256-byte tail
  hipStream_t st = as_stream(stream);
  const int grid = cdiv(a.nchunks, 4);
  RS_CHECK_ARG(D % 4 == 0 && ldo % 4 == 0 && aligned16(dout) && aligned16(grad),
               "rs_segsum: D, ldo multiples of 4 and 16-byte aligned dout / grad required");
  const int bgrid = cdiv(cdiv(a.nchunks, kFixBlock), 4);
#define RS_SEGSUM(NV, G)                                               \
  segsum_kernel<NV, G><<<grid, 256, 0, st>>>(a);                       \
  RS_CHECK_LAUNCH("rs_segsum");                                        \
  segsum_fix_kernel<NV><<<bgrid, 256, 0, st>>>(a);                     \
  RS_CHECK_LAUNCH("rs_segsum fix");
  if (D <= 16) { RS_SEGSUM(1, 4) }
  else if (D <= 32) { RS_SEGSUM(1, 8) }
  else if (D <= 64) { RS_SEGSUM(1, 16) }
  else if (D <= 128) { RS_SEGSUM(2, 32) }
  else { RS_SEGSUM(4, 64) }
#undef RS_SEGSUM
  return 0;
}

extern "C" int rs_segsum_batch(const rs_segsum_call_t* calls, int ncalls, int D, void* stream) {
  RS_CHECK_ARG(calls && ncalls >= 1 && ncalls <= kSegCalls && D >= 1 && D <= 256 && D % 4 == 0,
               "rs_segsum_batch: bad args (ncalls %d, D %d)", ncalls, D);
  SegBatch b{};
  int blk = 0, fblk = 0;
  for (int i = 0; i < ncalls; ++i) {
    const rs_segsum_call_t& c = calls[i];
    RS_CHECK_ARG(c.keys && c.vals && c.dout && c.grad && c.ws && c.n >= 1 && c.n < ((int64_t)1 << 31) &&
                     c.bag >= 1 && c.mode >= 0 && c.mode <= 2 && c.ldo >= D && c.ldo % 4 == 0 &&
                     aligned16(c.dout) && aligned16(c.grad),
                 "rs_segsum_batch: bad call %d", i);
    for (int j = 0; j < i; ++j)
      RS_CHECK_ARG(calls[j].grad != c.grad, "rs_segsum_batch: calls %d and %d write one table", j, i);
    SegArgs& a = b.c[i];
    a.keys = c.keys; a.vals = c.vals; a.n = c.n; a.bag = c.bag; a.mode = c.mode; a.pad = c.pad; a.dout = c.dout;
    a.ldo = c.ldo; a.D = D; a.grad = c.grad; a.accumulate = c.accumulate;
    a.nchunks = cdiv(c.n, kChunk);
    a.part = static_cast<float*>(c.ws);
    const int64_t np = a.nchunks + (a.nchunks + kFixBlock - 1) / kFixBlock;
    a.flags = reinterpret_cast<int*>(a.part + np * 2 * D);
    a.cnt = a.flags + np;
    b.blk0[i] = blk;
    b.fblk0[i] = fblk;
    blk += cdiv(a.nchunks, 4);
    fblk += cdiv(cdiv(a.nchunks, kFixBlock), 4);
  }
  b.blk0[ncalls] = blk;
  b.fblk0[ncalls] = fblk;
  b.n = ncalls;
  hipStream_t st = as_stream(stream);
#define RS_SEGSUM_B(NV, G)                                     \
  segsum_batch_kernel<NV, G><<<blk, 256, 0, st>>>(b);          \
  RS_CHECK_LAUNCH("rs_segsum_batch");                          \
  segsum_fix_batch_kernel<NV><<<fblk, 256, 0, st>>>(b);        \
  RS_CHECK_LAUNCH("rs_segsum_batch fix");
  if (D <= 16) { RS_SEGSUM_B(1, 4) }
  else if (D <= 32) { RS_SEGSUM_B(1, 8) }
  else if (D <= 64) { RS_SEGSUM_B(1, 16) }
  else if (D <= 128) { RS_SEGSUM_B(2, 32) }
  else { RS_SEGSUM_B(4, 64) }
#undef RS_SEGSUM_B
  return 0;
}

// ---------------------------------------------------------------- data-parallel exchange packing
// The data-parallel exchange of a large table (dist.py) all-gathers, per lookup call, the ids as
// int32 [rows, bag] and the call's output gradient [rows, D]; every rank then sorts the gathered
// ids and runs rs_segsum over them (identical inputs -> bitwise identical gradients on every rank).
namespace rs {
namespace {
__global__ void pack_ids_kernel(const void* __restrict__ ids, int id_bytes, int64_t rows, int bag,
                                int64_t stride, int32_t* __restrict__ out) {
  const int64_t n = rows * bag;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / bag, l = e - r * bag;
    out[e] = id_bytes == 8 ? (int32_t) static_cast<const int64_t*>(ids)[r * stride + l]
                           : static_cast<const int32_t*>(ids)[r * stride + l];
  }
}

__global__ void pack_rows_kernel(const float* __restrict__ src, int64_t ld, int64_t rows, int D,
                                 float* __restrict__ dst) {
  const int64_t n = rows * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    dst[e] = src[r * ld + (e - r * D)];
  }
}
}  // namespace
}  // namespace rs

// Row-sharded tables (flat.py / dist.py): rank `rank` of `world` owns the rows id % world ==
// rank, stored at local row id / world. Maps the all-gathered int32 ids of a lookup call to local
// rows (int64, -1 where another rank owns the row: the gather reads it as 0 and the sort puts it
// last); out-of-range ids raise the error flag as the gather would, except INT32_MIN, the pad
// slot of a ragged call's exchange (dist.EMPTY_ID).
constexpr int32_t kEmptyId = INT32_MIN;  // dist.EMPTY_ID
__global__ void shard_map_kernel(const int32_t* __restrict__ ids, int64_t n, int64_t V, int world, int rank,
                                 int64_t* __restrict__ local, int* err) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t id = ids[i];
    const bool ok = id >= 0 && id < V;
    bad |= !ok && id != kEmptyId;  // kEmptyId: an exchange pad slot (ragged calls), not an id
    local[i] = ok && id % world == rank ? id / world : -1;
  }
  if (bad && err) atomicOr(err, 1);
}

extern "C" int rs_shard_map_ids(const int32_t* ids, int64_t n, int64_t vocab, int world, int rank,
                                int64_t* local, int* err_flag, void* stream) {
  RS_CHECK_ARG(ids && local && n >= 0 && vocab >= 1 && world >= 1 && rank >= 0 && rank < world,
               "rs_shard_map_ids: bad args");
  if (n == 0) return 0;
  shard_map_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, as_stream(stream)>>>(ids, n, vocab, world,
                                                                                            rank, local, err_flag);
  RS_CHECK_LAUNCH("rs_shard_map_ids");
  return 0;
}

// max-pooled bag backward as per-lookup gradient rows (data parallel: the arg-max scatter's
// contributions exchanged like single-id lookups): out[r * bag + l][c] = dout[r][c] where l is
// the first position of bag r whose row holds the bag's maximum in column c (torch.max(dim)'s
// backward, as gather_bwd's RS_POOL_MAX scatter), 0 elsewhere and for the padding row / invalid
// ids. One thread per (bag, column).
__global__ __launch_bounds__(256) void pool_max_grad_kernel(const float* __restrict__ table, const void* ids,
                                                            int id_bytes, int64_t rows, int bag, int64_t stride,
                                                            int64_t vocab, int D, int64_t pad,
                                                            const float* __restrict__ dout, int64_t ldo,
                                                            float* __restrict__ out) {
  const int64_t n = rows * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D;
    const int c = (int)(i - r * D);
    float best = -INFINITY;
    int arg = -1;
    for (int l = 0; l < bag; ++l) {
      const int64_t e = r * stride + l;
      const int64_t id = id_bytes == 8 ? static_cast<const int64_t*>(ids)[e] : static_cast<const int32_t*>(ids)[e];
      const float v = id >= 0 && id < vocab ? table[id * D + c] : 0.f;
      if (v > best || arg < 0) {
        best = v;
        arg = l;
      }
    }
    const float g = dout[r * ldo + c];
    for (int l = 0; l < bag; ++l) {
      const int64_t e = r * stride + l;
      const int64_t id = id_bytes == 8 ? static_cast<const int64_t*>(ids)[e] : static_cast<const int32_t*>(ids)[e];
      const bool take = l == arg && id >= 0 && id < vocab && id != pad;
      out[(r * bag + l) * D + c] = take ? g : 0.f;
    }
  }
}

extern "C" int rs_pool_max_grad(const float* table, const void* ids, int id_bytes, int64_t rows, int bag,
                                int64_t row_stride, int64_t vocab, int D, int64_t pad, const float* dout,
                                int64_t ldo, float* out, void* stream) {
  RS_CHECK_ARG(table && ids && dout && out && rows >= 0 && bag >= 1 && row_stride >= bag && vocab >= 1 &&
                   D >= 1 && ldo >= D && (id_bytes == 4 || id_bytes == 8),
               "rs_pool_max_grad: bad args");
  const int64_t n = rows * D;
  if (n == 0) return 0;
  pool_max_grad_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, as_stream(stream)>>>(
      table, ids, id_bytes, rows, bag, row_stride, vocab, D, pad, dout, ldo, out);
  RS_CHECK_LAUNCH("rs_pool_max_grad");
  return 0;
}

extern "C" int rs_pack_ids(const void* ids, int id_bytes, int64_t rows, int bag, int64_t row_stride,
                           int32_t* out, void* stream) {
  RS_CHECK_ARG(ids && out && rows >= 0 && bag >= 1 && row_stride >= bag &&
                   (id_bytes == 4 || id_bytes == 8),
               "rs_pack_ids: bad args");
  const int64_t n = rows * bag;
  if (n == 0) return 0;
  pack_ids_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, as_stream(stream)>>>(
      ids, id_bytes, rows, bag, row_stride, out);
  RS_CHECK_LAUNCH("rs_pack_ids");
  return 0;
}

extern "C" int rs_pack_rows(const float* src, int64_t ld, int64_t rows, int D, float* dst,
                            void* stream) {
  RS_CHECK_ARG(src && dst && rows >= 0 && D >= 1 && ld >= D, "rs_pack_rows: bad args");
  const int64_t n = rows * D;
  if (n == 0) return 0;
  pack_rows_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, as_stream(stream)>>>(
      src, ld, rows, D, dst);
  RS_CHECK_LAUNCH("rs_pack_rows");
  return 0;
}
