// Row-sharded large tables, all-to-all exchange (flat.py LazyTable.shard_lookup_a2a, dist.py).
//
// Under data parallelism rank r owns the rows id % W == r (at local row id / W). A lookup call
// whose ids are one per output row (a single-id feature, or the per-token history of the
// sequence encoder: SURVEY §8f.4, C5) exchanges ROWS only for the distinct ids each rank needs:
//   requester: sort the call's ids (rs_lookup_sort) -> keys / vals;
//              rs_shard_bucket: the distinct ids per owner, packed in fixed-capacity buckets
//              [W][cap] (all_to_all_single with equal splits: no host sync, graph-capturable),
//              the compact slot o * cap + s of every lookup (idx, in lookup order: the forward
//              gather reads the returned rows through it) and of every sorted position (ckey:
//              the backward segment sum writes the gradient of each distinct id into its slot);
//   owner    : rs_shard_recv: the received local rows, as gather ids (invalid slots -> row 0)
//              and as sort ids (invalid -> out of range, i.e. last and skipped), sorted into the
//              owner's lookup call (catch-up, segment sum of the returned gradients, Adam).
// Per-rank work and traffic are O(the call's distinct ids), independent of W, against the
// all-gather / reduce-scatter form's O(W x rows) (kept for pooled bags, whose partial sums are
// one row per bag).
#include "common.h"

namespace rs {
namespace {

constexpr uint32_t kSentinel = 0xFFFFFFFFu;
constexpr int kBT = 1024;       // positions per block
constexpr int kBW = kBT / 64;   // waves per block
constexpr int kMaxWorld = 64;

__device__ __forceinline__ bool is_head(const uint32_t* keys, int64_t i, uint32_t k) {
  return k != kSentinel && (i == 0 || keys[i - 1] != k);
}

// per block: the number of distinct ids (run heads) per owner
__global__ __launch_bounds__(kBT) void shard_count_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                          int W, int* __restrict__ block_counts) {
  __shared__ int cnt[kMaxWorld];
  if (threadIdx.x < W) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = blockIdx.x * (int64_t)kBT + threadIdx.x;
  if (i < n) {
    const uint32_t k = keys[i];
    if (is_head(keys, i, k)) atomicAdd(&cnt[k % (uint32_t)W], 1);  // LDS integer count
  }
  __syncthreads();
  if (threadIdx.x < W) block_counts[(int64_t)blockIdx.x * W + threadIdx.x] = cnt[threadIdx.x];
}

// one workgroup: per owner, the exclusive prefix of the block counts over the blocks, and the
// totals (capped at cap; the overflow flag when a bucket is too small)
__global__ __launch_bounds__(kBT) void shard_scan_kernel(const int* __restrict__ block_counts, int nb, int W,
                                                         int cap, int* __restrict__ block_base,
                                                         int* __restrict__ counts, int* __restrict__ flag) {
  __shared__ int part[kBT];
  const int t = threadIdx.x;
  const int per = (nb + kBT - 1) / kBT;
  const int b0 = t * per, b1 = min(nb, b0 + per);
  for (int o = 0; o < W; ++o) {
    int s = 0;
    for (int b = b0; b < b1; ++b) s += block_counts[(int64_t)b * W + o];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < kBT; off <<= 1) {  // inclusive Hillis-Steele scan of the thread sums
      const int v = t >= off ? part[t - off] : 0;
      __syncthreads();
      part[t] += v;
      __syncthreads();
    }
    int run = part[t] - s;  // exclusive prefix of this thread's chunk
    for (int b = b0; b < b1; ++b) {
      block_base[(int64_t)b * W + o] = run;
      run += block_counts[(int64_t)b * W + o];
    }
    if (t == kBT - 1) {
      const int total = part[t];
      counts[o] = total < cap ? total : cap;
      if (total > cap && flag) atomicOr(flag, 2);
    }
    __syncthreads();
  }
}

// per block: each distinct id's slot in its owner's bucket (block base + earlier waves + rank in
// the wave, in key order), the bucket entry (the owner's local row) and comp[i] = o * cap + slot
// (-1 past the capacity) at the run head
__global__ __launch_bounds__(kBT) void shard_assign_kernel(const uint32_t* __restrict__ keys, int64_t n, int W,
                                                           int cap, const int* __restrict__ block_base,
                                                           int32_t* __restrict__ send_ids,
                                                           int* __restrict__ comp) {
  __shared__ int wcnt[kBW][kMaxWorld];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t i = blockIdx.x * (int64_t)kBT + threadIdx.x;
  const uint32_t k = i < n ? keys[i] : kSentinel;
  const bool head = i < n && is_head(keys, i, k);
  const int own = head ? (int)(k % (uint32_t)W) : -1;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int rank = 0;
  for (int o = 0; o < W; ++o) {
    const uint64_t m = __ballot(own == o);
    if (own == o) rank = __popcll(m & lt);
    if (lane == 0) wcnt[wave][o] = __popcll(m);
  }
  __syncthreads();
  if (head) {
    int slot = block_base[(int64_t)blockIdx.x * W + own] + rank;
    for (int w = 0; w < wave; ++w) slot += wcnt[w][own];
    if (slot < cap) {
      const int c = own * cap + slot;
      send_ids[c] = (int32_t)(k / (uint32_t)W);
      comp[i] = c;
    } else {
      comp[i] = -1;
    }
  }
}

// lower_bound of key k in keys[0, hi): the head of k's run
__device__ __forceinline__ int64_t run_head(const uint32_t* keys, int64_t hi, uint32_t k) {
  int64_t lo = 0;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// every sorted position: the gather index of its lookup (lookup order) and its segment-sum key
// (sorted order; padding / out-of-range / overflowed -> sentinel, no gradient). A lookup whose id
// is out of range or overflowed its owner's bucket reads `zrow`, the zero row the requester keeps
// after the returned buckets -- never another id's row (both are flagged and raise at the next
// check_errors)
__global__ __launch_bounds__(256) void shard_fill_kernel(const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, int64_t n,
                                                         int64_t pad, const int* __restrict__ comp, int64_t zrow,
                                                         int64_t* __restrict__ idx, uint32_t* __restrict__ ckey,
                                                         int* __restrict__ flag) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    const uint32_t e = vals[i];
    if (k == kSentinel) {  // out-of-range id: the reference's IndexError (flagged; reads zeros)
      bad = true;
      idx[e] = zrow;
      ckey[i] = kSentinel;
      continue;
    }
    const int64_t h = is_head(keys, i, k) ? i : run_head(keys, i, k);
    const int c = comp[h];
    idx[e] = c < 0 ? zrow : c;
    ckey[i] = (c < 0 || (int64_t)k == pad) ? kSentinel : (uint32_t)c;
  }
  if (bad && flag) atomicOr(flag, 1);
}

// owner side: bucket entries past the sender's count are not ids
__global__ __launch_bounds__(256) void shard_recv_kernel(const int32_t* __restrict__ recv_ids,
                                                         const int* __restrict__ recv_counts, int W, int cap,
                                                         int64_t vocab, int64_t* __restrict__ ids64,
                                                         int32_t* __restrict__ ids32, int* __restrict__ flag) {
  const int64_t n = (int64_t)W * cap;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(i / cap), s = (int)(i - (int64_t)o * cap);
    const int32_t id = recv_ids[i];
    const bool valid = s < recv_counts[o];
    const bool ok = valid && id >= 0 && id < vocab;
    bad |= valid && !ok;
    ids64[i] = ok ? id : 0;
    ids32[i] = ok ? id : (int32_t)vocab;  // out of range: sorted last as the sentinel
  }
  if (bad && flag) atomicOr(flag, 1);
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int64_t rs_shard_bucket_ws_bytes(int64_t n, int world) {
  const int64_t nb = (n + kBT - 1) / kBT;
  return (2 * nb * world + n) * (int64_t)sizeof(int) + 256;
}

extern "C" int rs_shard_bucket(const uint32_t* keys, const uint32_t* vals, int64_t n, int world, int cap,
                               int64_t pad, int32_t* send_ids, int* counts, uint32_t* ckey, int64_t* idx,
                               int* flag, void* ws, void* stream) {
  RS_CHECK_ARG(keys && vals && send_ids && counts && ckey && idx && ws && n >= 0 && world >= 1 &&
                   world <= kMaxWorld && cap >= 1,
               "rs_shard_bucket: bad args (world <= %d)", kMaxWorld);
  RS_CHECK_ARG((int64_t)world * cap < ((int64_t)1 << 31) && n < ((int64_t)1 << 31), "rs_shard_bucket: too large");
  hipStream_t st = as_stream(stream);
  const int nb = n > 0 ? cdiv(n, kBT) : 1;
  int* block_counts = static_cast<int*>(ws);
  int* block_base = block_counts + (int64_t)nb * world;
  int* comp = block_base + (int64_t)nb * world;
  if (n == 0) {
    RS_RET_IF((int)hipMemsetAsync(counts, 0, sizeof(int) * world, st));
    return 0;
  }
  shard_count_kernel<<<nb, kBT, 0, st>>>(keys, n, world, block_counts);
  RS_CHECK_LAUNCH("rs_shard_bucket count");
  shard_scan_kernel<<<1, kBT, 0, st>>>(block_counts, nb, world, cap, block_base, counts, flag);
  RS_CHECK_LAUNCH("rs_shard_bucket scan");
  shard_assign_kernel<<<nb, kBT, 0, st>>>(keys, n, world, cap, block_base, send_ids, comp);
  RS_CHECK_LAUNCH("rs_shard_bucket assign");
  shard_fill_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, st>>>(keys, vals, n, pad, comp,
                                                                           (int64_t)world * cap, idx, ckey, flag);
  RS_CHECK_LAUNCH("rs_shard_bucket fill");
  return 0;
}

extern "C" int rs_shard_recv(const int32_t* recv_ids, const int* recv_counts, int world, int cap,
                             int64_t vocab, int64_t* ids64, int32_t* ids32, int* flag, void* stream) {
  RS_CHECK_ARG(recv_ids && recv_counts && ids64 && ids32 && world >= 1 && cap >= 1 && vocab >= 1 &&
                   vocab < ((int64_t)1 << 31),
               "rs_shard_recv: bad args");
  const int64_t n = (int64_t)world * cap;
  shard_recv_kernel<<<std::min<int64_t>(cdiv(n, 256), 8192), 256, 0, as_stream(stream)>>>(
      recv_ids, recv_counts, world, cap, vocab, ids64, ids32, flag);
  RS_CHECK_LAUNCH("rs_shard_recv");
  return 0;
}
