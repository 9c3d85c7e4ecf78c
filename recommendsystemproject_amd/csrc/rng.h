// Counter-based dropout masks. A dropout site draws keep/drop for element `idx` from a hash of
// (seed, call counter, site, idx): no RNG state per element, nothing saved for backward (the
// backward re-derives the same mask), and graph-replay safe because the (seed, counter) key
// lives in device memory and is advanced by a kernel (rs_rng_next) on every forward call.
#pragma once
#include <stdint.h>

namespace rs {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct DropKey {
  uint32_t k0, k1;  // per (seed, counter, site) stream keys
  uint32_t thresh;  // keep iff the element's 16 hash bits >= thresh = floor(p * 2^16)
  float scale;      // 1 / (1 - p)
};

__device__ __forceinline__ DropKey make_key(const int64_t* key, int site, float p) {
  DropKey k;
  const uint64_t b = mix64((uint64_t)key[0] ^ mix64((uint64_t)key[1] * 0x9e3779b97f4a7c15ULL +
                                                    (uint64_t)site * 0xd1b54a32d192ed03ULL));
  k.k0 = (uint32_t)b;
  k.k1 = (uint32_t)(b >> 32);
  const double t = (double)p * 65536.0;
  k.thresh = t >= 65536.0 ? 65536u : (uint32_t)t;
  k.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return k;
}

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// One 32-bit hash per PAIR of elements (2j, 2j+1): the low 16 bits decide element 2j, the high
// 16 bits element 2j+1. The hash is the murmur3 finaliser (a bijection with full avalanche) of
// the pair index keyed by the 64-bit stream key (k0 before, k1 after); its two integer
// multiplies are the expensive part on the VALU, so kernels that own consecutive elements draw
// two masks per hash (keep_pair); keep_mult gives the same draw element by element.
__device__ __forceinline__ uint32_t pair_hash32(const DropKey& k, uint32_t pair) {
  return fmix32(pair ^ k.k0) ^ k.k1;
}
__device__ __forceinline__ uint32_t pair_hash(const DropKey& k, uint64_t pair) {
  // indices >= 2^33 fold their high word in (an odd multiple keeps distinct pairs distinct
  // within a 2^32 window); below 2^33 this is pair_hash32
  return pair_hash32(k, (uint32_t)pair ^ ((uint32_t)(pair >> 32) * 0x9e3779b9u));
}

// multiplier for element idx: 0 (dropped) or 1/(1-p) (kept)
__device__ __forceinline__ float keep_mult(const DropKey& k, uint64_t idx) {
  const uint32_t h = pair_hash(k, idx >> 1);
  const uint32_t bits = (idx & 1) ? (h >> 16) : (h & 0xffffu);
  return bits >= k.thresh ? k.scale : 0.f;
}

// the same draw for an index known to be < 2^32 (callers check their index range on the host):
// no 64-bit index arithmetic per element
__device__ __forceinline__ float keep_mult32(const DropKey& k, uint32_t idx) {
  const uint32_t h = pair_hash32(k, idx >> 1);
  const uint32_t bits = (idx & 1) ? (h >> 16) : (h & 0xffffu);
  return bits >= k.thresh ? k.scale : 0.f;
}

// multipliers of elements 2*pair and 2*pair + 1 from one hash
__device__ __forceinline__ void keep_pair(const DropKey& k, uint64_t pair, float& m0, float& m1) {
  const uint32_t h = pair_hash(k, pair);
  m0 = (h & 0xffffu) >= k.thresh ? k.scale : 0.f;
  m1 = (h >> 16) >= k.thresh ? k.scale : 0.f;
}
__device__ __forceinline__ void keep_pair32(const DropKey& k, uint32_t pair, float& m0, float& m1) {
  const uint32_t h = pair_hash32(k, pair);
  m0 = (h & 0xffffu) >= k.thresh ? k.scale : 0.f;
  m1 = (h >> 16) >= k.thresh ? k.scale : 0.f;
}

// elements idx0 .. idx0+3 (idx0 even: two hashes)
__device__ __forceinline__ void keep4(const DropKey& k, uint64_t idx0, float (&mk)[4]) {
  if ((idx0 & 1) == 0) {
    keep_pair(k, idx0 >> 1, mk[0], mk[1]);
    keep_pair(k, (idx0 >> 1) + 1, mk[2], mk[3]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) mk[i] = keep_mult(k, idx0 + i);
  }
}
__device__ __forceinline__ void keep4_32(const DropKey& k, uint32_t idx0, float (&mk)[4]) {
  if ((idx0 & 1) == 0) {
    keep_pair32(k, idx0 >> 1, mk[0], mk[1]);
    keep_pair32(k, (idx0 >> 1) + 1, mk[2], mk[3]);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) mk[i] = keep_mult32(k, idx0 + i);
  }
}

}  // namespace rs
