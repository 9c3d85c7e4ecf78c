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
  uint32_t thresh;  // keep iff hash >= thresh, thresh = p * 2^32
  float scale;      // 1 / (1 - p)
};

__device__ __forceinline__ DropKey make_key(const int64_t* key, int site, float p) {
  DropKey k;
  const uint64_t b = mix64((uint64_t)key[0] ^ mix64((uint64_t)key[1] * 0x9e3779b97f4a7c15ULL +
                                                    (uint64_t)site * 0xd1b54a32d192ed03ULL));
  k.k0 = (uint32_t)b;
  k.k1 = (uint32_t)(b >> 32);
  const double t = (double)p * 4294967296.0;
  k.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
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

// multiplier for element idx: 0 (dropped) or 1/(1-p) (kept); two 32-bit finalisers (cheap on
// the VALU: no 64-bit multiplies) keyed by the 64-bit stream key
__device__ __forceinline__ float keep_mult(const DropKey& k, uint64_t idx) {
  const uint32_t h = fmix32(fmix32((uint32_t)idx ^ k.k0) + k.k1 + (uint32_t)(idx >> 32));
  return h >= k.thresh ? k.scale : 0.f;
}

}  // namespace rs
