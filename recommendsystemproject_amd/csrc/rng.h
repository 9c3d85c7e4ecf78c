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
  uint64_t base;
  float p, scale;  // scale = 1/(1-p)
};

__device__ __forceinline__ DropKey make_key(const int64_t* key, int site, float p) {
  DropKey k;
  k.base = mix64((uint64_t)key[0] ^ mix64((uint64_t)key[1] * 0x9e3779b97f4a7c15ULL +
                                          (uint64_t)site * 0xd1b54a32d192ed03ULL));
  k.p = p;
  k.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  return k;
}

// multiplier for element idx: 0 (dropped) or 1/(1-p) (kept)
__device__ __forceinline__ float keep_mult(const DropKey& k, uint64_t idx) {
  const uint64_t h = mix64(k.base + idx * 0x9e3779b97f4a7c15ULL);
  const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0, 1), 24 bits
  return u >= k.p ? k.scale : 0.f;
}

}  // namespace rs
