// Standalone sweep of pooled-bag gather forms (profiling tool, not product code): C3's history
// shape (B bags x L positions into a V x 128 fp32 table, mean pooling), 8 rotating id sets so the
// rows come from HBM. Variants: positions of a bag split over GPB groups of 32 lanes (one float4
// per lane: one 512-B row per group and instruction), NB rows in flight per group, default or
// non-temporal row loads. Prints GB/s of algorithmic bytes (rows read + bags written + ids).
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_sweep tools/gather_sweep.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int NB, int GPB, bool NT>
__global__ __launch_bounds__(256) void bag_gather(const float* __restrict__ table, const int64_t* __restrict__ ids,
                                                  int B, int L, float* __restrict__ out) {
  __shared__ float4 red[256];
  const int grp = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int g = blockIdx.x * 8 + grp;
  const int bag = g / GPB, part = g % GPB;
  const bool active = bag < B;
  const int per = (L + GPB - 1) / GPB;
  const int lb = min(part * per, L), le = min(lb + per, L);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (active) {
    const int64_t* id = ids + (int64_t)bag * L;
    int64_t raw[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) raw[u] = lb + u < le ? id[lb + u] : 0;
    for (int l0 = lb; l0 < le; l0 += NB) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      f4v v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const f4v* p = reinterpret_cast<const f4v*>(table + raw[u] * 128) + lane;
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) raw[u] = l0 + NB + u < le ? id[l0 + NB + u] : 0;
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (l0 + u < le) {
          acc.x += v[u][0]; acc.y += v[u][1]; acc.z += v[u][2]; acc.w += v[u][3];
        }
      }
    }
  }
  if constexpr (GPB > 1) {
    red[threadIdx.x] = acc;
    __syncthreads();
    if (!active || part != 0) return;
    for (int q = 1; q < GPB; ++q) {
      const float4 t = red[threadIdx.x + 32 * q];
      acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
    }
  } else if (!active) {
    return;
  }
  const float s = 1.f / (float)L;
  reinterpret_cast<float4*>(out + (int64_t)bag * 128)[lane] = make_float4(acc.x * s, acc.y * s, acc.z * s, acc.w * s);
}

template <int NB, int GPB, bool NT>
void run(const char* name, const float* table, std::vector<int64_t*>& idsets, int B, int L, float* out, int iters) {
  const int groups = B * GPB;
  const int grid = (groups + 7) / 8;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) bag_gather<NB, GPB, NT><<<grid, 256>>>(table, idsets[w % idsets.size()], B, L, out);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) bag_gather<NB, GPB, NT><<<grid, 256>>>(table, idsets[i % idsets.size()], B, L, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double bytes = (double)B * L * 512 + (double)B * 512 + (double)B * L * 8;
  printf("{\"variant\": \"%s\", \"NB\": %d, \"GPB\": %d, \"nt\": %d, \"B\": %d, \"L\": %d, \"us\": %.2f, \"GBs\": %.1f, \"frac_8TBs\": %.4f}\n",
         name, NB, GPB, (int)NT, B, L, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
}

__global__ void fill_ids(int64_t* ids, int64_t n, uint64_t seed, int64_t V) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    ids[i] = 1 + (int64_t)(x % (uint64_t)(V - 1));
  }
}

int main(int argc, char** argv) {
  const int64_t V = 10000000;
  const int B = argc > 1 ? atoi(argv[1]) : 4096, L = 50, sets = 8, iters = 40;
  float* table;
  CK(hipMalloc(&table, V * 128 * sizeof(float)));
  CK(hipMemset(table, 0, V * 128 * sizeof(float)));
  float* out;
  CK(hipMalloc(&out, (size_t)B * 128 * sizeof(float)));
  std::vector<int64_t*> idsets(sets);
  for (int s = 0; s < sets; ++s) {
    CK(hipMalloc(&idsets[s], (size_t)B * L * sizeof(int64_t)));
    fill_ids<<<1024, 256>>>(idsets[s], (int64_t)B * L, 1234 + s * 7919, V);
  }
  CK(hipDeviceSynchronize());
#define R(NB, GPB, NT) run<NB, GPB, NT>("bag_gather", table, idsets, B, L, out, iters)
  R(4, 1, false); R(8, 4, false);
  R(2, 1, true); R(4, 1, true); R(8, 1, true);
  R(2, 2, true); R(4, 2, true); R(8, 2, true);
  R(2, 4, true); R(4, 4, true); R(8, 4, true);
  R(2, 8, true); R(4, 8, true); R(8, 8, true);
  CK(hipDeviceSynchronize());
  return 0;
}
