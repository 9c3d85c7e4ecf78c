// The random 512-byte-row read ceiling of one MI355X at the launch sizes of the two-tower step's
// embedding gathers (profiling tool, not product code). VERDICT r5 #3 asks for it beside
// rs_gather_fwd's in-step fraction: C3's item gather is 4,096 single rows (2 MB) a launch, the
// pooled history gather 204,800 rows (105 MB), C5's per-token history 819,200.
//
// Kernels (fp32 x 128 rows = 512 B, one float4 per lane, a 32-lane group per row, NB rows in flight
// per group, the sums written once per group so nothing is dead code):
//   rows  : the bare ceiling -- each group reads NB-row batches of its own contiguous id range;
//   bags  : the product's pooled-mean form (bags of 50 positions split GPB ways, NB rows in flight).
// Id sets rotate so a launch never re-reads the previous launch's rows: enough sets that their rows
// exceed the 256 MB Infinity Cache ("cold", HBM) -- or the SAME set back to back ("warm": the rows
// the previous launch left on chip, as the step's catch-up leaves them for the gather).
// Output: one JSON line per (kernel, rows, temperature) with the event time per launch and GB/s of
// algorithmic bytes (rows read + ids + output) against 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -o tools/row_ceiling tools/row_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));

template <int NB>
__global__ __launch_bounds__(256) void rows_kernel(const float* __restrict__ table, const int32_t* __restrict__ ids,
                                                   int n, int per_group, float* __restrict__ out) {
  const int grp = blockIdx.x * 8 + (threadIdx.x >> 5), lane = threadIdx.x & 31;
  const int b = grp * per_group, e = min(n, b + per_group);
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  for (int i0 = b; i0 < e; i0 += NB) {
    int r[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) r[u] = ids[min(i0 + u, e - 1)];
    f4v v[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) v[u] = reinterpret_cast<const f4v*>(table + (int64_t)r[u] * 128)[lane];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (i0 + u < e) acc += v[u];
  }
  if (b < n) reinterpret_cast<f4v*>(out + (int64_t)grp * 128)[lane] = acc;
}

template <int NB, int GPB>
__global__ __launch_bounds__(256) void bags_kernel(const float* __restrict__ table, const int32_t* __restrict__ ids,
                                                   int B, int L, float* __restrict__ out) {
  __shared__ f4v red[256];
  const int grp = threadIdx.x >> 5, lane = threadIdx.x & 31;
  const int g = blockIdx.x * 8 + grp;
  const int bag = g / GPB, part = g % GPB;
  const bool active = bag < B;
  const int per = (L + GPB - 1) / GPB;
  const int lb = min(part * per, L), le = min(lb + per, L);
  f4v acc = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    const int32_t* id = ids + (int64_t)bag * L;
    for (int l0 = lb; l0 < le; l0 += NB) {
      int r[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) r[u] = id[min(l0 + u, le - 1)];
      f4v v[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) v[u] = reinterpret_cast<const f4v*>(table + (int64_t)r[u] * 128)[lane];
#pragma unroll
      for (int u = 0; u < NB; ++u)
        if (l0 + u < le) acc += v[u];
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (!active || part != 0) return;
  for (int q = 1; q < GPB; ++q) acc += red[threadIdx.x + 32 * q];
  reinterpret_cast<f4v*>(out + (int64_t)bag * 128)[lane] = acc * (1.f / (float)L);
}

__global__ void fill_ids(int32_t* ids, int64_t n, uint64_t seed, int64_t V) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    ids[i] = (int32_t)(1 + (int64_t)(x % (uint64_t)(V - 1)));
  }
}

template <typename F>
float time_launches(F launch, int nsets, bool warm, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) launch(warm ? 0 : w % nsets);
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch(warm ? 0 : (i + 3) % nsets);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms / iters;
}

void report(const char* kernel, int rows, const char* temp, int nb, int gpb, double bytes, float ms) {
  printf("{\"kernel\": \"%s\", \"rows\": %d, \"row_bytes\": 512, \"temperature\": \"%s\", \"NB\": %d, \"GPB\": %d, "
         "\"alg_bytes\": %.0f, \"us\": %.2f, \"GBs\": %.1f, \"frac_8TBs\": %.4f}\n",
         kernel, rows, temp, nb, gpb, bytes, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const int64_t V = 10000000;  // C3's 10M x 128 fp32 table (5.1 GB)
  const int L = 50;
  std::vector<int> sizes = {4096, 16384, 65536, 204800, 819200};
  if (argc > 1) {
    sizes.clear();
    for (int i = 1; i < argc; ++i) sizes.push_back(atoi(argv[i]));
  }
  float* table;
  CK(hipMalloc(&table, V * 128 * sizeof(float)));
  CK(hipMemset(table, 0, V * 128 * sizeof(float)));
  float* out;
  CK(hipMalloc(&out, (size_t)819200 * 128 * sizeof(float)));
  for (int n : sizes) {
    // cold: id sets whose rows together exceed the Infinity Cache twice over
    const int64_t launch_bytes = (int64_t)n * 512;
    const int nsets = (int)std::max<int64_t>(8, (512ll << 20) / launch_bytes + 1);
    std::vector<int32_t*> sets(nsets);
    for (int s = 0; s < nsets; ++s) {
      CK(hipMalloc(&sets[s], (size_t)n * sizeof(int32_t)));
      fill_ids<<<256, 256>>>(sets[s], n, 1234 + s * 7919ull, V);
    }
    CK(hipDeviceSynchronize());
    const int iters = n <= 16384 ? 200 : 40;
    for (int warm = 0; warm < 2; ++warm) {
      const char* temp = warm ? "warm" : "cold";
      // bare rows, 2 rows per group (one per wave-half pair at 4096 rows: 256 workgroups) .. 16
      for (int per : {1, 2, 4, 16}) {
        const int groups = (n + per - 1) / per;
        const int grid = (groups + 7) / 8;
        auto go4 = [&](int s) { rows_kernel<4><<<grid, 256>>>(table, sets[s], n, per, out); };
        const float ms = time_launches(go4, nsets, warm, iters);
        report(per == 1 ? "rows_1" : per == 2 ? "rows_2" : per == 4 ? "rows_4" : "rows_16", n, temp, 4, per,
               (double)n * (512 + 4) + (double)groups * 512, ms);
      }
      // the product's pooled form: bags of 50 (n / 50 bags), 16 rows in flight split 4 ways
      if (n % L == 0 || n >= 204800) {
        const int B = n / L;
        const int grid = (B * 4 + 7) / 8;
        auto gob = [&](int s) { bags_kernel<16, 4><<<grid, 256>>>(table, sets[s], B, L, out); };
        const float ms = time_launches(gob, nsets, warm, iters);
        report("bags_16x4", B * L, temp, 16, 4, (double)B * L * (512 + 4) + (double)B * 512, ms);
      }
    }
    for (auto p : sets) CK(hipFree(p));
  }
  CK(hipFree(table));
  CK(hipFree(out));
  return 0;
}
