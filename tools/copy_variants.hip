// Probe: float4 copy variants for the on-box HBM peak (tools only; not part of the library).
// Build: hipcc --offload-arch=gfx950 -O3 tools/copy_variants.hip -o tools/copy_variants
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void oneshot(const floatx4* __restrict__ s, floatx4* __restrict__ d, long n) {
  const long b = (long)blockIdx.x * 256 * U + threadIdx.x;
  floatx4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    long i = b + u * 256;
    v[u] = i < n ? (NT ? __builtin_nontemporal_load(s + i) : s[i]) : floatx4{};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    long i = b + u * 256;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void stride(const floatx4* __restrict__ s, floatx4* __restrict__ d, long n) {
  for (long b0 = (long)blockIdx.x * 256 * U; b0 < n; b0 += (long)gridDim.x * 256 * U) {
    floatx4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = b0 + u * 256 + threadIdx.x;
      v[u] = i < n ? (NT ? __builtin_nontemporal_load(s + i) : s[i]) : floatx4{};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long i = b0 + u * 256 + threadIdx.x;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], d + i);
        else d[i] = v[u];
      }
    }
  }
}

template <typename F>
static void run(const char* name, F launch, long bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9f;
  for (int r = 0; r < 6; ++r) {
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (r && ms < best) best = ms;
  }
  printf("%-28s %8.1f GB/s (%.3f ms)\n", name, 2.0 * bytes / (best * 1e-3) / 1e9, best);
}

int main() {
  const long bytes = 2L << 30, n = bytes / 16;
  floatx4 *s, *d;
  if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
  hipMemset(s, 1, bytes);
  hipMemset(d, 0, bytes);
  run("oneshot U4", [&] { oneshot<4, false><<<(n + 1023) / 1024, 256>>>(s, d, n); }, bytes);
  run("oneshot U4 nt", [&] { oneshot<4, true><<<(n + 1023) / 1024, 256>>>(s, d, n); }, bytes);
  run("oneshot U8", [&] { oneshot<8, false><<<(n + 2047) / 2048, 256>>>(s, d, n); }, bytes);
  run("oneshot U1", [&] { oneshot<1, false><<<(n + 255) / 256, 256>>>(s, d, n); }, bytes);
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stride U8 g%d", g);
    run(nm, [&] { stride<8, false><<<g, 256>>>(s, d, n); }, bytes);
    snprintf(nm, sizeof nm, "stride U16 nt g%d", g);
    run(nm, [&] { stride<16, true><<<g, 256>>>(s, d, n); }, bytes);
    snprintf(nm, sizeof nm, "stride U4 g%d", g);
    run(nm, [&] { stride<4, false><<<g, 256>>>(s, d, n); }, bytes);
  }
  return 0;
}
