// Device-side batch assembly: the ragged part of the reference's collate_fn
// (DataLoader.py:250-288, called per tower by CombineTwoTower.py:62-92). A list-valued column is
// stored once in HBM as CSR -- values [nnz, T] (T = 1 for id lists, T = tags per token for
// [L, T] lists) and offsets [rows + 1] -- and a batch of row indices is written as the zero
// right-padded [B, Lb, T] int64 tensor the reference builds with np.pad + np.stack, Lb = the
// longest list in the batch (the caller passes it; the host knows every row's length). Fixed
// width columns (the sparse id matrix, the dense matrix) use rs_catalog_gather.
#include "common.h"

namespace rs {
namespace {

template <typename T>
__global__ void collate_ragged_kernel(const T* __restrict__ values, int tw,
                                      const int64_t* __restrict__ offsets, int64_t rows,
                                      const int64_t* __restrict__ idx, int B, int Lb,
                                      int64_t* __restrict__ out, int* __restrict__ err) {
  const int64_t total = (int64_t)B * Lb * tw;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(e % tw);
    const int64_t bp = e / tw;
    const int p = (int)(bp % Lb), b = (int)(bp / Lb);
    const int64_t i = idx[b];
    int64_t v = 0;
    if (i < 0 || i >= rows) {
      if (p == 0 && t == 0) atomicOr(err, 1);
    } else {
      const int64_t o0 = offsets[i], len = offsets[i + 1] - o0;
      if (p < len) v = (int64_t)values[(o0 + p) * tw + t];
      if (p == 0 && t == 0 && len > Lb) atomicOr(err, 2);  // would be truncated
    }
    out[e] = v;
  }
}

// Up to kCopyMax device-to-device copies in one launch (a batch's columns into the static input
// buffers of a captured step: one dispatch instead of one blit per tensor). Workgroup b copies
// chunk b - first[i] of copy i; 16-byte lanes where both ends are 16-byte aligned, bytes else.
constexpr int kCopyMax = 32;
constexpr int64_t kCopyChunk = 256 * 16 * 4;  // bytes per workgroup
struct CopyList {
  const unsigned char* src[kCopyMax];
  unsigned char* dst[kCopyMax];
  int64_t bytes[kCopyMax];
  int first[kCopyMax + 1];
  int n;
};

__global__ __launch_bounds__(256) void copy_many_kernel(CopyList c) {
  int i = 0;
  while (i + 1 < c.n && (int)blockIdx.x >= c.first[i + 1]) ++i;
  const int64_t off = (int64_t)(blockIdx.x - c.first[i]) * kCopyChunk;
  const int64_t len = c.bytes[i] - off < kCopyChunk ? c.bytes[i] - off : kCopyChunk;
  const unsigned char* s = c.src[i] + off;
  unsigned char* d = c.dst[i] + off;
  if ((((uintptr_t)s | (uintptr_t)d) & 15) == 0) {
    const int64_t n16 = len / 16;
    for (int64_t k = threadIdx.x; k < n16; k += 256)
      reinterpret_cast<uint4*>(d)[k] = reinterpret_cast<const uint4*>(s)[k];
    for (int64_t k = n16 * 16 + threadIdx.x; k < len; k += 256) d[k] = s[k];
  } else {
    for (int64_t k = threadIdx.x; k < len; k += 256) d[k] = s[k];
  }
}

}  // namespace
}  // namespace rs

using namespace rs;

extern "C" int rs_copy_many(int n, const void* const* src, void* const* dst, const int64_t* bytes, void* stream) {
  RS_CHECK_ARG(n >= 0 && n <= kCopyMax && (n == 0 || (src && dst && bytes)), "rs_copy_many: bad args (n=%d)", n);
  CopyList c{};
  c.n = n;
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    RS_CHECK_ARG(bytes[i] >= 0 && (bytes[i] == 0 || (src[i] && dst[i])), "rs_copy_many: copy %d: bad buffer", i);
    c.src[i] = static_cast<const unsigned char*>(src[i]);
    c.dst[i] = static_cast<unsigned char*>(dst[i]);
    c.bytes[i] = bytes[i];
    c.first[i] = wg;
    wg += (int)((bytes[i] + kCopyChunk - 1) / kCopyChunk);
  }
  c.first[n] = wg;
  if (wg == 0) return 0;
  copy_many_kernel<<<wg, 256, 0, as_stream(stream)>>>(c);
  RS_CHECK_LAUNCH("rs_copy_many");
  return 0;
}

extern "C" int rs_collate_ragged(const void* values, int elem, int tw, const int64_t* offsets,
                                 int64_t rows, const int64_t* idx, int B, int Lb, int64_t* out,
                                 int* err_flag, void* stream) {
  RS_CHECK_ARG(values && offsets && idx && out && err_flag && rows >= 0 && B >= 0 && Lb >= 0 && tw >= 1,
               "rs_collate_ragged: bad args");
  RS_CHECK_ARG(elem == 4 || elem == 8, "rs_collate_ragged: elem must be 4 (int32) or 8 (int64)");
  const int64_t total = (int64_t)B * Lb * tw;
  if (total == 0) return 0;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipStream_t st = as_stream(stream);
  if (elem == 4)
    collate_ragged_kernel<int32_t><<<blocks, 256, 0, st>>>(static_cast<const int32_t*>(values), tw, offsets,
                                                          rows, idx, B, Lb, out, err_flag);
  else
    collate_ragged_kernel<int64_t><<<blocks, 256, 0, st>>>(static_cast<const int64_t*>(values), tw, offsets,
                                                          rows, idx, B, Lb, out, err_flag);
  RS_CHECK_LAUNCH("rs_collate_ragged");
  return 0;
}
