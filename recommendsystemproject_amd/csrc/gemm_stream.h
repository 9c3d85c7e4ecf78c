// Shared between gemm.hip (dispatch) and gemm_stream.hip (streaming kernels): ONE definition of
// the launch arguments, so both translation units agree on the layout.
#pragma once
#include "common.h"

namespace rs {

struct StreamArgs {
  int M, N, K;
  float alpha, beta;
  const float* A; int lda;
  const float* B; int ldb;
  float* C; int ldc;
  int epi;
  const float* bias;
  const float* aux; int ld_aux, aux_mod;
  float* rowsum;
  float* ws;
  int transB;
  int vec_epi;  // rowgemm: C / aux / bias rows 16-byte addressable -> float4 epilogue I/O
  float drop_p;
  const int64_t* drop_key;
  int site_a, site_b;
};

bool rowgemm_supported(int transA, int M, int N, int K, const float* A, int lda);
int rowgemm_launch(const StreamArgs& s, hipStream_t st);
bool wgrad_supported(int transA, int transB, int M, int N, int K, const float* A, int lda,
                     const float* B, int ldb, int ldc, int epi);
int64_t wgrad_ws_bytes(int M, int N, int K);
int wgrad_launch(const StreamArgs& s, hipStream_t st);

}  // namespace rs
