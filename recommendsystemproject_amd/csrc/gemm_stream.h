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
  // fused residual + LayerNorm epilogue (rowgemm LN instances, N == 64):
  //   h = drop_a(alpha*acc + bias) + aux  -> C;   y = LN(h) * gamma + beta -> ln_y
  const float* ln_gamma;
  const float* ln_beta;
  float* ln_y;
  float* ln_mean;
  float* ln_rstd;
  float ln_eps;
  // LN instances, optional: the residual row of output row m is aux row m * aux_bag + aux_rows[m]
  // (the pruned last encoder layer reads x[b, last[b]] in place instead of a gathered copy)
  const int64_t* aux_rows;
  int aux_bag;
};

bool rowgemm_supported(int transA, int M, int N, int K, const float* A, int lda);
int rowgemm_launch(const StreamArgs& s, hipStream_t st);
bool rowgemm_ln_supported(int M, int N, int K, const float* A, int lda);
int rowgemm_ln_launch(const StreamArgs& s, hipStream_t st);
bool wgrad_instance(int M, int N);  // an instance exists for this (padded) dW tile
bool wgrad_supported(int transA, int transB, int M, int N, int K, const float* A, int lda,
                     const float* B, int ldb, int ldc, int epi);
int64_t wgrad_ws_bytes(int M, int N, int K);
int wgrad_launch(const StreamArgs& s, hipStream_t st);
// bf16 MFMA weight gradient; y_bf16 / x_bf16: dY (A) / X (B) are stored as bf16
int wgrad_bf16_launch(const StreamArgs& s, bool y_bf16, bool x_bf16, hipStream_t st);

}  // namespace rs
