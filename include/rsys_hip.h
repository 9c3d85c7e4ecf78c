/*
 * rsys_hip.h — C ABI of librsys_hip.so, the MI355X (gfx950) hot path of the two-tower DSSM
 * training step (feature gather, Transformer encoder, MLP towers, in-batch softmax loss,
 * clip + Adam). Every entry point replaces an ATen op the reference reaches through the
 * nn.Module API in project/models/TwoTower/ (file:line cited per function).
 *
 * Conventions
 *   - Plain pointers and sizes only; every pointer is DEVICE memory unless stated otherwise.
 *     The caller owns all memory (tensors and workspaces); the library never allocates or frees.
 *   - `stream` is a hipStream_t passed as void*; all work is enqueued on it, no implicit sync.
 *     Every entry point is graph-capturable (no alloc/sync/memcpy inside).
 *   - Return 0 on success, <0 for a bad argument (message in rs_last_error()), >0 a hipError_t.
 *   - fp32 data, int64 ids (the reference's torch.long batches, DataLoader.py:259,287).
 */
#ifndef RSYS_HIP_H
#define RSYS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- library */
int rs_version(void);                 /* ABI version (integer, bumps on signature change) */
const char* rs_last_error(void);      /* thread-local message of the last failing call */
int rs_device_check(void);            /* 0 if a gfx950 device is current, else hipError / -1 */
/* Profiling only: launches an empty one-lane kernel (prof_marker_kernel) on the stream so that
 * a rocprofv3 --pmc pass can attribute the dispatches between two markers to one entry point
 * (bench.py --pmc-bracket, tools/pmc_traffic.py). Not on the training path. */
int rs_prof_marker(int tag, void* stream);
/* Measurement only (bench.py, not on the training path): the on-box peaks the rooflines are
 * reported against beside the datasheet's. rs_peak_copy: a float4 streaming copy
 * of `bytes` (16-byte aligned buffers); rs_peak_mfma: `blocks` 256-thread workgroups each wave
 * issuing iters x 4 back-to-back v_mfma_f32_32x32x16_bf16; rs_peak_mfma_flops: its flop count. */
int rs_peak_copy(const void* src, void* dst, int64_t bytes, void* stream);
int rs_peak_mfma(float* out, int blocks, int iters, void* stream);
int64_t rs_peak_mfma_flops(int blocks, int iters);

/* ---------------------------------------------------------------- GEMM (fp32 MFMA)
 * C = epi(alpha * op(A) @ op(B))  with op(A)[m,k] = transA ? A[k*lda+m] : A[m*lda+k],
 * op(B)[k,n] = transB ? B[n*ldb+k] : B[k*ldb+n]. Epilogue, in this order (flags bitwise):
 *   v = alpha * acc
 *   RS_EPI_BIAS     v += bias[n]
 *   RS_EPI_AUX_MASK v = aux[m*ld_aux+n] > 0 ? v : 0        (ReLU backward)
 *   RS_EPI_RELU     v = max(v, 0)
 *   RS_EPI_DROP_A   v *= dropout mask of (drop_key, site_a) at element m*N+n  (rs_dropout_fwd)
 *   RS_EPI_AUX_ADD  v += aux[(m % aux_mod)*ld_aux + n]     (residual / positional rows)
 *   RS_EPI_DROP_B   v *= dropout mask of (drop_key, site_b) at element m*N+n
 *   beta != 0       v += beta * C_old
 * rowsum != NULL: rowsum[m] += alpha * sum_k op(A)[m, k] — fused into the staged A tiles; with
 *   transA this is the bias gradient of a weight-gradient GEMM (dW = dY^T X, db = colsum dY).
 * split_k > 1 needs the workspace rs_gemm_ws_bytes(M, N, K, split_k).
 * Replaces nn.Linear / addmm / matmul / bmm on the hot path: Tower.py:16-25,
 * SequenceFeatureProcessor.py:77, TransformerEncoderLayer in/out_proj + linear1/2
 * (SequenceEncoder.py:17-23), TwoTowerModel.py:95 (U @ I^T) and all their backwards. */
#define RS_EPI_BIAS 1
#define RS_EPI_RELU 2
#define RS_EPI_AUX_ADD 4
#define RS_EPI_AUX_MASK 8
#define RS_EPI_DROP_A 16
#define RS_EPI_DROP_B 32
/* Flag in the same word: the caller allows bf16 operands (bf16 compute mode). Where a bf16-MFMA
 * instance exists (the encoder's streaming shapes) A and B are rounded to bf16 (RNE) and the
 * products accumulate in fp32; every other shape runs the fp32 kernels unchanged. */
#define RS_GEMM_BF16 256
/* Storage flags in the same word (bf16 compute mode only): A holds bf16 elements (lda counted in
 * elements) / C is written as bf16 (RNE of the fp32 epilogue result). For operands that are only
 * ever consumed as bf16 MFMA operands (the encoder's packed qkv and its gradient) this halves their
 * HBM bytes without changing any product. Only the streaming bf16 instances accept them; a call
 * none covers fails with a bad-argument error (never a silent conversion). */
#define RS_GEMM_A_BF16 512
#define RS_GEMM_C_BF16 1024
int rs_gemm_auto_split(int M, int N, int K);   /* split_k that fills the chip for long K */
int64_t rs_gemm_ws_bytes(int M, int N, int K, int split_k);
int rs_gemm_f32(int transA, int transB, int M, int N, int K, float alpha,
                const float* A, int lda, const float* B, int ldb, float beta, float* C, int ldc,
                int epilogue, const float* bias, const float* aux, int ld_aux, int aux_mod,
                float drop_p, const int64_t* drop_key, int site_a, int site_b,
                float* rowsum, int split_k, float* ws, void* stream);

/* ---------------------------------------------------------------- column reductions
 * out[n] = beta*out[n] + scale * sum_{m<M} X[m*ldx + n]   (bias / pos-emb / LN grads)
 * ws: rs_colsum_ws_bytes(M, N) bytes. */
int64_t rs_colsum_ws_bytes(int M, int N);
int rs_colsum(const float* X, int M, int N, int ldx, float scale, float beta, float* out,
              float* ws, void* stream);

/* ---------------------------------------------------------------- feature gather
 * Descriptor-driven multi-table gather into a row-major concat buffer out[rows, ldo].
 * One segment per feature (kind: 0 single sparse id, 1 pooled bag, 2 dense Linear(1,D),
 * 3 last-valid row of a [rows*L, D] sequence, 4 plain [rows, D] slice copy). Segments are
 * passed by value into the kernel arguments (at most 20 per call). Replaces GenericTower.forward feature loop (GenericTower.py:133-233,
 * K1/K2/K11 + torch.cat), SequenceFeatureProcessor.forward gather/tag-pool/cat
 * (SequenceFeatureProcessor.py:57-76, K3) and SequenceEncoder._gather_last_valid
 * (SequenceEncoder.py:58-74, K10). Segment layout: rs_feature_seg_t below. */
#define RS_SEG_SPARSE 0
#define RS_SEG_POOL 1
#define RS_SEG_DENSE 2
#define RS_SEG_LASTVALID 3
#define RS_SEG_COPY 4
#define RS_POOL_MEAN 0
#define RS_POOL_SUM 1
#define RS_POOL_MAX 2
typedef struct rs_feature_seg {
  int kind;               /* RS_SEG_* */
  int dim;                /* D: output columns of this segment */
  int out_col;            /* first column in the concat buffer */
  int pool_mode;          /* RS_POOL_* (kind 1) */
  int bag;                /* kind 1: ids per row; kind 3: L (rows per sample in src) */
  int pad_idx;            /* row whose gradient is dropped (padding_idx); -1 none */
  int64_t vocab;          /* table rows (bounds check) */
  int64_t idx_stride;     /* elements between consecutive rows' ids (kind 0/1), x (kind 2) */
  const int64_t* idx;     /* kind 0/1 ids; kind 3: int64 last-valid index per row */
  const float* table;     /* kind 0/1 [vocab, dim]; kind 2 weight [dim]; kind 3 src [rows*bag, dim];
                             kind 4 src [rows, dim] */
  const float* bias;      /* kind 2 bias [dim] */
  const float* x;         /* kind 2 input column */
  float* grad;            /* backward destination: kind 0/1 table grad [vocab, dim];
                             kind 2 weight grad [dim]; kind 3 src grad [rows*bag, dim] (+=);
                             kind 4 src grad [rows, dim] (=) */
  float* grad_bias;       /* kind 2 bias grad [dim] */
  const int* touch_count; /* kind 0/1, nullable: per-row lookup count of this optimizer step
                             (rs_sparse_touch); a row looked up once gets its gradient by a
                             plain store instead of an atomic add */
  const int* lazy_last;   /* kind 0/1, nullable, rs_gather_fwd_lazy only: `last` of a lazy-Adam
                             table (the optimizer step each row was last brought to); the rows are
                             returned brought to the current step without being written */
  const uint32_t* hot_keys; /* kind 1 (mean / sum), nullable, forward only: this call's ids sorted
                             by row (rs_lookup_sort keys, hot_n of them). The rows looked up at
                             least 2 x 256 times (the padding row, Zipf-hot rows; up to 64 of them)
                             are found from the sorted keys and staged once per workgroup into LDS,
                             and their lookups are served from there (same values, same order:
                             the result is bitwise the plain gather's) */
  int64_t hot_n;
} rs_feature_seg_t;

int rs_gather_fwd(const rs_feature_seg_t* segs, int nseg, int rows, float* out, int ldo,
                  int* err_flag, void* stream);
/* The same gather with a read-through catch-up for the segments whose lazy_last is set (large
 * lazy-Adam tables, sparse or sum / mean pooled, D % 4 == 0): each row is returned as
 * rs_sorted_catchup would leave it -- the zero-gradient Adam steps last+1 .. *step replayed in
 * registers from its exp_avg / exp_avg_sq, found m_off / v_off floats past the parameter element
 * (one flat buffer per state) -- and nothing is written; rs_sorted_adam replays the same steps
 * before its own. consts, beta1, beta2, eps, weight_decay: as rs_sorted_catchup. */
int rs_gather_fwd_lazy(const rs_feature_seg_t* segs, int nseg, int rows, float* out, int ldo,
                       int* err_flag, int64_t m_off, int64_t v_off, const int64_t* step,
                       const float* consts, float beta1, float beta2, float eps, float weight_decay,
                       void* stream);
/* Backward: table grads by scatter-add (padding row skipped), dense grads via column
 * reductions (ws: rs_gather_ws_bytes), last-valid rows copied into a pre-zeroed src grad.
 * Replaces the embedding backward of the reference's nn.Embedding lookups (GenericTower.py:153-
 * 184, SequenceFeatureProcessor.py:57-66; torch's embedding_dense_backward). */
int64_t rs_gather_ws_bytes(const rs_feature_seg_t* segs_host, int nseg, int rows);
int rs_gather_bwd(const rs_feature_seg_t* segs, int nseg, int rows, const float* dout, int ldo,
                  float* ws, void* stream);
/* Deterministic table gradients for every later rs_gather_bwd / rs_gather_ws_bytes (on != 0; also
 * RSYS_DETERMINISTIC=1): the small tables through slot-private LDS images and the tables of up to
 * 4 MB through the ranged LDS-image kernel, partials summed in fixed orders -- bitwise
 * reproducible, slower than the float-atomic default at B = 4096 (torch.use_deterministic_
 * algorithms(True) in the caller switches it on, as it does for torch's own index_add / embedding
 * backward). Returns the previous setting. */
int rs_set_deterministic(int on);

/* h = dropout(A W^T + bias) + resid; y = LayerNorm(h)*gamma + beta; per-row mean / rstd.
 * The post-LN residual block of nn.TransformerEncoderLayer (x + dropout(sublayer(x)) -> norm,
 * SequenceEncoder.py:17-29) with the sublayer's closing Linear fused in: one streaming kernel
 * for the encoder width (N = 64; K = 64 or 256), otherwise rs_gemm_f32 + rs_add_layernorm_fwd.
 * A [M, lda], W [N, ldw] (nn.Linear weight), resid / h / y [M, N]; bias nullable. Dropout mask
 * of element (m, n): site `site`, index m*N + n (the same draw as rs_add_layernorm_fwd). */
int rs_gemm_add_layernorm(int M, int N, int K, const float* A, int lda, const float* W, int ldw,
                          const float* bias, const float* resid, float* h, float* y,
                          const float* gamma, const float* beta, float* mean, float* rstd, float eps,
                          float p, const int64_t* key, int site, int flags, void* stream);
/* flags: RS_GEMM_BF16 (bf16 operands for the GEMM part; LayerNorm stays fp32) or 0. */
/* The same with the residual read in place (round 5): row m's residual is resid row
 * m * resid_bag + resid_rows[m] -- the pruned last encoder layer's x[b, last[b]]
 * (SequenceEncoder.py:58-74), no gathered copy. bf16 mode (flags & RS_GEMM_BF16), M % 16 == 0,
 * N == 64, K in {64, 256}; anything else fails (the caller gathers the rows and calls
 * rs_gemm_add_layernorm). */
int rs_gemm_add_layernorm_rows(int M, int N, int K, const float* A, int lda, const float* W, int ldw,
                               const float* bias, const float* resid, const int64_t* resid_rows,
                               int resid_bag, float* h, float* y, const float* gamma, const float* beta,
                               float* mean, float* rstd, float eps, float p, const int64_t* key, int site,
                               int flags, void* stream);

/* ---------------------------------------------------------------- fused feed-forward block (bf16 mode)
 * x2 = norm2(x1 + dropout2(linear2(dropout(relu(linear1(x1)))))) of nn.TransformerEncoderLayer
 * (SequenceEncoder.py:17-29), d_model = 64, F = dim_feedforward = 256, bf16 operands / fp32
 * accumulation (the RS_GEMM_BF16 compute mode). The [M, F] inner activation stays in registers:
 *   rs_ffn_fwd_bf16: x [M,64] (x1; also the residual), W1 [F,64], b1, W2 [64,F], b2, gamma, beta
 *     -> h [M,64] (pre-norm sum), y [M,64] (x2), mean/rstd [M], mask [rs_ffn_mask_words] uint64
 *     (bit set where f1 > 0). Dropout: linear1's output site1 (element m*F + n), linear2's site2
 *     (m*64 + n) -- the draws of the unfused rs_gemm_f32 / rs_gemm_add_layernorm calls.
 *   rs_ffn_bwd_bf16: dff [M,64] = gradient of linear2's output (after dropout2's backward);
 *     writes f1 and dPre1 (gradient of linear1's output) as bf16 [M,F] for the weight gradients
 *     and dx [M,64] = dres + dPre1 W1 (dres: the residual-path gradient; dx may alias dres but
 *     not dff). M % 16 == 0. */
int64_t rs_ffn_mask_words(int M, int F);
int rs_ffn_fwd_bf16(int M, int F, const float* x, const float* W1, const float* b1, const float* W2,
                    const float* b2, const float* gamma, const float* beta, float eps, float* h,
                    float* y, float* mean, float* rstd, uint64_t* mask, float p, const int64_t* key,
                    int site1, int site2, void* stream);
int rs_ffn_bwd_bf16(int M, int F, const float* x, const float* W1, const float* b1, const float* W2,
                    const uint64_t* mask, const float* dff, const float* dres, float* dx, void* f1,
                    void* dpre, float p, void* stream);
/* rs_ffn_bwd_bf16 with the backward of the LayerNorm that produced x (norm1 of the same
 * TransformerEncoderLayer, x1 = LN1(h1)) fused into its epilogue: dx never reaches HBM; writes
 * dh1 = LN1-backward(dx) (h1, gamma1, mean1, rstd1 of the forward), dsa = dropout-backward of
 * dh1 at `site` (element m*64 + n; nullable when p == 0), and accumulates dgamma1 / dbeta1
 * (fixed-order partials in ws: rs_ffn_bwd_ln_ws_bytes). Replaces the rs_ffn_bwd_bf16 +
 * rs_layernorm_bwd pair of SequenceEncoder's layer backward. dh1 may alias dres (not dff). */
int64_t rs_ffn_bwd_ln_ws_bytes(int M, int F);
int rs_ffn_bwd_ln_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                       const float* W2, const uint64_t* mask, const float* dff, const float* dres,
                       const float* h1, const float* gamma1, const float* mean1, const float* rstd1,
                       float* dh1, float* dsa, float* dgamma1, float* dbeta1, void* f1, void* dpre,
                       float p, const int64_t* key, int site, float* ws, void* stream);
/* rs_ffn_bwd_ln_bf16 with norm2's backward as its prologue (bf16 mode, F = 256, M % 16 == 0):
 * x2 = LN2(x1 + drop2(ffn(x1))) with x1 = LN1(h1). Reads dy2 = dL/dx2 and h2 (+ norm2's
 * mean2 / rstd2 / gamma2) instead of dff / dres; writes dff = drop2(dh2) [M, 64] (the operand of
 * rs_ffn_wgrad_bf16), dh1, dsa (p > 0) and accumulates dgamma1/dbeta1, dgamma2/dbeta2
 * (fixed-order partials in ws: rs_ffn_bwd_ln2_ws_bytes). Replaces rs_layernorm_bwd (norm2) +
 * rs_ffn_bwd_ln_bf16 of TransformerEncoderLayer's backward (SequenceEncoder.py:17-29; post-LN,
 * norm_first=False). Only dh1 may alias dy2. */
int64_t rs_ffn_bwd_ln2_ws_bytes(int M, int F);
int rs_ffn_bwd_ln2_bf16(int M, int F, const float* x, const float* W1, const float* b1,
                        const float* W2, const uint64_t* mask, const float* dy2, const float* h2,
                        const float* gamma2, const float* mean2, const float* rstd2, float* dff,
                        float* dgamma2, float* dbeta2, const float* h1, const float* gamma1,
                        const float* mean1, const float* rstd1, float* dh1, float* dsa,
                        float* dgamma1, float* dbeta1, float p, const int64_t* key, int site1,
                        int site2, float* ws, void* stream);
/* dW[Mo,No] = beta*dW + dY^T X over `rows` rows on bf16 MFMA (fp32 accumulate, fixed-order
 * reduction); db[Mo] += colsum(dY) (nullable). dY / X are fp32 or, with dy_bf16 / x_bf16, bf16
 * (the fused FFN's f1 / dPre1). Replaces the weight-gradient part of autograd's Linear backward
 * (Tower.py:16-25, TransformerEncoderLayer). ws: rs_wgrad_ws_bytes. */
int64_t rs_wgrad_ws_bytes(int Mo, int No, int rows);
/* The FFN block's weight gradients without its [M, F] activations in HBM (bf16 mode):
 * dW1 += dPre1^T x, db1 += colsum(dPre1), dW2 += dff^T f1, db2 += colsum(dff), with f1 and
 * dPre1 recomputed from x, dff and the forward's mask exactly as rs_ffn_bwd_bf16 forms them
 * (which then runs with f1 = dpre = NULL). Replaces the two rs_wgrad_bf16 calls of
 * linear2.weight / linear1.weight (.grad accumulation of nn.TransformerEncoderLayer's
 * feed-forward, SequenceEncoder.py:17-29). ws: rs_ffn_wgrad_ws_bytes; deterministic. */
int64_t rs_ffn_wgrad_ws_bytes(int M, int F);
int rs_ffn_wgrad_bf16(int M, int F, const float* x, const float* W1, const float* b1, const float* W2,
                      const uint64_t* mask, const float* dff, float p, float* dW1, float* db1,
                      float* dW2, float* db2, float* ws, void* stream);
int rs_wgrad_bf16(int rows, int Mo, int No, const void* dy, int ldy, int dy_bf16, const void* x,
                  int ldx, int x_bf16, float beta, float* dW, int ldw, float* db, float* ws,
                  void* stream);

/* ---------------------------------------------------------------- sequence mask
 * padding mask from the first sequence feature (== pad_value) with the all-padding-row fix,
 * and last-valid index (SequenceEncoder.py:36-46, :66-70; traps T6/T7).
 * key_pad[b*L+l] = 1 if masked; last[b] = clamp(sum(valid)-1, 0). */
int rs_seq_mask(const int64_t* seq, int64_t ld_seq, int B, int L, int64_t pad_value,
                uint8_t* key_pad, int64_t* last, void* stream);

/* ---------------------------------------------------------------- attention
 * Masked multi-head self-attention core on packed qkv [B*L, 3d] (in_proj output), heads of
 * hd = d/H columns; out [B*L, d]; lse [B*H*L] saved for backward. Replaces the SDPA math path
 * inside nn.MultiheadAttention (SequenceEncoder.py:17-29 via TransformerEncoderLayer, K6).
 * p > 0: dropout on the attention probabilities with the rs_dropout mask of (key, site).
 * flags: RS_GEMM_BF16 -> the products on bf16 MFMA (operands rounded to bf16; softmax, dropout
 * and dS arithmetic in fp32) where the MFMA kernels apply (head_dim 16, L <= 64), else 0.
 * RS_ATTN_QKV_BF16 (with RS_GEMM_BF16, on that path only): qkv is bf16 storage and rs_attn_bwd
 * writes dqkv as bf16 (RNE); Q, K, V are MFMA operands only, so the products are unchanged. */
#define RS_ATTN_QKV_BF16 2048
/* zbits (optional, may be NULL; after stream so that callers of the earlier signature stay
 * valid): on the bf16 path with L <= 64 and p > 0, rs_attn_fwd stores the dropout keep decisions
 * there -- B*H*ceil(L/16)*64 uint16 words, bit 4 tk + e of word (b H + h, tq, lane) -- and
 * rs_attn_bwd given the same buffer reads them instead of drawing them again (identical draws).
 * Pass NULL to both, or the same buffer to both; elsewhere it is ignored. */
int rs_attn_fwd(const float* qkv, const uint8_t* key_pad, float* out, float* lse,
                int B, int L, int d, int H, float scale, float p, const int64_t* key, int site,
                int flags, void* stream, uint16_t* zbits);
int rs_attn_bwd(const float* qkv, const uint8_t* key_pad, const float* out, const float* dout,
                const float* lse, float* dqkv, int B, int L, int d, int H, float scale, float p,
                const int64_t* key, int site, int flags, void* stream, const uint16_t* zbits);

/* Attention for ONE query row per sample, i_b = last[b] (the final encoder layer: the encoder
 * returns context[b, last[b]] only, SequenceEncoder.py:58-74 (T7), so the final layer's other
 * query rows are dead). Keys / values: all L rows of qkv [B*L, 3d] under key_pad. out [B, d],
 * lse [B*H]. rs_attn_rows_bwd: dout [B, d] -> dqkv [B*L, 3d], every element written (dQ is zero
 * off the selected rows; dK / dV dense). Dropout draws are rs_attn_fwd's for (b, h, i_b, j).
 * flags as rs_attn_fwd (RS_GEMM_BF16: bf16-rounded operands; RS_ATTN_QKV_BF16: bf16 qkv/dqkv).
 * L <= 256, head_dim 8/16/32/64. */
int rs_attn_rows_fwd(const float* qkv, const uint8_t* key_pad, const int64_t* last, float* out,
                     float* lse, int B, int L, int d, int H, float scale, float p,
                     const int64_t* key, int site, int flags, void* stream);
int rs_attn_rows_bwd(const float* qkv, const uint8_t* key_pad, const int64_t* last,
                     const float* dout, const float* lse, float* dqkv, int B, int L, int d, int H,
                     float scale, float p, const int64_t* key, int site, int flags, void* stream);

/* ---------------------------------------------------------------- layer norm (post-LN)
 * h = dropout(a) + b (written back into a), y = LN(h)*gamma + beta; mean/rstd [M] saved.
 * Replaces norm1/norm2(x + dropout1/2(sublayer)) of TransformerEncoderLayer (K8). */
int rs_add_layernorm_fwd(float* a, const float* b, const float* gamma, const float* beta,
                         float* y, float* mean, float* rstd, int M, int N, float eps, float p,
                         const int64_t* key, int site, void* stream);
/* dh = LN backward (written to dh, may alias dy); dgamma/dbeta accumulated (+=); if da != NULL
 * da = dropout-backward(dh) (the sublayer-branch gradient). ws: rs_layernorm_ws_bytes(M, N). */
int64_t rs_layernorm_ws_bytes(int M, int N);
int rs_layernorm_bwd(const float* h, const float* dy, const float* gamma, const float* mean,
                     const float* rstd, float* dh, float* dgamma, float* dbeta, int M, int N,
                     float* da, float p, const int64_t* key, int site, float* ws, void* stream);

/* ---------------------------------------------------------------- batch norm (training)
 * x [G*Bg, C] in G independent groups of Bg rows (hard-negative slots, T13), batch statistics,
 * running stats updated group by group (momentum), num_batches_tracked += G, optional ReLU.
 * mean/rstd [G*C] saved. training == 0 normalises with the running statistics (eval mode).
 * Replaces BatchNorm1d (GenericTower.py:234, Tower.py:17; K12/K13).
 * drop_p > 0 (with relu): the MLP block's following nn.Dropout (Tower.py:19) is applied to the
 * output, mask of element (row*C + c) from (key, site) -- the rs_dropout_fwd draw. In the
 * backward, drop_scale = 1/(1-p) (1 without dropout): y > 0 <=> positive and kept, so the
 * gradient of relu-then-dropout is dy * drop_scale where y > 0. */
int64_t rs_batchnorm_ws_bytes(int G, int Bg, int C);
int rs_batchnorm_fwd(const float* x, float* y, const float* w, const float* b,
                     float* running_mean, float* running_var, int64_t* num_batches,
                     float* mean, float* rstd, int G, int Bg, int C, float momentum, float eps,
                     int relu, int training, float drop_p, const int64_t* key, int site, float* ws,
                     void* stream);
int rs_batchnorm_bwd(const float* x, const float* y, const float* dy, const float* w,
                     const float* mean, const float* rstd, float* dx, float* dw, float* db,
                     int G, int Bg, int C, int relu, float drop_scale, float* ws, void* stream);

/* ---------------------------------------------------------------- fused DSSM tower chain
 * GenericTower.feature_bn + MLP_Tower in training mode (GenericTower.py:229-236, Tower.py:16-41;
 * K12-K14): one kernel per Linear. A BatchNorm's batch statistics are produced by the kernel
 * that writes its input: per-row-tile column values go to `part` (rs_tower_part_floats(G, Bg, N,
 * kind) floats; kind 0 = rs_tower_stats, 1 = the GEMM kernels) and the last workgroup of each
 * (group, 64-column block) merges them in a fixed order and publishes the results; `sync` is
 * rs_tower_sync_ints(G, N) ints that must be ZERO on entry (they are zero again on exit:
 * allocate once, reuse), `scratch` is G * 2 * N doubles. bf16 != 0: GEMM operands rounded to
 * bf16 (bf16 compute mode), fp32 otherwise; accumulation and every stored tensor fp32.
 *
 * rs_tower_stats: feature_bn's batch statistics of x [G*Bg, C] (GenericTower.py:234): mean /
 *   rstd [G*C] published, running statistics updated group by group (momentum, unbiased
 *   variance), num_batches_tracked += G. rng_state non-NULL: also the MLP's dropout key of this
 *   step, key_out[0..1] = rng_state[0..1], rng_state[1] += 1 (rs_rng_next folded in).
 * rs_tower_fwd: A [G*Bg, K] -> BN with the published in_mean / in_rstd and bn_w / bn_b (+ ReLU
 *   + dropout (key, site) when relu: the rs_dropout_fwd draw of element row*K + k, Tower.py:17-19)
 *   -> h (written to h_out when non-NULL: the weight-gradient operand) -> h W^T + bias (W [N][K],
 *   nn.Linear, Tower.py:16). Hidden layer: z [G*Bg, N] with the statistics of ITS BatchNorm
 *   published as for rs_tower_stats (mean / rstd, running statistics); final layer (z == NULL):
 *   out = F.normalize(.) (Tower.py:41) and norm [G*Bg] (N <= 128).
 * rs_tower_bwd: the input gradient through one Linear. Prologue, y != NULL: dz = F.normalize
 *   backward of gin (y = out, norm); else dz = BatchNorm backward of gin (the masked gradient at
 *   that BN's output) from z, its mean / rstd / bn_w and the published means mg, mgx of g and
 *   g*xhat. dz is written (the weight-gradient operand). N > 0: g = mask(dz W) (W [K][N]), mask =
 *   the ReLU + dropout of the BatchNorm below (e_relu, e_drop_p, e_key, e_site; recomputed from
 *   its pre-BN ez and e_mean / e_rstd / e_w / e_b), written, and that BatchNorm's means of g and
 *   g*xhat published to out_mg / out_mgx with e_dgamma += sum g*xhat, e_dbeta += sum g.
 *   N == 0: dz is feature_bn's dx (no GEMM). */
int64_t rs_tower_part_floats(int G, int Bg, int N, int kind);
/* profiling only: per-workgroup phase timestamps of the tower GEMM kernels into buf (NULL: off) */
int rs_tower_debug_buffer(unsigned long long* buf);
int rs_tower_sync_ints(int G, int N);
int rs_tower_stats(const float* x, int G, int Bg, int C, float* part, int* sync, double* scratch,
                   float* mean, float* rstd, float* running_mean, float* running_var,
                   int64_t* num_batches, float momentum, float eps, int64_t* rng_state, int64_t* key_out,
                   void* stream);
int rs_tower_fwd(const float* A, int G, int Bg, int K, const float* in_mean, const float* in_rstd,
                 const float* bn_w, const float* bn_b, int relu, float drop_p, const int64_t* key,
                 int site, float* h_out, const float* W, const float* bias, int N, float* z,
                 float* part, int* sync, double* scratch, float* mean, float* rstd,
                 float* running_mean, float* running_var, int64_t* num_batches, float momentum,
                 float eps, float* out, float* norm, float l2_eps, int bf16, void* stream);
/* Weight gradients of up to 4 tower Linears in one launch (bf16 compute mode; Tower.py:16 nn.Linear
 * backward): per layer i, dW_i [N_i][K_i] += dz_i^T h_i over M rows, db_i [N_i] += colsum(dz_i)
 * (db_i may be NULL). ws_i: rs_tower_wgrad_ws_floats(M, N_i, K_i) floats of scratch; sync_i:
 * rs_tower_wgrad_sync_ints(N_i, K_i) ints, zero on entry and again on exit. The row splits of a
 * tile are summed in a fixed order (deterministic). Host arrays (Ns, Ks, pointer arrays) are read
 * during the call only. bf16 != 0: products of bf16-rounded operands; 0: exact fp32 products. */
int rs_tower_wgrad_split(int M, int N, int K);
int64_t rs_tower_wgrad_ws_floats(int M, int N, int K);
int rs_tower_wgrad_sync_ints(int N, int K);
int rs_tower_wgrad(int nlayers, int M, const int* Ns, const int* Ks, const float* const* dz,
                   const float* const* h, float* const* dW, float* const* db, float* const* ws,
                   int* const* sync, int bf16, void* stream);
int rs_tower_bwd(const float* gin, int G, int Bg, int K, const float* y, const float* norm,
                 float l2_eps, const float* z, const float* mean, const float* rstd,
                 const float* bn_w, const float* mg, const float* mgx, float* dz, const float* W,
                 int N, const float* ez, const float* e_mean, const float* e_rstd,
                 const float* e_w, const float* e_b, int e_relu, float e_drop_p,
                 const int64_t* e_key, int e_site, float* g, float* part, int* sync,
                 double* scratch, float* out_mg, float* out_mgx, float* e_dgamma, float* e_dbeta,
                 int bf16, void* stream);

/* ---------------------------------------------------------------- misc elementwise */
/* y = x / max(||x||_2, eps) per row (F.normalize, Tower.py:41; K14); norm [M] saved */
int rs_l2norm_fwd(const float* x, float* y, float* norm, int M, int N, float eps, void* stream);
int rs_l2norm_bwd(const float* y, const float* norm, const float* dy, float* dx, int M, int N,
                  float eps, void* stream);

/* ---------------------------------------------------------------- in-batch softmax loss
 * logits = S/T (S = U I^T, [B, ld_s]), off-diagonal equal-item-id collisions -> -1e9, hard
 * negative logits U_i.H_in/T appended un-masked, cross-entropy with labels arange(B), mean.
 * item_ids may be NULL (compute_loss(item_ids=None): no collision mask).
 * TwoTowerModel.compute_loss (TwoTowerModel.py:81-140; trap T12; K15-K17).
 * fwd: per-row lse [B] and the mean loss (scalar) ; bwd: S <- dlogits (in place, scaled by
 * *grad_out / B / T so the next GEMMs need alpha 1), dhl [B, N] likewise.
 * Hard negatives: element (i, n, c) of H at Hn[i*h_row_stride + n*h_slot_stride + c] (0, 0 =
 * contiguous [B, N, D]; the grouped item-tower pass hands over [N, B, D] as row D, slot B*D). */
int rs_inbatch_ce_fwd(const float* S, int ld_s, const float* U, const float* Hn,
                      int64_t h_row_stride, int64_t h_slot_stride,
                      const int64_t* item_ids, int64_t id_stride, int B, int N, int D, float T,
                      float* lse, float* row_loss, float* loss, void* stream);
int rs_inbatch_ce_bwd(float* S, int ld_s, const float* U, const float* Hn,
                      int64_t h_row_stride, int64_t h_slot_stride,
                      const int64_t* item_ids, int64_t id_stride, int B, int N, int D, float T,
                      const float* lse, const float* grad_out, float* dhl, void* stream);
/* The logits matrix of the same loss, materialised: out [B, ld_out >= B + N] (diagnostics and
 * TwoTowerModel.compute_logits; the loss kernels never store it). */
int rs_inbatch_logits(const float* S, int ld_s, const float* U, const float* Hn,
                      int64_t h_row_stride, int64_t h_slot_stride, const int64_t* item_ids,
                      int64_t id_stride, int B, int N, int D, float T, float* out, int64_t ld_out,
                      void* stream);
/* The same loss with S never stored (bf16 compute mode; D = 64 or 128): the 32 x 32 tiles of
 * U I^T are recomputed on bf16 MFMA where needed -- an online log-sum-exp per user in the
 * forward, dU = dS I and dI = dS^T U accumulated from dS tiles held in registers in the
 * backward (fixed-order split reduction). Same semantics as the pair above (collision mask,
 * hard negatives, mean); the products run on bf16-rounded U, I. ws: rs_inbatch_ce_fused_ws_bytes.
 * The backward writes dU, dI (overwrite) and dhl; rs_hardneg_bwd then adds the hard-negative
 * terms to dU and writes dH. */
int64_t rs_inbatch_ce_fused_ws_bytes(int B, int D);
int rs_inbatch_ce_fused_fwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                            int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                            int N, int D, float T, float* lse, float* row_loss, float* loss, float* ws,
                            void* stream);
int rs_inbatch_ce_fused_bwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                            int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                            int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                            float* dI, float* dhl, float* ws, void* stream);
/* The bf16 pair with the rounding of U and I done once, in the forward's tiles: the forward also
 * writes ui_bf16 ([2][B][D] bf16, U then I, 16-byte aligned), which the backward streams instead
 * of rounding U and I in a launch of its own (keep it from forward to backward). Same results. */
int rs_inbatch_ce_fused_fwd_uib(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                int N, int D, float T, float* lse, float* row_loss, float* loss, float* ws,
                                void* ui_bf16, void* stream);
int rs_inbatch_ce_fused_bwd_uib(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                                float* dI, float* dhl, float* ws, const void* ui_bf16, void* stream);
/* The same pair in fp32 compute mode: the tiles run on v_mfma_f32_32x32x2_f32 with fp32 operands
 * (exact f32 products, no rounding of U, I); same arguments, workspace and outputs, plus S:
 * [B][rs_inbatch_ce_s_ld(B)] fp32 scratch that the forward fills with U I^T (raw dot products)
 * and the backward reads instead of recomputing the tiles (keep it from forward to backward). */
int64_t rs_inbatch_ce_s_ld(int B);
int rs_inbatch_ce_fused_f32_fwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                int N, int D, float T, float* lse, float* row_loss, float* loss, float* S,
                                float* ws, void* stream);
int rs_inbatch_ce_fused_f32_bwd(const float* U, const float* I, const float* Hn, int64_t h_row_stride,
                                int64_t h_slot_stride, const int64_t* item_ids, int64_t id_stride, int B,
                                int N, int D, float T, const float* lse, const float* grad_out, float* dU,
                                float* dI, float* dhl, const float* S, float* ws, void* stream);
/* dU[i] += sum_n dhl[i,n] H[i,n];  dH[i,n] = dhl[i,n] U[i]   (hard-negative bmm backward; dH in
 * the layout of H) */
int rs_hardneg_bwd(const float* U, const float* Hn, int64_t h_row_stride, int64_t h_slot_stride,
                   const float* dhl, float* dU, float* dH, int B, int N, int D, void* stream);

/* ---------------------------------------------------------------- hard-negative catalog
 * Materialise N item-tower feature rows per sample from an on-device item catalog (SURVEY §8f.2;
 * the reference leaves `hard_negatives` as a TODO in CombineTwoTower.py:86-90 and samples the
 * ids in parsing.py:215-250): out[(n*B + b)*ld_out + f] = cat[ids[b*ld_ids + n]*ld_cat + f] for
 * f < F, i.e. the N slots stacked along the batch ([N*B, F], one grouped tower pass). elem = 4
 * or 8 bytes (copied as is); widen = 1 reads int32 and writes int64 (id columns). An id outside
 * [0, V) writes zeros (the padding row) and sets *err_flag |= 1. */
int rs_catalog_gather(const void* cat, int elem, int widen, int64_t V, int F, int64_t ld_cat,
                      const int64_t* ids, int B, int N, int64_t ld_ids, void* out, int64_t ld_out,
                      int* err_flag, void* stream);

/* ---------------------------------------------------------------- device batch assembly
 * The ragged part of collate_fn (DataLoader.py:250-288; per tower in CombineTwoTower.py:62-92):
 * rows idx[0..B) of a CSR list column (values [nnz, tw] int32 (elem 4) or int64 (elem 8),
 * offsets [rows + 1] int64) -> out [B, Lb, tw] int64, zero right-padded (np.pad(..., 0)); Lb >=
 * the longest selected list (the caller's batch maximum, as the reference pads to it). Row index
 * out of range: zeros, *err_flag |= 1; a list longer than Lb: truncated, *err_flag |= 2.
 * Fixed-width columns (sparse id matrix, dense matrix) use rs_catalog_gather with N = 1. */
/* dst[i][0 .. bytes[i]) = src[i][...] for i < n <= 32 device buffers, one launch (host arrays read
 * during the call only; the copies must not overlap). */
int rs_copy_many(int n, const void* const* src, void* const* dst, const int64_t* bytes, void* stream);
int rs_collate_ragged(const void* values, int elem, int tw, const int64_t* offsets, int64_t rows,
                      const int64_t* idx, int B, int Lb, int64_t* out, int* err_flag, void* stream);

/* ---------------------------------------------------------------- validation / Recall@K
 * The reference's validate() (training_utils.py:121-275) on the device: scores = U I_all^T via
 * rs_gemm_f32, then
 *   rs_mask_history: column c = hist_idx[j] -> -inf for j in [hist_off[u], hist_off[u+1]), u =
 *     user_ids[b*uid_stride] (CSR of each user's training items as catalog column indices;
 *     replaces the per-user Python loop :238-252); S holds catalog columns [col0, col0+ncols)
 *     (one column chunk) at S[b*ld + c - col0];
 *   rs_topk_rows: per row the K (<= 256) largest of S[b, 0:N], sorted descending, ties by the
 *     lower column; out_idx[b*ld_out + i] = column + col_offset, or idx_in[b*ld_idx_in + column]
 *     when idx_in is given (merging per-chunk candidates); out_val nullable (torch.topk :256);
 *   rs_recall_hits: hits[i] += #rows whose target item is among the first ks[i] of its list
 *     (item_ids[col] == targets[b*target_stride]; :258-262). */
int rs_mask_history(float* S, int64_t ld, int B, int64_t col0, int64_t ncols,
                    const int64_t* user_ids, int64_t uid_stride, const int64_t* hist_off,
                    const int32_t* hist_idx, int64_t num_users, void* stream);
int rs_topk_rows(const float* S, int64_t ld, int B, int N, int K, const int32_t* idx_in,
                 int64_t ld_idx_in, int col_offset, int32_t* out_idx, float* out_val,
                 int64_t ld_out, void* stream);
int rs_recall_hits(const int32_t* topk_idx, int B, int K, const int64_t* item_ids,
                   const int64_t* targets, int64_t target_stride, const int32_t* ks, int nk,
                   int32_t* hits, void* stream);

/* ---------------------------------------------------------------- clip + Adam
 * Flat multi-tensor path over a contiguous fp32 range (all parameters packed in one buffer).
 * rs_grad_sqnorm: partial sums of (scale*g)^2 into ws; rs_clip_coef: total norm and
 * coef = min(1, max_norm/(norm+1e-6)) written to device scalars (clip_grad_norm_,
 * training_utils.py:53-54; K18). rs_adam_step: torch.optim.Adam (default betas/eps, L2
 * weight decay) on p, m, v with g*scale*(*coef) (train_twotower.py:111; K19); when
 * write_grad != 0 the clipped gradient is stored back into g. With step_dev != NULL the bias
 * corrections use the device step count *step_dev instead of `step`. */
int64_t rs_sqnorm_ws_bytes(int64_t n);
int rs_sqnorm_parts(int64_t n);          /* number of double partials rs_grad_sqnorm writes */
int rs_grad_sqnorm(const float* g, int64_t n, float scale, double* ws, void* stream);
/* sums nparts double partials (dense + sparse-table contributions) into norm and coef */
int rs_clip_coef(const double* ws, int nparts, float max_norm, float* total_norm, float* coef,
                 void* stream);
/* the same, and *counter += 1 in the same launch (the optimizer's device step count, which
 * rs_adam_step's step_dev then reads: the step that clips needs no separate counter launch) */
/* the same, and in the same launch the lazy tables' Adam constants of the next step (rs_adam_prepare:
 * *step += 1, consts[*step] = {lr / bc1, 1 / sqrt(bc2)}); one launch instead of two (round 5) */
int rs_clip_coef_prepare(const double* ws, int nparts, float max_norm, float* total_norm, float* coef,
                         int64_t* step, float* consts, int cap, float lr, float beta1, float beta2,
                         void* stream);
int rs_clip_coef_step(const double* ws, int nparts, float max_norm, float* total_norm, float* coef,
                      int64_t* counter, void* stream);
/* rs_grad_sqnorm + rs_clip_coef_step in one launch (round 5): the last workgroup of the partials
 * makes the coefficient (same bits) and advances *counter (nullable). ticket: one int, zero
 * before the first call; the call leaves it zero (clip_grad_norm_, training_utils.py:53-54) */
int rs_grad_sqnorm_clip_step(const float* g, int64_t n, float scale, double* ws, int* ticket, float max_norm,
                             float* total_norm, float* coef, int64_t* counter, void* stream);
int rs_scale_inplace(float* g, int64_t n, float scale, const float* coef, void* stream);
int rs_adam_step(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1,
                 float beta2, float eps, float weight_decay, int step, const int64_t* step_dev,
                 float scale, const float* coef, int write_grad, void* stream);
/* *counter += delta on the stream (device-side Adam step count: replayable in a hipGraph) */
int rs_counter_add(int64_t* counter, int64_t delta, void* stream);

/* ---------------------------------------------------------------- lazy-exact Adam (large tables)
 * Dense-gradient Adam semantics (every row moves every step, T16) without sweeping the table:
 * rows carry last[V][2] int32 = the optimizer step a row's moments (m, v) and its parameters (p)
 * were last brought to (p can be ahead: with weight_decay == 0 the forward catch-up writes p
 * alone and the optimizer step replays the moments again; otherwise the two are equal); consts[s] =
 * {lr/bc1(s), sqrt(bc2(s))} is written once per step by rs_adam_prepare (which also advances
 * the device step count; consts[0] holds {capacity, overflow flag} as int bits and every reader
 * clamps its step index to the capacity). rs_sparse_flush brings every row to the current step
 * (checkpoint / state_dict). The per-step row work runs over sorted lookups (below).
 * Replaces torch.optim.Adam on sparse=False embeddings (GenericTower.py:45-49; train_twotower.py:111). */
int rs_adam_prepare(int64_t* step, float* consts, int cap, float lr, float beta1, float beta2,
                    void* stream);
int rs_sparse_flush(float* p, float* m, float* v, int* last, int64_t V, int D, const int64_t* step,
                    const float* consts, float beta1, float beta2, float eps, float weight_decay,
                    void* stream);

/* ---------------------------------------------------------------- sorted lookups (large tables)
 * One forward lookup of a large table (a [rows, bag] id matrix, int64 or int32, row stride
 * row_stride) is sorted by row id: keys[n] ascending (ids outside [0, vocab) last, as
 * 0xFFFFFFFF), vals[n] = the lookup index r * bag + l, ascending within a row (stable LSD radix
 * sort of rs_lookup_sort_ws_bytes of workspace; n <= 4096: one workgroup's radix passes, one
 * launch; 4096 < n <= 8192: a counting sort over the whole chip, two launches).
 * Every per-row operation then walks the distinct rows (run heads) of keys:
 *   rs_sorted_catchup  replay skipped zero-gradient Adam steps before the gather reads the rows
 *                      (bitwise equal to dense Adam); rs_lookup_catchup does the same straight
 *                      from the unsorted id matrix (one compare-and-swap on last[row] picks the
 *                      lookup that replays the row), so the sort can leave the forward path;
 *   rs_segsum          the table gradient = embedding_dense_backward of the call
 *                      (GenericTower.py:182; pooled mean/sum GenericTower.py:141-162): per row
 *                      the contributions of its lookups in lookup order (mode 0: dout row r per
 *                      lookup, 1: dout row / bag, 2: dout row), `pad` skipped; plain stores
 *                      (accumulate = 1: added to the row), no atomics, bitwise reproducible;
 *                      dout points at the feature's first column, row stride ldo floats;
 *   rs_sorted_sqnorm   clip-norm partials (rs_sorted_sqnorm_parts doubles into ws);
 *   rs_sorted_adam     step t on each row with its (scaled, clipped) gradient, gradient zeroed;
 *   rs_sorted_owner    owner[row] = min(owner[row], call): with several calls in a step, sqnorm
 *                      and Adam take a row only in the call equal to its owner (Adam resets it);
 *   rs_sorted_zero_grad zero the rows' gradient.
 * rs_pack_ids / rs_pack_rows: contiguous int32 ids and gradient rows of a call for the
 * data-parallel all-gather (each rank then sorts and segment-sums the gathered
 * calls, so all ranks hold bitwise-identical table gradients; replaces a dense all-reduce of
 * [V, D] embedding gradients). */
int64_t rs_lookup_sort_ws_bytes(int64_t n, int64_t vocab);
int rs_lookup_sort(const void* ids, int id_bytes, int rows, int bag, int64_t row_stride,
                   int64_t vocab, uint32_t* keys, uint32_t* vals, void* ws, void* stream);
int rs_sorted_catchup(const uint32_t* keys, int64_t n, int D, float* p, float* m, float* v,
                      int* last, const int64_t* step, const float* consts, float beta1, float beta2,
                      float eps, float weight_decay, void* stream);
int rs_lookup_catchup(const void* ids, int id_bytes, int rows, int bag, int64_t row_stride,
                      int64_t vocab, int D, float* p, float* m, float* v, int* last,
                      const int64_t* step, const float* consts, float beta1, float beta2, float eps,
                      float weight_decay, void* stream);
/* Several sorted calls in one launch (at most 8, every D in one lanes-per-row class: D <= 16, 32,
 * 64, 128, else). keys, n, D, call and owner as for the single-call entry points; p, m, v, last
 * (Adam) and g are the call's table slices. rs_sorted_sqnorm_batch writes call c's
 * rs_sorted_sqnorm_parts() partials at ws + c * parts. */
typedef struct rs_sorted_call {
  const uint32_t* keys;
  int64_t n;
  int D;
  int call;
  float* p;
  float* g;
  float* m;
  float* v;
  int* last;
  int* owner;
} rs_sorted_call_t;
int rs_sorted_adam_batch(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                         const float* consts, float beta1, float beta2, float eps, float weight_decay,
                         float scale, const float* coef, void* stream);
/* rs_sorted_catchup of up to 8 sorted calls (of one row-width class) in one launch (round 6):
 * each call's distinct rows brought to the optimizer step (g, owner unused). Replaces back-to-back
 * forward catch-ups of several large tables (GenericTower.py:150-157: the tower's lookups). */
int rs_sorted_catchup_batch(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                            const float* consts, float beta1, float beta2, float eps, float weight_decay,
                            void* stream);
/* The same two batches with the flat buffer's dense region [0, n) in the same launch (round 5):
 * rs_grad_sqnorm's partials of g (rs_sqnorm_parts(n) of them) into ws_dense, and rs_adam_step's
 * update of p, g, m, v (step constants from *step, lr) -- the same partitions, the same bits as the
 * separate launches (clip_grad_norm_ + Adam.step, training_utils.py:53-56, train_twotower.py:111). */
int rs_sorted_sqnorm_batch_dense(const rs_sorted_call_t* calls, int ncalls, float scale, double* ws,
                                 const float* g, int64_t n, double* ws_dense, void* stream);
int rs_sorted_adam_batch_dense(const rs_sorted_call_t* calls, int ncalls, const int64_t* step,
                               const float* consts, float beta1, float beta2, float eps, float weight_decay,
                               float scale, const float* coef, float* p, float* g, float* m, float* v,
                               int64_t n, float lr, void* stream);
int rs_sorted_sqnorm_batch(const rs_sorted_call_t* calls, int ncalls, float scale, double* ws,
                           void* stream);
int rs_sorted_adam(const uint32_t* keys, int64_t n, int D, float* p, float* g, float* m, float* v,
                   int* last, int* owner, int call, const int64_t* step, const float* consts,
                   float beta1, float beta2, float eps, float weight_decay, float scale,
                   const float* coef, void* stream);
int rs_sorted_sqnorm_parts(void);
int rs_sorted_sqnorm(const uint32_t* keys, int64_t n, int D, const float* g, int* owner, int call,
                     float scale, double* ws, void* stream);
int rs_sorted_owner(const uint32_t* keys, int64_t n, int* owner, int call, void* stream);
int rs_sorted_zero_grad(const uint32_t* keys, int64_t n, int D, float* g, void* stream);
int64_t rs_segsum_ws_bytes(int64_t n, int D);
int rs_segsum(const uint32_t* keys, const uint32_t* vals, int64_t n, int bag, int mode, int64_t pad,
              const float* dout, int64_t ldo, int D, float* grad, int accumulate, void* ws,
              void* stream);
/* Up to 4 rs_segsum calls of one row width D on DIFFERENT tables (distinct grad) in one launch
 * pair (round 5); each call's arguments as rs_segsum's, its own ws (rs_segsum_ws_bytes), n >= 1.
 * Same results as the calls one by one. */
typedef struct rs_segsum_call {
  const uint32_t* keys;
  const uint32_t* vals;
  int64_t n;
  int bag;
  int mode;
  int64_t pad;
  const float* dout;
  int64_t ldo;
  float* grad;
  int accumulate;
  void* ws;
} rs_segsum_call_t;
int rs_segsum_batch(const rs_segsum_call_t* calls, int ncalls, int D, void* stream);
/* Row-sharded large tables under data parallelism (dist.py): rank r of W owns rows id % W == r
 * at local row id / W. Maps all-gathered int32 ids to int64 local rows (-1: owned elsewhere);
 * out-of-range ids set *err_flag (nullable) as rs_gather_fwd does (GenericTower.py:184-196),
 * except INT32_MIN: the empty pad slot of a ragged call's exchange (ranks' bags of different
 * lengths padded to a common shape). */
int rs_shard_map_ids(const int32_t* ids, int64_t n, int64_t vocab, int world, int rank, int64_t* local,
                     int* err_flag, void* stream);
/* All-to-all row exchange of a one-id-per-row lookup of a row-sharded table (csrc/shard.hip;
 * replaces the reference's nn.Embedding lookup, GenericTower.py:182 / SequenceFeatureProcessor.py:60,
 * when the table is split across ranks). rs_shard_bucket, from a call's sorted keys / vals
 * (rs_lookup_sort over global ids): its distinct ids packed per owner into send_ids [world][cap]
 * (the owner's local row id / world), counts[o] (capped; *flag |= 2 past cap), idx [n] (lookup
 * order: the slot o * cap + s holding the lookup's row once the rows come back) and ckey [n]
 * (sorted order: the slot, or 0xFFFFFFFF for the padding id / out-of-range ids, the keys of the
 * backward's segment sum into the [world * cap, D] slot gradient; *flag |= 1 on an out-of-range
 * id). rs_shard_recv, owner side: received slots as gather ids (ids64, invalid slots -> 0) and
 * sort ids (ids32, invalid -> vocab: sorted last and skipped). */
int64_t rs_shard_bucket_ws_bytes(int64_t n, int world);
int rs_shard_bucket(const uint32_t* keys, const uint32_t* vals, int64_t n, int world, int cap, int64_t pad,
                    int32_t* send_ids, int* counts, uint32_t* ckey, int64_t* idx, int* flag, void* ws,
                    void* stream);
int rs_shard_recv(const int32_t* recv_ids, const int* recv_counts, int world, int cap, int64_t vocab,
                  int64_t* ids64, int32_t* ids32, int* flag, void* stream);
int rs_pack_ids(const void* ids, int id_bytes, int64_t rows, int bag, int64_t row_stride,
                int32_t* out, void* stream);
int rs_pack_rows(const float* src, int64_t ld, int64_t rows, int D, float* dst, void* stream);
/* rs_pool_max_grad: a max-pooled [rows, bag] lookup's backward as per-lookup gradient rows
 * out [rows * bag, D]: dout[r] at the first arg-max position of each column of bag r (torch.max(dim)
 * backward), zero elsewhere (and for the padding id / invalid ids) -- the data-parallel exchange
 * then treats the call as rows * bag single-id lookups. Replaces the arg-max scatter of
 * GenericTower.py:159-160's pooled max under data parallelism. */
int rs_pool_max_grad(const float* table, const void* ids, int id_bytes, int64_t rows, int bag, int64_t row_stride,
                     int64_t vocab, int D, int64_t pad, const float* dout, int64_t ldo, float* out, void* stream);

/* ---------------------------------------------------------------- dropout
 * Counter-based masks: element i of site `site` is kept iff hash(key[0], key[1], site, i) >= p,
 * kept values scaled by 1/(1-p) (nn.Dropout semantics). key = {seed, counter} in device memory;
 * rs_rng_next copies the state into a fresh key and advances the counter (graph-replay safe).
 * rs_dropout_fwd: x = dropout(x + aux[(i/N % aux_mod)*ld_aux + i%N])  (aux optional: the
 * positional embedding between the two input dropouts, SequenceFeatureProcessor.py:77-83).
 * rs_dropout_bwd: dx *= mask/(1-p). */
int rs_rng_next(int64_t* state, int64_t* key, void* stream);
int rs_dropout_fwd(float* x, int64_t n, int N, const float* aux, int ld_aux, int aux_mod, float p,
                   const int64_t* key, int site, void* stream);
/* Backward of SequenceFeatureProcessor's drop_b(drop_a(.) + pos[l]) (SequenceFeatureProcessor.py:
 * 77-83) in one pass over dx [rows, N = L*d]: dx <- dx * mask_b * mask_a, pos_grad[n] += sum over
 * rows of dx * mask_b (deterministic). Replaces rs_dropout_bwd + rs_colsum + rs_dropout_bwd.
 * ws: rs_seq_input_dropout_bwd_ws_bytes. */
int64_t rs_seq_input_dropout_bwd_ws_bytes(int rows, int N);
int rs_seq_input_dropout_bwd(float* dx, int rows, int N, float p, const int64_t* key, int site_a,
                             int site_b, float* pos_grad, float* ws, void* stream);
int rs_dropout_bwd(float* dx, int64_t n, float p, const int64_t* key, int site, void* stream);

/* ---------------------------------------------------------------- reductions */
/* Deferred parameter-gradient reductions (round 5; no reference counterpart -- the optimizer step
 * of training_utils.py:28-60 is the only reader of these gradients). After rs_reduce_defer(1) the
 * weight-gradient entry points (rs_gemm_f32's transposed-A weight gradients, rs_wgrad_bf16,
 * rs_ffn_wgrad_bf16), the fused FFN backward's LayerNorm partials and rs_seq_input_dropout_bwd's
 * positional partials queue their final split reduction instead of launching it; rs_reduce_flush
 * runs every queued reduction in one launch on `stream` (the bits of the immediate path) and
 * rs_reduce_defer(0) ends the queueing. The caller keeps each call's workspace alive until the
 * flush is queued, and reads none of those gradients before it. */
int rs_reduce_defer(int on);
int rs_reduce_flush(void* stream);
/* out = scale * sum(x[0..n)) (deterministic; mean loss) */
int rs_sum(const float* x, int n, float scale, float* out, void* stream);
/* *flag |= bit if x[0..n) holds a NaN (x 16-byte aligned). The loss inputs' NaN guard of
 * TwoTowerModel.compute_loss (TwoTowerModel.py:88-91, 99-100): checked on the device every step,
 * raised by the host at its log-point sync. */
/* The same for up to 4 tensors in one launch: flag |= bits[i] if x[i][0 .. n[i]) holds a NaN
 * (host arrays read during the call only). */
int rs_nan_check_many(int k, const float* const* x, const int64_t* n, const int* bits, int* flag,
                      void* stream);
int rs_nan_check(const float* x, int64_t n, int* flag, int bit, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RSYS_HIP_H */
