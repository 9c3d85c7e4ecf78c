"""Thin tensor-level wrappers over the C ABI (pointers, strides, current HIP stream).

Only torch is used here for device memory (torch.empty on the caching allocator) and for the
current stream handle; all arithmetic runs in librsys_hip.so.
"""
from __future__ import annotations

import contextlib
import os
import threading

import numpy as np
import torch

from . import _hip, precision
from ._hip import call

_ZERO = {}


def P(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


class _DeferState(threading.local):
    """deferred_reduce's scope state, per host thread like the library's queue (csrc/reduce.hip
    g_defer / g_jobs are thread_local): a scope opened on one thread (the autograd device thread
    running the encoder backward) neither sees nor keeps another thread's workspaces."""

    def __init__(self):
        self.keep = []  # the workspaces of each open scope, alive until its flush is queued


_DEFER = _DeferState()


def ws(nbytes: int, device) -> torch.Tensor:
    """Workspace from the caching allocator (capture-safe)."""
    t = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
    if _DEFER.keep:
        _DEFER.keep[-1].append(t)  # a queued reduction reads it at the flush
    return t


@contextlib.contextmanager
def deferred_reduce(on=True):
    """The parameter-gradient reductions queued inside run as ONE launch at the end of the scope
    (rs_reduce_defer / rs_reduce_flush, round 5): nothing inside may read those gradients. Off
    (plain pass-through) when `on` is false, in a nested scope, or with RSYS_DEFER_REDUCE=0. The
    scope belongs to the calling host thread (library-side queue and this side's workspaces are
    thread-local): reductions issued by other threads meanwhile are not deferred."""
    if not on or _DEFER.keep or os.environ.get('RSYS_DEFER_REDUCE', '1') == '0':
        yield
        return
    _DEFER.keep.append([])
    call('rs_reduce_defer', 1)
    try:
        yield
    finally:
        call('rs_reduce_defer', 0)
        try:
            call('rs_reduce_flush', stream())
        finally:
            _DEFER.keep.pop()


def gemm(A, B, C, M, N, K, *, transA, transB, lda, ldb, ldc, alpha=1.0, beta=0.0, epi=0,
         bias=None, aux=None, ld_aux=0, aux_mod=0, split=None, rowsum=None, drop_p=0.0,
         drop_key=None, site_a=0, site_b=0):
    L = _hip.lib()
    if split is None:
        split = L.rs_gemm_auto_split(M, N, K)
    w = None
    if split > 1:
        w = ws(L.rs_gemm_ws_bytes(M, N, K, split), C.device)
    call('rs_gemm_f32', int(transA), int(transB), M, N, K, float(alpha), P(A), lda, P(B), ldb,
         float(beta), P(C), ldc, epi | precision.gemm_flags(), P(bias), P(aux), ld_aux, aux_mod,
         float(drop_p), P(drop_key),
         site_a, site_b, P(rowsum), split, P(w), stream())
    return C


def _io_flags(a, c):
    """bf16 storage of the A operand / the output C (bf16 compute mode, streaming instances)."""
    return (_hip.RS_GEMM_A_BF16 if a.dtype == torch.bfloat16 else 0) | \
        (_hip.RS_GEMM_C_BF16 if c.dtype == torch.bfloat16 else 0)


def linear_fwd(x, W, b=None, out=None, *, relu=False, aux=None, aux_mod=0, beta=0.0,
               drop_p=0.0, drop_key=None, site_a=None, site_b=None, out_dtype=torch.float32):
    """out[M,N] = drop_b(drop_a(relu(x[M,K] @ W[N,K]^T + b)) + aux[m % aux_mod]) (+ beta*out);
    dropout stages are active when drop_p > 0 and their site is given. out_dtype bf16: the
    result is stored as bf16 (only for outputs consumed as bf16 MFMA operands)."""
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=out_dtype)
    epi = (_hip.RS_EPI_BIAS if b is not None else 0) | (_hip.RS_EPI_RELU if relu else 0) | \
        (_hip.RS_EPI_AUX_ADD if aux is not None else 0) | _io_flags(x, out)
    if drop_p > 0:
        epi |= (_hip.RS_EPI_DROP_A if site_a is not None else 0) | (_hip.RS_EPI_DROP_B if site_b is not None else 0)
    return gemm(x, W, out, M, N, K, transA=0, transB=1, lda=x.stride(0), ldb=W.stride(0),
                ldc=out.stride(0), beta=beta, epi=epi, bias=b, aux=aux,
                ld_aux=(aux.stride(0) if aux is not None else 0), aux_mod=aux_mod, drop_p=drop_p,
                drop_key=drop_key, site_a=site_a or 0, site_b=site_b or 0)


def linear_bwd_input(dy, W, out=None, *, beta=0.0, relu_mask_of=None, alpha=1.0):
    """out[M,K] = (dy[M,N] @ W[N,K]) (* (relu_mask_of > 0)) (+ beta*out)."""
    M, N = dy.shape
    K = W.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=torch.float32)
    epi = (_hip.RS_EPI_AUX_MASK if relu_mask_of is not None else 0) | _io_flags(dy, out)
    return gemm(dy, W, out, M, K, N, transA=0, transB=0, lda=dy.stride(0), ldb=W.stride(0),
                ldc=out.stride(0), alpha=alpha, beta=beta, epi=epi, aux=relu_mask_of,
                ld_aux=(relu_mask_of.stride(0) if relu_mask_of is not None else 0))


def linear_bwd_weight(dy, x, dW, *, beta=1.0, db=None):
    """dW[N,K] (+)= dy[M,N]^T @ x[M,K] (reduction over M, split-K); db[N] += colsum(dy) fused."""
    M, N = dy.shape
    K = x.shape[1]
    return gemm(dy, x, dW, N, K, M, transA=1, transB=0, lda=dy.stride(0), ldb=x.stride(0),
                ldc=dW.stride(0), beta=beta, rowsum=db)


def ffn_supported(x, W1):
    """The fused feed-forward block: bf16 compute mode, d_model 64, dim_feedforward 256."""
    return (precision.compute_dtype() == 'bf16' and not os.environ.get('RSYS_UNFUSED_FFN') and
            x.dim() == 2 and x.shape[1] == 64 and
            tuple(W1.shape) == (256, 64) and x.shape[0] % 16 == 0 and x.is_contiguous())


def ffn_fwd_bf16(x, W1, b1, W2, b2, gamma, beta, eps, p, key, site1, site2):
    """x2 = LN(x + drop2(linear2(drop(relu(linear1(x)))))) -> (h, x2, mean, rstd, mask)."""
    M, F = x.shape[0], W1.shape[0]
    dev = x.device
    h = torch.empty(M, 64, device=dev)
    y = torch.empty(M, 64, device=dev)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    mask = torch.empty(int(_hip.lib().rs_ffn_mask_words(M, F)), dtype=torch.int64, device=dev)
    call('rs_ffn_fwd_bf16', M, F, P(x), P(W1), P(b1), P(W2), P(b2), P(gamma), P(beta), float(eps), P(h),
         P(y), P(mean), P(rstd), P(mask), float(p), P(key), site1, site2, stream())
    return h, y, mean, rstd, mask


def ffn_bwd_bf16(x, W1, b1, W2, mask, dff, dres, p, dx=None, acts=True):
    """-> (dx = dres + dPre1 W1, f1 bf16 [M,F], dPre1 bf16 [M,F]); acts=False: f1 / dPre1 are
    not written (None; the weight gradients by ffn_wgrad_bf16)."""
    M, F = x.shape[0], W1.shape[0]
    dev = x.device
    if dx is None:
        dx = torch.empty_like(dres)
    f1 = torch.empty(M, F, device=dev, dtype=torch.bfloat16) if acts else None
    dpre = torch.empty(M, F, device=dev, dtype=torch.bfloat16) if acts else None
    call('rs_ffn_bwd_bf16', M, F, P(x), P(W1), P(b1), P(W2), P(mask), P(dff), P(dres), P(dx), P(f1), P(dpre),
         float(p), stream())
    return dx, f1, dpre


def ffn_bwd_ln_bf16(x, W1, b1, W2, mask, dff, dres, h1, gamma1, mean1, rstd1, dgamma1, dbeta1, p,
                    key, site, acts=True):
    """ffn_bwd_bf16 with norm1's backward fused: -> (dh1, dsa or None, f1 bf16, dPre1 bf16)
    (acts=False: f1 / dPre1 None, as in ffn_bwd_bf16)."""
    M, F = x.shape[0], W1.shape[0]
    dev = x.device
    dh1 = torch.empty_like(dres)
    dsa = torch.empty_like(dres) if p > 0 else None
    f1 = torch.empty(M, F, device=dev, dtype=torch.bfloat16) if acts else None
    dpre = torch.empty(M, F, device=dev, dtype=torch.bfloat16) if acts else None
    w = ws(_hip.lib().rs_ffn_bwd_ln_ws_bytes(M, F), dev)
    call('rs_ffn_bwd_ln_bf16', M, F, P(x), P(W1), P(b1), P(W2), P(mask), P(dff), P(dres), P(h1), P(gamma1),
         P(mean1), P(rstd1), P(dh1), P(dsa), P(dgamma1), P(dbeta1), P(f1), P(dpre), float(p), P(key), site,
         P(w), stream())
    return dh1, dsa, f1, dpre


def ffn_bwd_ln2_bf16(x, W1, b1, W2, mask, dy2, h2, gamma2, mean2, rstd2, dgamma2, dbeta2, h1, gamma1,
                     mean1, rstd1, dgamma1, dbeta1, p, key, site1, site2):
    """norm2's backward + the FFN backward + norm1's backward in one pass (weight gradients by
    ffn_wgrad_bf16 from the returned dff): -> (dh1, dsa or None, dff = drop2(dh2))."""
    M, F = x.shape[0], W1.shape[0]
    dff = torch.empty_like(dy2)
    dh1 = torch.empty_like(dy2)
    dsa = torch.empty_like(dy2) if p > 0 else None
    w = ws(_hip.lib().rs_ffn_bwd_ln2_ws_bytes(M, F), x.device)
    call('rs_ffn_bwd_ln2_bf16', M, F, P(x), P(W1), P(b1), P(W2), P(mask), P(dy2), P(h2), P(gamma2), P(mean2),
         P(rstd2), P(dff), P(dgamma2), P(dbeta2), P(h1), P(gamma1), P(mean1), P(rstd1), P(dh1), P(dsa),
         P(dgamma1), P(dbeta1), float(p), P(key), site1, site2, P(w), stream())
    return dh1, dsa, dff


def ffn_wgrad_bf16(x, W1, b1, W2, mask, dff, p, dW1, db1, dW2, db2):
    """dW1 += dPre1^T x, db1 += colsum(dPre1), dW2 += dff^T f1, db2 += colsum(dff), f1 / dPre1
    recomputed on chip (csrc/ffn.hip rs_ffn_wgrad_bf16)."""
    M, F = x.shape[0], W1.shape[0]
    w = ws(_hip.lib().rs_ffn_wgrad_ws_bytes(M, F), x.device)
    call('rs_ffn_wgrad_bf16', M, F, P(x), P(W1), P(b1), P(W2), P(mask), P(dff), float(p), P(dW1), P(db1),
         P(dW2), P(db2), P(w), stream())


def wgrad_bf16(dy, x, dW, *, db=None, beta=1.0):
    """dW[Mo,No] = beta*dW + dy[rows,Mo]^T x[rows,No] on bf16 MFMA; db += colsum(dy). dy / x may be
    fp32 or bf16 tensors."""
    rows, Mo = dy.shape
    No = x.shape[1]
    w = ws(_hip.lib().rs_wgrad_ws_bytes(Mo, No, rows), dy.device)
    call('rs_wgrad_bf16', rows, Mo, No, P(dy), dy.stride(0), int(dy.dtype == torch.bfloat16), P(x), x.stride(0),
         int(x.dtype == torch.bfloat16), float(beta), P(dW), dW.stride(0), P(db), P(w), stream())
    return dW


def colsum(X, out, *, scale=1.0, beta=1.0, M=None, N=None, ldx=None):
    """out[n] = beta*out[n] + scale*sum_m X[m, n]."""
    if M is None:
        M, N = X.shape
        ldx = X.stride(0)
    w = ws(_hip.lib().rs_colsum_ws_bytes(M, N), X.device)
    call('rs_colsum', P(X), M, N, ldx, float(scale), float(beta), P(out), P(w), stream())
    return out


def seq_mask(seq, pad_value=0):
    B, L = seq.shape[0], seq.shape[1]
    key_pad = torch.empty(B, L, dtype=torch.uint8, device=seq.device)
    last = torch.empty(B, dtype=torch.int64, device=seq.device)
    call('rs_seq_mask', P(seq), seq.stride(0), B, L, int(pad_value), P(key_pad), P(last), stream())
    return key_pad, last


def segments_array(segs):
    arr = (_hip.FeatureSeg * len(segs))(*segs)
    return arr


def gather_fwd(segs, rows, out, err_flag=None, lazy=None):
    """rs_gather_fwd; with `lazy` = (m_off, v_off, step, consts, b1, b2, eps, wd) the segments
    whose lazy_last is set read their rows through the lazy-Adam catch-up (rs_gather_fwd_lazy)."""
    arr = segments_array(segs)
    if lazy is not None and any(s.lazy_last for s in segs):
        call('rs_gather_fwd_lazy', arr, len(segs), rows, P(out), out.stride(0), P(err_flag), *lazy, stream())
    else:
        call('rs_gather_fwd', arr, len(segs), rows, P(out), out.stride(0), P(err_flag), stream())
    return out


_DETERMINISTIC = [None]


def sync_deterministic():
    """Mirror torch.are_deterministic_algorithms_enabled() into the library (rs_set_deterministic):
    deterministic table gradients (slot-image / ranged kernels) instead of the float-atomic
    scatter. RSYS_DETERMINISTIC=1 turns it on regardless."""
    on = bool(torch.are_deterministic_algorithms_enabled())
    if on != _DETERMINISTIC[0]:
        _hip.lib().rs_set_deterministic(int(on))
        _DETERMINISTIC[0] = on


def deterministic_enabled() -> bool:
    """Deterministic table gradients requested (torch.use_deterministic_algorithms or
    RSYS_DETERMINISTIC=1)."""
    return bool(torch.are_deterministic_algorithms_enabled()) or os.environ.get('RSYS_DETERMINISTIC', '0') == '1'


def gather_bwd(segs, rows, dout):
    sync_deterministic()
    arr = segments_array(segs)
    # hot mid-size tables (C2's 3,500-row history table) reduce per-chunk partials from ws
    w = ws(_hip.lib().rs_gather_ws_bytes(arr, len(segs), rows), dout.device)
    call('rs_gather_bwd', arr, len(segs), rows, P(dout), dout.stride(0), P(w), stream())


STREAM_BF16_MIN_ROWS = 32768  # gemm_stream.hip kSmallM: the bf16-storage GEMM instances are big-M only


def qkv_bf16_ok(L, d, H, M):
    """Store the packed qkv (and dqkv) as bf16: bf16 compute mode on the bf16 MFMA attention
    path (head_dim 16, L <= 256), where Q, K, V are only MFMA operands (RS_ATTN_QKV_BF16), for
    token counts M the bf16-storage streaming GEMMs cover (M >= 32768, a multiple of 16)."""
    return (precision.compute_dtype() == 'bf16' and d // H == 16 and L <= 256 and
            M >= STREAM_BF16_MIN_ROWS and M % 16 == 0 and
            not os.environ.get('RSYS_ATTN_VALU') and not os.environ.get('RSYS_QKV_FP32'))


def _attn_flags(qkv):
    return precision.gemm_flags() | (_hip.RS_ATTN_QKV_BF16 if qkv.dtype == torch.bfloat16 else 0)


def _zbits_words(B, L, d, H, p, flags):
    """uint16 words of rs_attn_fwd's saved dropout keep bits (include/rsys_hip.h): the bf16 MFMA
    path with L <= 64 and p > 0 (the dispatch condition of attention.hip), else 0."""
    if not (p > 0 and flags & _hip.RS_GEMM_BF16 and d // H == 16 and L <= 64 and B * H * L * L < 2 ** 32
            and not os.environ.get('RSYS_ATTN_VALU')):
        return 0
    return B * H * ((L + 15) // 16) * 64


def attn_fwd(qkv, key_pad, B, L, d, H, p=0.0, key=None, site=0):
    """-> out [B*L, d], lse [B*H*L]. Where the kernel saves its dropout keep bits for the backward
    (_zbits_words), they live in lse's storage past its B*H*L floats, so whoever keeps lse for
    attn_bwd keeps them too; an lse without that tail makes attn_bwd draw them again."""
    out = torch.empty(B * L, d, device=qkv.device, dtype=torch.float32)
    flags = _attn_flags(qkv)
    n, zw = B * H * L, _zbits_words(B, L, d, H, p, flags)
    if zw:
        buf = torch.empty(n + (zw + 1) // 2 + 4, device=qkv.device, dtype=torch.float32)
        lse, zb = buf[:n], _zbits_ptr(buf, n)
    else:
        lse, zb = torch.empty(n, device=qkv.device, dtype=torch.float32), None
    call('rs_attn_fwd', P(qkv), P(key_pad), P(out), P(lse), B, L, d, H,
         float((d // H) ** -0.5), float(p), P(key), site, flags, stream(), zb)
    return out, lse


def _zbits_ptr(lse, n):
    return (lse.data_ptr() + 4 * n + 15) // 16 * 16  # 16-byte aligned start past the lse floats


def attn_bwd(qkv, key_pad, out, dout, lse, B, L, d, H, p=0.0, key=None, site=0):
    """dqkv has qkv's storage dtype (bf16 with RS_ATTN_QKV_BF16)."""
    dqkv = torch.empty(B * L, 3 * d, device=qkv.device, dtype=qkv.dtype)
    flags = _attn_flags(qkv)
    n, zw = B * H * L, _zbits_words(B, L, d, H, p, flags)
    zb = None
    if zw and lse.storage_offset() == 0 and lse.numel() == n and \
            lse.untyped_storage().nbytes() == 4 * (n + (zw + 1) // 2 + 4):
        zb = _zbits_ptr(lse, n)  # attn_fwd's tail (its docstring; exactly its allocation's size)
    call('rs_attn_bwd', P(qkv), P(key_pad), P(out), P(dout), P(lse), P(dqkv), B, L, d, H,
         float((d // H) ** -0.5), float(p), P(key), site, flags, stream(), zb)
    return dqkv


def attn_rows_fwd(qkv, key_pad, last, B, L, d, H, p=0.0, key=None, site=0):
    """Attention of the selected query row last[b] of each sample -> out [B, d], lse [B*H]."""
    out = torch.empty(B, d, device=qkv.device, dtype=torch.float32)
    lse = torch.empty(B * H, device=qkv.device, dtype=torch.float32)
    call('rs_attn_rows_fwd', P(qkv), P(key_pad), P(last), P(out), P(lse), B, L, d, H,
         float((d // H) ** -0.5), float(p), P(key), site, _attn_flags(qkv), stream())
    return out, lse


def attn_rows_bwd(qkv, key_pad, last, dout, lse, B, L, d, H, p=0.0, key=None, site=0):
    """-> dqkv [B*L, 3d] (qkv's dtype), dQ zero off the selected rows."""
    dqkv = torch.empty(B * L, 3 * d, device=qkv.device, dtype=qkv.dtype)
    call('rs_attn_rows_bwd', P(qkv), P(key_pad), P(last), P(dout), P(lse), P(dqkv), B, L, d, H,
         float((d // H) ** -0.5), float(p), P(key), site, _attn_flags(qkv), stream())
    return dqkv


def linear_add_layernorm(x, W, bias, resid, gamma, beta, eps=1e-5, p=0.0, key=None, site=0):
    """h = dropout(x W^T + bias) + resid, y = LayerNorm(h): one fused kernel at the encoder
    width. Returns h (kept for the backward), y, mean, rstd."""
    M, K = x.shape
    N = W.shape[0]
    if tuple(resid.shape) != (M, N) or not resid.is_contiguous():
        raise RuntimeError('linear_add_layernorm: resid must be a contiguous [M, N] tensor')
    dev = x.device
    h = torch.empty(M, N, device=dev, dtype=torch.float32)
    y = torch.empty(M, N, device=dev, dtype=torch.float32)
    mean = torch.empty(M, device=dev, dtype=torch.float32)
    rstd = torch.empty(M, device=dev, dtype=torch.float32)
    call('rs_gemm_add_layernorm', M, N, K, P(x), x.stride(0), P(W), W.stride(0), P(bias), P(resid),
         P(h), P(y), P(gamma), P(beta), P(mean), P(rstd), float(eps), float(p), P(key), site,
         precision.gemm_flags(), stream())
    return h, y, mean, rstd


def linear_add_layernorm_rows(x, W, bias, table, rows, bag, gamma, beta, eps=1e-5, p=0.0, key=None, site=0):
    """linear_add_layernorm with the residual rows read in place: row m's residual is
    table[m * bag + rows[m]] (rs_gemm_add_layernorm_rows). None when the fused bf16 kernel does not
    take the shape (the caller gathers the rows instead)."""
    M, K = x.shape
    N = W.shape[0]
    if not (precision.gemm_flags() & _hip.RS_GEMM_BF16) or M % 16 or N != 64 or K not in (64, 256) or \
            x.stride(0) % 4 or W.stride(0) % 4 or rows.dtype != torch.int64 or not table.is_contiguous():
        return None
    dev = x.device
    h = torch.empty(M, N, device=dev, dtype=torch.float32)
    y = torch.empty(M, N, device=dev, dtype=torch.float32)
    mean = torch.empty(M, device=dev, dtype=torch.float32)
    rstd = torch.empty(M, device=dev, dtype=torch.float32)
    call('rs_gemm_add_layernorm_rows', M, N, K, P(x), x.stride(0), P(W), W.stride(0), P(bias), P(table), P(rows),
         int(bag), P(h), P(y), P(gamma), P(beta), P(mean), P(rstd), float(eps), float(p), P(key), site,
         precision.gemm_flags(), stream())
    return h, y, mean, rstd


def add_layernorm_fwd(a, b, gamma, beta, eps=1e-5, p=0.0, key=None, site=0):
    """h = dropout(a) + b (into a); returns y, mean, rstd."""
    M, N = a.shape
    y = torch.empty_like(a)
    mean = torch.empty(M, device=a.device, dtype=torch.float32)
    rstd = torch.empty(M, device=a.device, dtype=torch.float32)
    call('rs_add_layernorm_fwd', P(a), P(b), P(gamma), P(beta), P(y), P(mean), P(rstd), M, N,
         float(eps), float(p), P(key), site, stream())
    return y, mean, rstd


def layernorm_bwd(h, dy, gamma, mean, rstd, dgamma, dbeta, dh=None, da=None, p=0.0, key=None,
                  site=0):
    """dh = LN backward (in place over dy by default); da = dropout-backward(dh) if given."""
    M, N = h.shape
    if dh is None:
        dh = dy
    w = ws(_hip.lib().rs_layernorm_ws_bytes(M, N), h.device)
    call('rs_layernorm_bwd', P(h), P(dy), P(gamma), P(mean), P(rstd), P(dh), P(dgamma), P(dbeta),
         M, N, P(da), float(p), P(key), site, P(w), stream())
    return dh


def rng_next(state):
    key = torch.empty(2, dtype=torch.int64, device=state.device)
    call('rs_rng_next', P(state), P(key), stream())
    return key


def dropout_fwd(x, p, key, site, aux=None, aux_mod=0):
    """x = dropout(x (+ aux[row % aux_mod])) in place; x is [M, N] contiguous."""
    N = x.shape[-1]
    call('rs_dropout_fwd', P(x), x.numel(), N, P(aux), aux.stride(0) if aux is not None else 0,
         aux_mod, float(p), P(key), site, stream())
    return x


def seq_input_dropout_bwd(dx, pos_grad, rows, N, p, key, site_a, site_b):
    """dx [rows, N] <- dx * mask_b * mask_a; pos_grad[:N] += colsum(dx * mask_b) (one pass)."""
    w = ws(_hip.lib().rs_seq_input_dropout_bwd_ws_bytes(rows, N), dx.device)
    call('rs_seq_input_dropout_bwd', P(dx), rows, N, float(p), P(key), site_a, site_b, P(pos_grad), P(w),
         stream())
    return dx


def dropout_bwd(dx, p, key, site):
    call('rs_dropout_bwd', P(dx), dx.numel(), float(p), P(key), site, stream())
    return dx


def batchnorm_fwd(x, bn, G, relu, training, momentum=None, eps=None, drop_p=0.0, drop_key=None,
                  drop_site=0):
    """x [G*Bg, C]; bn: nn.BatchNorm1d-like (weight, bias, running_*, num_batches_tracked).
    drop_p > 0: the following nn.Dropout fused into the output (relu and training only)."""
    M, Cc = x.shape
    Bg = M // G
    y = torch.empty_like(x)
    mean = torch.empty(G * Cc, device=x.device, dtype=torch.float32)
    rstd = torch.empty(G * Cc, device=x.device, dtype=torch.float32)
    mom = bn.momentum if momentum is None else momentum
    if mom is None:
        raise NotImplementedError('BatchNorm1d(momentum=None) (cumulative average) is not supported')
    track = bn.track_running_stats and bn.running_mean is not None
    batch_stats = training or not track          # nn.BatchNorm1d: eval uses running stats
    update = training and track
    run = update or not batch_stats
    w = ws(_hip.lib().rs_batchnorm_ws_bytes(G, Bg, Cc), x.device)
    call('rs_batchnorm_fwd', P(x), P(y), P(bn.weight), P(bn.bias),
         P(bn.running_mean) if run else None, P(bn.running_var) if run else None,
         P(bn.num_batches_tracked) if update else None,
         P(mean), P(rstd), G, Bg, Cc, float(mom), float(bn.eps if eps is None else eps), int(relu),
         int(batch_stats), float(drop_p), P(drop_key), drop_site, P(w), stream())
    return y, mean, rstd


def batchnorm_bwd(x, y, dy, weight, mean, rstd, dw, db, G, relu, dx=None, drop_p=0.0):
    M, Cc = x.shape
    Bg = M // G
    if dx is None:
        dx = torch.empty_like(x)
    w = ws(_hip.lib().rs_batchnorm_ws_bytes(G, Bg, Cc), x.device)
    # the fused dropout's scale, in the forward's fp32 arithmetic (rng.h make_key)
    scale = float(np.float32(1.0) / (np.float32(1.0) - np.float32(drop_p))) if drop_p > 0 else 1.0
    call('rs_batchnorm_bwd', P(x), P(y), P(dy), P(weight), P(mean), P(rstd), P(dx), P(dw), P(db),
         G, Bg, Cc, int(relu), scale, P(w), stream())
    return dx


def l2norm_fwd(x, eps=1e-12):
    M, N = x.shape
    y = torch.empty_like(x)
    norm = torch.empty(M, device=x.device, dtype=torch.float32)
    call('rs_l2norm_fwd', P(x), P(y), P(norm), M, N, float(eps), stream())
    return y, norm


def l2norm_bwd(y, norm, dy, eps=1e-12):
    M, N = y.shape
    dx = torch.empty_like(y)
    call('rs_l2norm_bwd', P(y), P(norm), P(dy), P(dx), M, N, float(eps), stream())
    return dx
