"""Per-entry-point kernel timing with HIP events on the launch stream, plus the algorithmic
work (FLOPs / HBM bytes) of every rs_* call, for the bench's roofline line.

Usage:
    with KernelTimer() as kt:
        step()
    kt.summary()  -> {name: {'ms': total, 'launches': n, 'flops': F, 'bytes': B}}
"""
from __future__ import annotations

import torch

from . import _hip


def _gemm_work(a):
    M, N, K = a[2], a[3], a[4]
    beta, epi = a[10], a[13]
    ea = 2.0 if epi & _hip.RS_GEMM_A_BF16 else 4.0  # bf16 storage of A / C
    ec = 2.0 if epi & _hip.RS_GEMM_C_BF16 else 4.0
    return 2.0 * M * N * K, ea * M * K + 4.0 * K * N + ec * M * N + (4.0 * M * N if beta != 0 else 0.0)


def _attn_fwd_work(a):
    B, L, d, H = a[4], a[5], a[6], a[7]
    hd = d // H
    eq = 2.0 if a[12] & _hip.RS_ATTN_QKV_BF16 else 4.0
    # QK^T twice (max pass + sum pass) and PV; qkv read, out + lse written
    return 2.0 * B * H * L * L * hd * 3, eq * B * L * 3 * d + 4.0 * (B * L * d + B * H * L)


def _attn_bwd_work(a):
    B, L, d, H = a[6], a[7], a[8], a[9]
    hd = d // H
    eq = 2.0 if a[14] & _hip.RS_ATTN_QKV_BF16 else 4.0
    # s, dp, dq, dk, dv; qkv read, dqkv written, dout and lse read; the bf16 path forms
    # D = rowsum(P dP) from its own tiles, the others read out (D = dO . O)
    bf = a[14] & _hip.RS_GEMM_BF16 and hd == 16 and L <= 64
    return 2.0 * B * H * L * L * hd * 5, eq * B * L * 3 * d * 2 + 4.0 * ((1 if bf else 2) * B * L * d + B * H * L)


def _gather_work(a, bwd=False):
    segs, nseg, rows = a[0], a[1], a[2]
    byts = 0.0
    for i in range(nseg):
        s = segs[i]
        if s.kind in (_hip.RS_SEG_SPARSE, _hip.RS_SEG_POOL):
            bag = s.bag if s.kind == _hip.RS_SEG_POOL else 1
            # table rows read (fwd) / scattered (bwd) + int64 ids; a read-through
            # lazy segment (rs_gather_fwd_lazy) also reads the row's two moment rows and `last`
            rt = not bwd and len(a) > 7 and bool(s.lazy_last)
            byts += rows * bag * (s.dim * 4 * (3 if rt else 1) + 8 + (4 if rt else 0))
        elif s.kind == _hip.RS_SEG_DENSE:
            byts += rows * 4
        else:
            byts += rows * s.dim * 4
        byts += rows * s.dim * 4  # concat slice written (fwd) / read (bwd)
    return 0.0, byts


def _ln_fwd_work(a):
    M, N = a[7], a[8]
    return 8.0 * M * N, 4.0 * M * N * 4


def _ln_bwd_work(a):
    M, N = a[8], a[9]
    return 12.0 * M * N, 4.0 * M * N * 3


def _bn_work(a, bwd=False):
    G, Bg, C = (a[9], a[10], a[11])
    n = G * Bg * C
    return 6.0 * n, 4.0 * n * (4 if bwd else 3)


def _tower_fwd_work(a):
    """rs_tower_fwd: A read (BN applied on the fly), W read, z / out written, h written when asked."""
    M, K, N = a[1] * a[2], a[3], a[15]
    byts = 4.0 * (M * K + N * K + M * N) + (4.0 * M * K if a[12] else 0.0) + (4.0 * M if a[28] else 0.0)
    return 2.0 * M * N * K, byts


def _tower_bwd_work(a):
    """rs_tower_bwd: the incoming gradient and the prologue's second operand (z or y) read, dz
    written; N > 0: W read, the lower BatchNorm's z read and g written."""
    M, K, N = a[1] * a[2], a[3], a[15]
    byts = 4.0 * M * K * 3 + (4.0 * (K * N + 2 * M * N) if N else 0.0)
    return 2.0 * M * N * K, byts


def _tower_wgrad_work(a):
    import ctypes as C
    n, M = a[0], a[1]
    Ns = C.cast(a[2], C.POINTER(C.c_int))
    Ks = C.cast(a[3], C.POINTER(C.c_int))
    fl = by = 0.0
    for i in range(n):
        N, K = Ns[i], Ks[i]
        fl += 2.0 * M * N * K
        by += 4.0 * M * (N + K) + 8.0 * N * K
    return fl, by


def _segsum_batch_work(a):
    import ctypes as C
    from . import _hip
    arr, D = C.cast(a[0], C.POINTER(_hip.SegsumCall)), a[2]
    return 0.0, sum(arr[i].n * D * 4.0 + arr[i].n / arr[i].bag * D * 4.0 + arr[i].n * 4.0 for i in range(a[1]))


def _adam_work(a):
    n = a[4]
    return 12.0 * n, 28.0 * n


def _gemm_ln_work(a):
    M, N, K = a[0], a[1], a[2]
    # A, W read; resid read; h, y written; mean / rstd
    return 2.0 * M * N * K, 4.0 * (M * K + N * K + 3 * M * N + 2 * M)


def _ffn_fwd_work(a):
    M, F = a[0], a[1]
    # x read (GEMM operand + residual: once from HBM), h, y written, mask bits, mean / rstd
    return 4.0 * M * F * 64, 4.0 * (3 * M * 64 + 2 * M) + M * F / 8.0


def _ffn_bwd_work(a, acts=None):
    M, F = a[0], a[1]
    if acts is None:
        acts = a[10] is not None
    # dff, dres read, dx written (fp32); mask bits read; with the activations (acts): x read,
    # linear1 recomputed, f1 and dPre1 written (bf16)
    if acts:
        return 6.0 * M * F * 64, 4.0 * 4 * M * 64 + 2.0 * 2 * M * F + M * F / 8.0
    return 4.0 * M * F * 64, 4.0 * 3 * M * 64 + M * F / 8.0


def _wgrad_work(a):
    rows, Mo, No = a[0], a[1], a[2]
    return 2.0 * rows * Mo * No, rows * (Mo * (2 if a[5] else 4) + No * (2 if a[8] else 4))


def _ce_work(a, bwd=False):
    B = a[8]
    return 0.0, 4.0 * B * B * 2  # fwd: two passes over S; bwd: S read + dS written


def _ce_fused_work(a, bwd=False):
    B, D = a[7], a[9]
    # forward: S = U I^T on the MFMA (one pass, never stored); backward: S recomputed in the dU
    # and the dI halves, then dU = dS I and dI = dS^T U. Bytes: U, I read (+ partial gradients
    # written and reduced in the backward: 2 directions x splits x B x D fp32, not counted).
    return (8.0 if bwd else 2.0) * B * B * D, 4.0 * 2 * B * D * (2 if bwd else 1)


def _ce_fused_f32_work(a, bwd=False):
    B, D = a[7], a[9]
    # fp32: the forward computes S once and stores it (B x B fp32 written); the backward reads it
    # back in both halves (2 x B x B fp32) and runs only dU = dS I and dI = dS^T U
    fl, by = _ce_fused_work(a, False)
    if bwd:
        return 4.0 * B * B * D, 2 * by + 8.0 * B * B
    return fl, by + 4.0 * B * B


def _ffn_bwd_ln_work(a):
    M, F = a[0], a[1]
    # the FFN backward's operands plus norm1's: h1 read, dh1 (+ dsa) written instead of dx1
    fl, by = _ffn_bwd_work(a, acts=a[17] is not None)
    return fl + 12.0 * M * 64, by + 4.0 * M * 64 * (2 if a[19] > 0 else 1) + 8.0 * M


def _ffn_bwd_ln2_work(a):
    M, F = a[0], a[1]
    # dy2, h2, h1 read, dff, dh1 (+ dsa) written (fp32); mask bits; both rows' mean / rstd
    return (4.0 * M * F * 64 + 24.0 * M * 64,
            4.0 * M * 64 * (5 + (1 if a[23] > 0 else 0)) + 16.0 * M + M * F / 8.0)


WORK = {
    'rs_ffn_bwd_ln_bf16': _ffn_bwd_ln_work,
    'rs_ffn_bwd_ln2_bf16': _ffn_bwd_ln2_work,
    'rs_inbatch_ce_fused_fwd': _ce_fused_work,
    'rs_inbatch_ce_fused_bwd': lambda a: _ce_fused_work(a, True),
    'rs_inbatch_ce_fused_fwd_uib': _ce_fused_work,
    'rs_inbatch_ce_fused_bwd_uib': lambda a: _ce_fused_work(a, True),
    'rs_inbatch_ce_fused_f32_fwd': _ce_fused_f32_work,
    'rs_inbatch_ce_fused_f32_bwd': lambda a: _ce_fused_f32_work(a, True),
    'rs_gemm_add_layernorm': _gemm_ln_work,
    'rs_ffn_fwd_bf16': _ffn_fwd_work,
    'rs_ffn_bwd_bf16': _ffn_bwd_work,
    'rs_wgrad_bf16': _wgrad_work,
    'rs_inbatch_ce_fwd': _ce_work,
    'rs_inbatch_ce_bwd': lambda a: _ce_work(a, True),
    'rs_gemm_f32': _gemm_work,
    'rs_attn_fwd': _attn_fwd_work,
    'rs_attn_bwd': _attn_bwd_work,
    'rs_gather_fwd': _gather_work,
    'rs_gather_fwd_lazy': _gather_work,
    'rs_gather_bwd': lambda a: _gather_work(a, True),
    'rs_add_layernorm_fwd': _ln_fwd_work,
    'rs_layernorm_bwd': _ln_bwd_work,
    'rs_batchnorm_fwd': _bn_work,
    'rs_batchnorm_bwd': lambda a: _bn_work(a, True),
    'rs_adam_step': _adam_work,
    'rs_tower_stats': lambda a: (3.0 * a[1] * a[2] * a[3], 4.0 * a[1] * a[2] * a[3]),
    'rs_tower_fwd': _tower_fwd_work,
    'rs_tower_bwd': _tower_bwd_work,
    'rs_tower_wgrad': _tower_wgrad_work,
    # large tables (csrc/lookup.hip): the sort reads the ids and writes keys + vals; the table
    # gradient is priced by SURVEY §8d's gather formula (lookups x D x 4 + dout rows x D x 4 +
    # ids) like the scatter it replaces; the per-row catch-up / Adam / sqnorm work depends on the
    # device-side distinct-row count and is timed only
    'rs_lookup_sort': lambda a: (0.0, a[2] * a[3] * (a[1] + 8.0)),
    'rs_segsum_batch': _segsum_batch_work,
    'rs_segsum': lambda a: (0.0, a[2] * a[8] * 4.0 + a[2] / a[3] * a[8] * 4.0 + a[2] * 4.0),
}


# Exponentials per call (the VALU-bound part of the softmax kernels): attention one v_exp per
# (query, key) pair in each direction (csrc/attention.hip: the backward recomputes P), the fused
# in-batch CE one per logit in the forward and one per logit in each backward half.
EXPS = {
    'rs_attn_fwd': lambda a: float(a[4] * a[7] * a[5] * a[5]),
    'rs_attn_bwd': lambda a: float(a[6] * a[9] * a[7] * a[7]),
    'rs_inbatch_ce_fused_fwd': lambda a: float(a[7]) * (a[7] + a[8]),
    'rs_inbatch_ce_fused_bwd': lambda a: 2.0 * a[7] * (a[7] + a[8]),
    'rs_inbatch_ce_fused_fwd_uib': lambda a: float(a[7]) * (a[7] + a[8]),
    'rs_inbatch_ce_fused_bwd_uib': lambda a: 2.0 * a[7] * (a[7] + a[8]),
    'rs_inbatch_ce_fused_f32_fwd': lambda a: float(a[7]) * (a[7] + a[8]),
    'rs_inbatch_ce_fused_f32_bwd': lambda a: 2.0 * a[7] * (a[7] + a[8]),
}


TOKEN_ROWS = 32768  # rs_gemm_f32 calls streaming >= this many rows: the encoder's token GEMMs


def entry_key(name, args):
    """Timing / PMC key of one rs_* call. rs_gemm_f32 is split into its two regimes, which are
    different kernels: the encoder's token-level streaming GEMMs (rows = B*L, HBM-bound) and the
    batch-level tower / loss GEMMs (rows = B, latency-bound small grids)."""
    if name == 'rs_gemm_f32':
        rows = args[4] if args[0] else args[2]  # (transA, transB, M, N, K, ...): rows streamed
        return 'rs_gemm_f32:tokens' if rows >= TOKEN_ROWS else 'rs_gemm_f32:batch'
    return name


class _CallPatch:
    """Swap `call` in _hip and in the modules that imported it by name."""

    def _install(self, fn):
        self._orig = _hip.call
        _hip.call = fn
        from . import ops, functions, optim
        self._patched = []
        for mod in (ops, functions, optim):
            if getattr(mod, 'call', None) is self._orig:
                self._patched.append(mod)
                mod.call = fn

    def __exit__(self, *exc):
        _hip.call = self._orig
        for mod in self._patched:
            mod.call = self._orig
        return False


class PmcBracket(_CallPatch):
    """Brackets every call of one entry point with rs_prof_marker dispatches, so that a
    rocprofv3 --pmc pass can sum the counters of exactly the kernels that entry point launched
    (tools/pmc_traffic.py). Records the algorithmic bytes/flops of the bracketed calls."""

    def __init__(self, target):
        self.target = target
        self.launches = 0
        self.flops = 0.0
        self.bytes = 0.0

    def __enter__(self):
        orig = _hip.call

        def bracketed(name, *args):
            if entry_key(name, args) != self.target:
                return orig(name, *args)
            st = torch.cuda.current_stream().cuda_stream
            orig('rs_prof_marker', 1, st)
            rc = orig(name, *args)
            orig('rs_prof_marker', 2, st)
            fl, by = WORK[name](args) if name in WORK else (0.0, 0.0)
            self.launches += 1
            self.flops += fl
            self.bytes += by
            return rc

        self._install(bracketed)
        return self


class KernelTimer(_CallPatch):
    """Wraps _hip.call: an event pair on the current (launch) stream around every rs_* call."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        orig = _hip.call

        def timed(name, *args):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(torch.cuda.current_stream())
            rc = orig(name, *args)
            e.record(torch.cuda.current_stream())
            fl, by = WORK[name](args) if name in WORK else (0.0, 0.0)
            ex = EXPS[name](args) if name in EXPS else 0.0
            shape = tuple(args[:5]) if name == 'rs_gemm_f32' else None
            self.records.append((entry_key(name, args), s, e, fl, by, shape, ex))
            return rc

        self._install(timed)
        return self

    def gemm_shapes(self):
        """{(transA, transB, M, N, K): [ms, launches, flops]} for rs_gemm_f32."""
        torch.cuda.synchronize()
        out = {}
        for name, s, e, fl, by, shape, _ in self.records:
            if shape is None:
                continue
            d = out.setdefault(shape, [0.0, 0, 0.0])
            d[0] += s.elapsed_time(e)
            d[1] += 1
            d[2] += fl
        return out

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, s, e, fl, by, _, ex in self.records:
            d = out.setdefault(name, {'ms': 0.0, 'launches': 0, 'flops': 0.0, 'bytes': 0.0, 'exps': 0.0})
            d['ms'] += s.elapsed_time(e)
            d['launches'] += 1
            d['flops'] += fl
            d['bytes'] += by
            d['exps'] += ex
        return out
