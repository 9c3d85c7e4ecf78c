"""ctypes binding of librsys_hip.so (include/rsys_hip.h).

The product path has no CPU fallback: if the library is missing or no gfx950 device is present,
every op raises. `lib()` loads the in-tree build (recommendsystemproject_amd/_lib/librsys_hip.so,
produced by __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('RSYS_LIB_PATH') or os.path.join(_HERE, '_lib', 'librsys_hip.so')

RS_EPI_BIAS, RS_EPI_RELU, RS_EPI_AUX_ADD, RS_EPI_AUX_MASK = 1, 2, 4, 8
RS_GEMM_BF16 = 256
RS_GEMM_A_BF16, RS_GEMM_C_BF16 = 512, 1024
RS_ATTN_QKV_BF16 = 2048
RS_EPI_DROP_A, RS_EPI_DROP_B = 16, 32
RS_SEG_SPARSE, RS_SEG_POOL, RS_SEG_DENSE, RS_SEG_LASTVALID, RS_SEG_COPY = 0, 1, 2, 3, 4
RS_POOL = {'mean': 0, 'sum': 1, 'max': 2}
MAX_SEGMENTS = 20

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_int64, C.c_float


class FeatureSeg(C.Structure):
    """Mirror of rs_feature_seg_t."""
    _fields_ = [('kind', i32), ('dim', i32), ('out_col', i32), ('pool_mode', i32), ('bag', i32),
                ('pad_idx', i32), ('vocab', i64), ('idx_stride', i64), ('idx', vp), ('table', vp),
                ('bias', vp), ('x', vp), ('grad', vp), ('grad_bias', vp), ('touch_count', vp),
                ('lazy_last', vp), ('hot_keys', vp), ('hot_n', i64)]


class SortedCall(C.Structure):
    """Mirror of rs_sorted_call_t."""
    _fields_ = [('keys', vp), ('n', i64), ('D', i32), ('call', i32), ('p', vp), ('g', vp), ('m', vp), ('v', vp),
                ('last', vp), ('owner', vp)]


class SegsumCall(C.Structure):
    """Mirror of rs_segsum_call_t."""
    _fields_ = [('keys', vp), ('vals', vp), ('n', i64), ('bag', i32), ('mode', i32), ('pad', i64), ('dout', vp),
                ('ldo', i64), ('grad', vp), ('accumulate', i32), ('ws', vp)]


# name -> (restype, argtypes). Every symbol declared in include/rsys_hip.h.
SIGNATURES = {
    'rs_version': (i32, []),
    'rs_last_error': (C.c_char_p, []),
    'rs_device_check': (i32, []),
    'rs_gemm_auto_split': (i32, [i32, i32, i32]),
    'rs_gemm_ws_bytes': (i64, [i32, i32, i32, i32]),
    'rs_gemm_f32': (i32, [i32, i32, i32, i32, i32, f32, vp, i32, vp, i32, f32, vp, i32, i32, vp, vp,
                          i32, i32, f32, vp, i32, i32, vp, i32, vp, vp]),
    'rs_gemm_add_layernorm': (i32, [i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp,
                                    f32, f32, vp, i32, i32, vp]),
    'rs_gemm_add_layernorm_rows': (i32, [i32, i32, i32, vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, vp, vp,
                                         vp, vp, f32, f32, vp, i32, i32, vp]),
    'rs_ffn_mask_words': (i64, [i32, i32]),
    'rs_ffn_fwd_bf16': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, f32, vp,
                              i32, i32, vp]),
    'rs_ffn_bwd_bf16': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, vp]),
    'rs_ffn_bwd_ln_ws_bytes': (i64, [i32, i32]),
    'rs_ffn_bwd_ln_bf16': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                 vp, vp, f32, vp, i32, vp, vp]),
    'rs_ffn_bwd_ln2_ws_bytes': (i64, [i32, i32]),
    'rs_ffn_bwd_ln2_bf16': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                  vp, vp, vp, vp, vp, vp, f32, vp, i32, i32, vp, vp]),
    'rs_wgrad_ws_bytes': (i64, [i32, i32, i32]),
    'rs_ffn_wgrad_ws_bytes': (i64, [i32, i32]),
    'rs_ffn_wgrad_bf16': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp]),
    'rs_wgrad_bf16': (i32, [i32, i32, i32, vp, i32, i32, vp, i32, i32, f32, vp, i32, vp, vp, vp]),
    'rs_colsum_ws_bytes': (i64, [i32, i32]),
    'rs_colsum': (i32, [vp, i32, i32, i32, f32, f32, vp, vp, vp]),
    'rs_gather_fwd': (i32, [vp, i32, i32, vp, i32, vp, vp]),
    'rs_sorted_adam_batch': (i32, [vp, i32, vp, vp, f32, f32, f32, f32, f32, vp, vp]),
    'rs_sorted_catchup_batch': (i32, [vp, i32, vp, vp, f32, f32, f32, f32, vp]),
    'rs_sorted_sqnorm_batch': (i32, [vp, i32, f32, vp, vp]),
    'rs_copy_many': (i32, [i32, vp, vp, vp, vp]),
    'rs_nan_check_many': (i32, [i32, vp, vp, vp, vp, vp]),
    'rs_gather_fwd_lazy': (i32, [vp, i32, i32, vp, i32, vp, i64, i64, vp, vp, f32, f32, f32, f32, vp]),
    'rs_gather_ws_bytes': (i64, [vp, i32, i32]),
    'rs_gather_bwd': (i32, [vp, i32, i32, vp, i32, vp, vp]),
    'rs_set_deterministic': (i32, [i32]),
    'rs_seq_mask': (i32, [vp, i64, i32, i32, i64, vp, vp, vp]),
    'rs_attn_fwd': (i32, [vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, i32, i32, vp, vp]),
    'rs_attn_bwd': (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, i32, i32, vp, vp]),
    'rs_attn_rows_fwd': (i32, [vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, i32, i32, vp]),
    'rs_attn_rows_bwd': (i32, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, vp, i32, i32, vp]),
    'rs_add_layernorm_fwd': (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, vp, i32, vp]),
    'rs_layernorm_ws_bytes': (i64, [i32, i32]),
    'rs_layernorm_bwd': (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, f32, vp, i32, vp, vp]),
    'rs_batchnorm_ws_bytes': (i64, [i32, i32, i32]),
    'rs_batchnorm_fwd': (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, i32, i32,
                               f32, vp, i32, vp, vp]),
    'rs_tower_part_floats': (i64, [i32, i32, i32, i32]),
    'rs_tower_debug_buffer': (i32, [vp]),
    'rs_tower_wgrad_split': (i32, [i32, i32, i32]),
    'rs_tower_wgrad_ws_floats': (i64, [i32, i32, i32]),
    'rs_tower_wgrad_sync_ints': (i32, [i32, i32]),
    'rs_tower_wgrad': (i32, [i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp]),
    'rs_tower_sync_ints': (i32, [i32, i32]),
    'rs_tower_stats': (i32, [vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, f32, f32, vp, vp, vp]),
    'rs_tower_fwd': (i32, [vp, i32, i32, i32, vp, vp, vp, vp, i32, f32, vp, i32, vp, vp, vp, i32, vp, vp,
                           vp, vp, vp, vp, vp, vp, vp, f32, f32, vp, vp, f32, i32, vp]),
    'rs_tower_bwd': (i32, [vp, i32, i32, i32, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp,
                           vp, vp, vp, i32, f32, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp]),
    'rs_batchnorm_bwd': (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp, vp]),
    'rs_l2norm_fwd': (i32, [vp, vp, vp, i32, i32, f32, vp]),
    'rs_l2norm_bwd': (i32, [vp, vp, vp, vp, i32, i32, f32, vp]),
    'rs_inbatch_ce_fused_ws_bytes': (i64, [i32, i32]),
    'rs_inbatch_ce_fused_fwd': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp]),
    'rs_inbatch_ce_fused_bwd': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp, vp,
                                      vp]),
    'rs_inbatch_ce_fused_fwd_uib': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp,
                                          vp]),
    'rs_inbatch_ce_fused_bwd_uib': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp,
                                          vp, vp, vp]),
    'rs_inbatch_ce_s_ld': (i64, [i32]),
    'rs_inbatch_ce_fused_f32_fwd': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp,
                                          vp]),
    'rs_inbatch_ce_fused_f32_bwd': (i32, [vp, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp,
                                          vp, vp, vp]),
    'rs_inbatch_ce_fwd': (i32, [vp, i32, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp]),
    'rs_inbatch_ce_bwd': (i32, [vp, i32, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp]),
    'rs_inbatch_logits': (i32, [vp, i32, vp, vp, i64, i64, vp, i64, i32, i32, i32, f32, vp, i64, vp]),
    'rs_hardneg_bwd': (i32, [vp, vp, i64, i64, vp, vp, vp, i32, i32, i32, vp]),
    'rs_mask_history': (i32, [vp, i64, i32, i64, i64, vp, i64, vp, vp, i64, vp]),
    'rs_topk_rows': (i32, [vp, i64, i32, i32, i32, vp, i64, i32, vp, vp, i64, vp]),
    'rs_recall_hits': (i32, [vp, i32, i32, vp, vp, i64, vp, i32, vp, vp]),
    'rs_collate_ragged': (i32, [vp, i32, i32, vp, i64, vp, i32, i32, vp, vp, vp]),
    'rs_catalog_gather': (i32, [vp, i32, i32, i64, i32, i64, vp, i32, i32, i64, vp, i64, vp, vp]),
    'rs_sqnorm_ws_bytes': (i64, [i64]),
    'rs_grad_sqnorm': (i32, [vp, i64, f32, vp, vp]),
    'rs_sqnorm_parts': (i32, [i64]),
    'rs_clip_coef': (i32, [vp, i32, f32, vp, vp, vp]),
    'rs_clip_coef_step': (i32, [vp, i32, f32, vp, vp, vp, vp]),
    'rs_grad_sqnorm_clip_step': (i32, [vp, i64, f32, vp, vp, f32, vp, vp, vp, vp]),
    'rs_clip_coef_prepare': (i32, [vp, i32, f32, vp, vp, vp, vp, i32, f32, f32, f32, vp]),
    'rs_sorted_sqnorm_batch_dense': (i32, [vp, i32, f32, vp, vp, i64, vp, vp]),
    'rs_sorted_adam_batch_dense': (i32, [vp, i32, vp, vp, f32, f32, f32, f32, f32, vp, vp, vp, vp, vp, i64, f32,
                                         vp]),
    'rs_scale_inplace': (i32, [vp, i64, f32, vp, vp]),
    'rs_adam_step': (i32, [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, i32, vp, f32, vp, i32, vp]),
    'rs_counter_add': (i32, [vp, i64, vp]),
    'rs_prof_marker': (i32, [i32, vp]),
    'rs_peak_copy': (i32, [vp, vp, i64, vp]),
    'rs_peak_mfma': (i32, [vp, i32, i32, vp]),
    'rs_peak_mfma_flops': (i64, [i32, i32]),
    'rs_sum': (i32, [vp, i32, f32, vp, vp]),
    'rs_reduce_defer': (i32, [i32]),
    'rs_reduce_flush': (i32, [vp]),
    'rs_nan_check': (i32, [vp, i64, vp, i32, vp]),
    'rs_rng_next': (i32, [vp, vp, vp]),
    'rs_adam_prepare': (i32, [vp, vp, i32, f32, f32, f32, vp]),
    'rs_sparse_flush': (i32, [vp, vp, vp, vp, i64, i32, vp, vp, f32, f32, f32, f32, vp]),
    'rs_lookup_sort_ws_bytes': (i64, [i64, i64]),
    'rs_lookup_sort': (i32, [vp, i32, i32, i32, i64, i64, vp, vp, vp, vp]),
    'rs_lookup_catchup': (i32, [vp, i32, i32, i32, i64, i64, i32, vp, vp, vp, vp, vp, vp, f32, f32, f32, f32,
                                vp]),
    'rs_sorted_catchup': (i32, [vp, i64, i32, vp, vp, vp, vp, vp, vp, f32, f32, f32, f32, vp]),
    'rs_sorted_adam': (i32, [vp, i64, i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, f32, f32, f32, f32, f32,
                             vp, vp]),
    'rs_sorted_sqnorm_parts': (i32, []),
    'rs_sorted_sqnorm': (i32, [vp, i64, i32, vp, vp, i32, f32, vp, vp]),
    'rs_sorted_owner': (i32, [vp, i64, vp, i32, vp]),
    'rs_sorted_zero_grad': (i32, [vp, i64, i32, vp, vp]),
    'rs_segsum_ws_bytes': (i64, [i64, i32]),
    'rs_segsum': (i32, [vp, vp, i64, i32, i32, i64, vp, i64, i32, vp, i32, vp, vp]),
    'rs_segsum_batch': (i32, [vp, i32, i32, vp]),
    'rs_shard_map_ids': (i32, [vp, i64, i64, i32, i32, vp, vp, vp]),
    'rs_shard_bucket_ws_bytes': (i64, [i64, i32]),
    'rs_shard_bucket': (i32, [vp, vp, i64, i32, i32, i64, vp, vp, vp, vp, vp, vp, vp]),
    'rs_shard_recv': (i32, [vp, vp, i32, i32, i64, vp, vp, vp, vp]),
    'rs_pack_ids': (i32, [vp, i32, i64, i32, i64, vp, vp]),
    'rs_pack_rows': (i32, [vp, i64, i64, i32, vp, vp]),
    'rs_pool_max_grad': (i32, [vp, vp, i32, i64, i32, i64, i64, i32, i64, vp, i64, vp, vp]),
    'rs_dropout_fwd': (i32, [vp, i64, i32, vp, i32, i32, f32, vp, i32, vp]),
    'rs_seq_input_dropout_bwd_ws_bytes': (i64, [i32, i32]),
    'rs_seq_input_dropout_bwd': (i32, [vp, i32, i32, f32, vp, i32, i32, vp, vp, vp]),
    'rs_dropout_bwd': (i32, [vp, i64, f32, vp, i32, vp]),
}

_LIB = None


class HipError(RuntimeError):
    pass


def lib():
    """Load librsys_hip.so once (no GPU needed to load; kernels need a gfx950 device)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(f'{LIB_PATH} missing: run __graft_entry__.build() (hipcc, gfx950)')
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def call(name: str, *args):
    """Invoke an rs_* entry point; raise HipError with rs_last_error() on failure."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.rs_last_error().decode(errors='replace')
        raise HipError(f'{name} failed (rc={rc}): {msg}')
    return rc


_DEVICE_OK = {}


def require_device(t) -> None:
    """Fail loudly unless `t` lives on a gfx950 HIP device (no CPU fallback)."""
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise HipError('recommendsystemproject_amd runs on MI355X only: move the model and the batch '
                       'to a cuda (HIP) device; there is no CPU fallback')
    dev = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if dev not in _DEVICE_OK:
        with torch.cuda.device(dev):
            call('rs_device_check')
        _DEVICE_OK[dev] = True
