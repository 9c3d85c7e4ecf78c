"""Compute-dtype switch for the encoder's GEMMs.

fp32 (default): f32-input MFMA, exact f32 products -- the parity-tested path.
bf16: the streaming GEMMs (encoder projections, FFN, their input gradients, the fused
GEMM + LayerNorm) round their operands to bf16 and accumulate in fp32 on the bf16 MFMA
(16x the f32 rate); master weights, optimizer, norms, softmax, embeddings and every other
kernel stay fp32. SURVEY.md §8d quotes C2 this way ("bf16 compute with fp32 master weights;
parity is run in fp32").

Set with set_compute_dtype('bf16') or RSYS_COMPUTE_DTYPE=bf16.
"""
from __future__ import annotations

import os

from . import _hip

_state = {'dtype': os.environ.get('RSYS_COMPUTE_DTYPE', 'fp32').lower()}


def set_compute_dtype(dtype: str) -> None:
    dtype = str(dtype).lower().replace('bfloat16', 'bf16').replace('float32', 'fp32')
    if dtype not in ('fp32', 'bf16'):
        raise ValueError(f"compute dtype must be 'fp32' or 'bf16', got {dtype!r}")
    _state['dtype'] = dtype


def compute_dtype() -> str:
    return _state['dtype']


def gemm_flags() -> int:
    return _hip.RS_GEMM_BF16 if _state['dtype'] == 'bf16' else 0
