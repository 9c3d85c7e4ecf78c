"""SequenceFeatureProcessor — drop-in for project/utils/SequenceFeatureProcessor.py.

Same constructor, attributes and state_dict keys (embeddings.<name>.weight,
feature_projection.0.{weight,bias}, pos_emb.weight); forward runs the fused HIP path
(per-token gather + tag pooling + projection + positional embedding + dropouts) on MI355X.
"""
import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip, ops
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.functions import seq_input_bwd, seq_input_fwd
from recommendsystemproject_amd.rng import new_rng_state


class _SeqInputFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, need, proc, seqd, *params):
        first = next(v for v in seqd.values())
        B, L = int(first.shape[0]), int(first.shape[1])
        if L > proc.pos_emb.num_embeddings:
            raise IndexError('index out of range in self')
        p = proc.dropout if proc.training else 0.0
        key = ops.rng_next(proc.rng_state) if p > 0 else None
        x, saved = seq_input_fwd(proc, seqd, B, L, p, key, proc.err_flag)
        if need:
            ctx.proc, ctx.saved, ctx.B, ctx.L, ctx.p, ctx.key = proc, saved, B, L, p, key
        return x.view(B, L, proc.target_dim)

    @staticmethod
    def backward(ctx, dx):
        dx = dx.contiguous().view(ctx.B * ctx.L, -1).clone()
        seq_input_bwd(ctx.proc, ctx.saved, dx, ctx.B, ctx.L, ctx.p, ctx.key)
        return (None, None, None) + (None,) * (len(ctx.needs_input_grad) - 3)


class SequenceFeatureProcessor(nn.Module):
    def __init__(self, feature_config_list, target_dim, max_seq_len, dropout=0.1):
        """SequenceFeatureProcessor.py:6-36 (T3: padding index key is 'padding_index')."""
        super().__init__()
        self.feature_config_list = feature_config_list
        self.target_dim = target_dim
        self.dropout = dropout
        self.embeddings = nn.ModuleDict()
        total_concat_dim = 0
        for feat_cfg in feature_config_list:
            self.embeddings[feat_cfg['name']] = nn.Embedding(
                num_embeddings=feat_cfg['vocab_size'], embedding_dim=feat_cfg['embedding_dim'],
                padding_idx=feat_cfg.get('padding_index', 0))
            total_concat_dim += feat_cfg['embedding_dim']
        self.feature_projection = nn.Sequential(nn.Linear(total_concat_dim, target_dim), nn.Dropout(dropout))
        self.pos_emb = nn.Embedding(max_seq_len, target_dim)
        self.register_buffer('rng_state', new_rng_state(), persistent=False)
        self.register_buffer('err_flag', torch.zeros(1, dtype=torch.int32), persistent=False)

    def forward(self, input_dict):
        """[B, L, target_dim] (SequenceFeatureProcessor.py:38-85)."""
        _hip.require_device(self.pos_emb.weight)
        ensure_flat(self)
        return _SeqInputFn.apply(torch.is_grad_enabled(), self, input_dict, *self.parameters())
