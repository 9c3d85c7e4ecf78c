"""SequenceFeatureProcessor — drop-in for project/utils/SequenceFeatureProcessor.py.

Same constructor, attributes and state_dict keys (embeddings.<name>.weight,
feature_projection.0.{weight,bias}, pos_emb.weight); forward runs the fused HIP path
(per-token gather + tag pooling + projection + positional embedding + dropouts) on MI355X as
the custom op rsys::seq_features (library.py; kernels in functions.SeqFeaturesFn).
"""
import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip, library
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.rng import new_rng_state


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
        return library.seq_features(self, input_dict)
