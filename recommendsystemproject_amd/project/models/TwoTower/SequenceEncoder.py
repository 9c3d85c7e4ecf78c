"""SequenceEncoder — drop-in for project/models/TwoTower/SequenceEncoder.py.

Same constructor and state_dict keys (feature_embedder.*, transformer_backbone.layers.{i}.*);
the torch nn.TransformerEncoder is kept as the parameter container, the forward/backward run
as one fused HIP op sequence: the custom op rsys::seq_encoder (library.py, kernels in
functions.SeqEncoderFn).
"""
import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip, library, ops
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.project.utils.SequenceFeatureProcessor import SequenceFeatureProcessor as pr
from recommendsystemproject_amd.rng import new_rng_state


class SequenceEncoder(nn.Module):
    def __init__(self, feature_config_list, model_dim=64, dim_feedforward=4 * 64, max_seq_len=20,
                 n_head=4, n_layers=1, dropout=0.1):
        """SequenceEncoder.py:6-29 (T8: post-LN, ReLU, batch_first, eps 1e-5)."""
        super().__init__()
        self.feature_embedder = pr(feature_config_list, model_dim, max_seq_len, dropout=dropout)
        encoder_layer = nn.TransformerEncoderLayer(d_model=model_dim, nhead=n_head,
                                                   dim_feedforward=dim_feedforward, dropout=dropout,
                                                   batch_first=True)
        self.transformer_backbone = nn.TransformerEncoder(encoder_layer, num_layers=n_layers,
                                                          enable_nested_tensor=False)
        self.n_head = n_head
        self.register_buffer('rng_state', new_rng_state(), persistent=False)
        self.register_buffer('err_flag', torch.zeros(1, dtype=torch.int32), persistent=False)

    @property
    def dropout_p(self):
        return float(self.transformer_backbone.layers[0].dropout.p)

    def forward(self, input_dict):
        """input_dict {name: [B, L] or [B, L, T]} -> [B, model_dim] (SequenceEncoder.py:32-56)."""
        _hip.require_device(self.feature_embedder.pos_emb.weight)
        ensure_flat(self)
        for lyr in self.transformer_backbone.layers:
            if getattr(lyr, 'norm_first', False) or getattr(lyr.activation, '__name__', 'relu') != 'relu':
                raise NotImplementedError('only the reference layer (post-LN, ReLU) is supported')
        return library.seq_encoder(self, input_dict)

    def _gather_last_valid(self, seq_output, padding_mask):
        """seq_output [B, L, D], padding_mask [B, L] bool -> [B, D] (SequenceEncoder.py:58-74)."""
        B, L, D = seq_output.shape
        _hip.require_device(seq_output)
        _, last = ops.seq_mask(padding_mask.to(torch.int64), 1)  # count of unmasked - 1, clamp 0
        out = torch.empty(B, D, device=seq_output.device, dtype=seq_output.dtype)
        from recommendsystemproject_amd.functions import _seg
        src = seq_output.contiguous()
        ops.gather_fwd([_seg(kind=_hip.RS_SEG_LASTVALID, dim=D, out_col=0, bag=L,
                             idx=last.data_ptr(), table=src.data_ptr())], B, out)
        return out
