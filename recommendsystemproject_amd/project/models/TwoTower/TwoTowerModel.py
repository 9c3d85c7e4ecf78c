"""TwoTowerModel — drop-in for project/models/TwoTower/TwoTowerModel.py (same API:
forward / predict / get_item_embeddings / compute_loss / set_feature_mappings). compute_loss is
one fused HIP op (functions.InBatchLossFn): U I^T on the MFMA GEMM, collision mask, hard
negatives and the softmax cross-entropy in one row kernel."""
import os

import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.functions import InBatchLossFn


class TwoTowerModel(nn.Module):
    def __init__(self, user_tower, item_tower, user_feature_mapping=None, item_feature_mapping=None):
        super().__init__()
        self.user_tower = user_tower
        self.item_tower = item_tower
        self.user_feature_mapping = user_feature_mapping
        self.item_feature_mapping = item_feature_mapping
        # the reference raises on NaN embeddings with a host sync per step (TwoTowerModel.py:88-91);
        # opt in with RSYS_CHECK_NAN=1 or model.check_nan = True
        self.check_nan = os.environ.get('RSYS_CHECK_NAN', '0') == '1'

    def set_feature_mappings(self, user_mapping, item_mapping):
        self.user_feature_mapping = user_mapping
        self.item_feature_mapping = item_mapping

    def forward(self, batch_data):
        """-> (user_emb [B,D], item_emb [B,D], hard_neg_emb [B,N,D] or None) (TwoTowerModel.py:35-62;
        T13: one item-tower pass per hard-negative slot, so BatchNorm statistics are per slot)."""
        _hip.require_device(self.user_tower.feature_bn.weight)
        ensure_flat(self)
        user_emb = self.user_tower(batch_data['user_tower'], self.user_feature_mapping)
        item_emb = self.item_tower(batch_data['item_tower'], self.item_feature_mapping)
        hard_neg_emb = None
        negs = batch_data.get('hard_negatives') if isinstance(batch_data, dict) else None
        if negs:
            stacked = getattr(negs, 'stacked', None)
            if stacked is not None:
                # materialised by ItemCatalog: the N slots are already one [N*B] batch; one item-tower
                # pass with per-slot BatchNorm statistics == N separate passes (T13)
                N = len(negs)
                out = self.item_tower(stacked, self.item_feature_mapping, groups=N)
                B = out.shape[0] // N
                hard_neg_emb = out.view(N, B, out.shape[1]).transpose(0, 1)  # [B, N, D] view
            else:
                hard_neg_emb = torch.stack([self.item_tower(neg, self.item_feature_mapping)
                                            for neg in negs], dim=1)
        return user_emb, item_emb, hard_neg_emb

    def predict(self, batch_data):
        user_emb, item_emb, _ = self.forward(batch_data)
        return (user_emb * item_emb).sum(dim=1)

    def get_item_embeddings(self, item_inputs):
        return self.item_tower(item_inputs, self.item_feature_mapping)

    def compute_loss(self, user_emb, item_emb, item_ids=None, hard_neg_emb=None, temperature=0.1):
        """In-batch softmax loss (TwoTowerModel.py:81-150)."""
        if self.check_nan:
            if torch.isnan(user_emb).any():
                raise RuntimeError('Found NaN in User Embedding')
            if torch.isnan(item_emb).any():
                raise RuntimeError('Found NaN in Item Embedding')
        batch_size = user_emb.shape[0]
        if hard_neg_emb is not None:
            if self.check_nan and torch.isnan(hard_neg_emb).any():
                raise RuntimeError('Found NaN in Hard Negative Embedding')
            assert hard_neg_emb.dim() == 3, f'Expected shape [B, N, D], got {hard_neg_emb.shape}'
            assert hard_neg_emb.size(0) == batch_size, 'Batch size mismatch'
        return InBatchLossFn.apply(user_emb, item_emb, item_ids, hard_neg_emb, float(temperature))
