"""MLP_Tower — drop-in for project/models/TwoTower/Tower.py (same Sequential layout
mlp.{0,1,4,5,8}, same init); forward/backward run as one HIP op sequence: the custom op
rsys::mlp_tower (library.py, kernels in functions.MLPFn)."""
import torch
import torch.nn as nn

from recommendsystemproject_amd import _hip, library
from recommendsystemproject_amd.flat import ensure_flat
from recommendsystemproject_amd.rng import new_rng_state


class MLP_Tower(nn.Module):
    """MLP's General Structure: MLP -> Normalize (Tower.py:5-41)."""

    def __init__(self, input_dim, hidden_dims, output_dim, dropout=0.1):
        super().__init__()
        layers = []
        curr_dim = input_dim
        for h_dim in hidden_dims:
            layers.append(nn.Linear(curr_dim, h_dim))
            layers.append(nn.BatchNorm1d(h_dim))
            layers.append(nn.ReLU())
            layers.append(nn.Dropout(dropout))
            curr_dim = h_dim
        layers.append(nn.Linear(curr_dim, output_dim))
        self.mlp = nn.Sequential(*layers)
        self.apply(self._init_weights)
        self.register_buffer('rng_state', new_rng_state(), persistent=False)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.BatchNorm1d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)

    @property
    def dropout_p(self):
        return float(self.mlp[3].p) if len(self.mlp) > 1 else 0.0

    def forward(self, x, groups=1):
        """x [G*B, input_dim] -> L2-normalised [G*B, output_dim]; `groups` > 1 keeps separate
        BatchNorm statistics per block of B rows (one hard-negative slot per block, T13)."""
        _hip.require_device(x)
        ensure_flat(self)
        return library.mlp_tower(self, x, int(groups))
