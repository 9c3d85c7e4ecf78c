"""Golden fixture for the device batch assembly, produced by the REFERENCE itself
(build container only; the reference is imported from /root/reference, never copied):

    python tests/golden/make_loader_golden.py      # writes tests/golden/loader_demo.npz

A seeded 200-row DataFrame with the demo schema (tests/test_device_loader.make_df,
histories ragged) goes through the reference's CombinedTwoTowerDataLoader (CombineTwoTower.py:13-105:
RecommendationDataset per tower, DataLoader(shuffle=True) under torch.manual_seed(7),
collate_fn of DataLoader.py:250-288). Stored: the DataFrame's columns (lists as flat values +
offsets) and every batch tensor of one epoch, keyed b{k}/{tower}/{sparse|dense|seq:<name>}, plus
the feature column mappings. The pickle the loader reads is written here, by this script.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, REF)

from test_device_loader import make_df  # noqa: E402

N, B, SEED = 200, 64, 7


def flat_lists(col):
    """A list-of-lists (or list-of-list-of-lists) column -> values, offsets."""
    offs = np.zeros(len(col) + 1, dtype=np.int64)
    vals = []
    for i, v in enumerate(col):
        offs[i + 1] = offs[i] + len(v)
        vals.extend(v)
    arr = np.array(vals, dtype=np.int64)
    return arr, offs


def main():
    from project.utils.CombineTwoTower import CombinedTwoTowerDataLoader
    # histories of 1..25 positions (ragged): the reference's collate raises on an EMPTY list of a
    # list-of-lists feature (np.stack of a (0,) and an (L, 3) array), so none is empty here
    df = make_df(N, seed=11, min_hist=1)
    pkl = '/tmp/rsys_loader_golden.pkl'
    df.to_pickle(pkl)
    cfg = os.path.join(ROOT, 'configs', 'demo.yaml')
    torch.manual_seed(SEED)
    loader = CombinedTwoTowerDataLoader(cfg, pkl, batch_size=B, shuffle=True)
    out = {}
    for c in df.columns:
        v = df[c].tolist()
        if isinstance(v[0], list) or any(isinstance(x, list) for x in v):
            vals, offs = flat_lists(v)
            out[f'df/{c}/vals'] = vals
            out[f'df/{c}/offs'] = offs
        else:
            out[f'df/{c}'] = np.asarray(v)
    nb = 0
    for k, batch in enumerate(loader):
        for tower, tb in batch.items():
            for key in ('sparse', 'dense'):
                if key in tb:
                    out[f'b{k}/{tower}/{key}'] = tb[key].numpy()
            for f, t in tb.get('sequence', {}).items():
                out[f'b{k}/{tower}/seq:{f}'] = t.numpy()
        nb += 1
    out['meta'] = np.frombuffer(json.dumps({'N': N, 'B': B, 'seed': SEED, 'batches': nb,
                                            'columns': list(df.columns),
                                            'mapping': loader.get_feature_mappings()}).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, 'loader_demo.npz'), **out)
    print('loader_demo.npz:', nb, 'batches,', len(out), 'arrays')


if __name__ == '__main__':
    main()
