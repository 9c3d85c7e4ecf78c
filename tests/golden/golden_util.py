"""Golden-fixture (de)serialisation shared by make_golden.py and the tests.

A fixture is data only: the case config, the seeded input batches, and the reference's outputs.
Large tensors are stored as a summary [sum, l2, <t, r>] with r a fixed pseudo-random probe
seeded from the key name, so any element error e shows up at ~|e| in the projection.
"""
from __future__ import annotations

import glob
import io
import os
import zlib

import numpy as np
import yaml

def training_fixtures(golden_dir: str):
    """The training-step fixtures of make_golden.py (per-step 'losses'); the loader and
    validate() fixtures beside them have their own tests."""
    return [p for p in sorted(glob.glob(os.path.join(golden_dir, '*.npz')))
            if 'losses' in np.load(p, allow_pickle=False).files]


FULL_LIMIT = 4096  # tensors with at most this many elements are stored whole in summary mode


def probe(key: str, shape) -> np.ndarray:
    rng = np.random.default_rng(zlib.crc32(key.encode()))
    return rng.standard_normal(size=shape).astype(np.float64)


def summarize(key: str, a) -> np.ndarray:
    a = np.asarray(a, dtype=np.float64)
    return np.array([a.sum(), np.sqrt((a * a).sum()), (a * probe(key, a.shape)).sum()])


def flatten_batch(batch, prefix: str, out: dict):
    if isinstance(batch, dict):
        for k, v in batch.items():
            flatten_batch(v, f'{prefix}/{k}', out)
    elif isinstance(batch, list):
        out[f'{prefix}/#len'] = np.array(len(batch))
        for i, v in enumerate(batch):
            flatten_batch(v, f'{prefix}/{i}', out)
    else:
        out[prefix] = np.asarray(batch)


def unflatten_batch(data: dict, prefix: str):
    keys = [k for k in data if k.startswith(prefix + '/')]
    if f'{prefix}/#len' in data:
        n = int(data[f'{prefix}/#len'])
        return [unflatten_batch(data, f'{prefix}/{i}') for i in range(n)]
    if prefix in data and not keys:
        return data[prefix]
    out = {}
    children = sorted({k[len(prefix) + 1:].split('/')[0] for k in keys})
    for c in children:
        out[c] = unflatten_batch(data, f'{prefix}/{c}')
    return out


def save(path, cfg: dict, meta: dict, arrays: dict):
    payload = dict(arrays)
    payload['__config__'] = np.frombuffer(yaml.safe_dump(cfg).encode(), dtype=np.uint8)
    payload['__meta__'] = np.frombuffer(yaml.safe_dump(meta).encode(), dtype=np.uint8)
    np.savez_compressed(path, **payload)


def load(path):
    with np.load(path, allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    cfg = yaml.safe_load(bytes(data.pop('__config__')).decode())
    meta = yaml.safe_load(bytes(data.pop('__meta__')).decode())
    return cfg, meta, data


def batches(meta: dict, data: dict):
    return [unflatten_batch(data, f'in/{s}') for s in range(meta['steps'])]


def stored(data: dict, kind: str, key: str):
    """('full', array) or ('sum', summary) for kind in {'grad', 'final'}."""
    if f'{kind}/{key}' in data:
        return 'full', data[f'{kind}/{key}']
    return 'sum', data[f'{kind}sum/{key}']


def check(kind_key: str, stored_pair, actual, rtol=1e-4, atol=1e-6):
    """Compare an actual tensor to a stored full array or summary; returns error string or ''."""
    mode, ref = stored_pair
    act = np.asarray(actual, dtype=np.float64)
    if mode == 'full':
        ref = np.asarray(ref, dtype=np.float64)
        if ref.shape != act.shape:
            return f'{kind_key}: shape {act.shape} != {ref.shape}'
        err = np.abs(act - ref).max() if act.size else 0.0
        scale = max(np.abs(ref).max() if ref.size else 0.0, 1.0)
        return '' if err <= atol + rtol * scale else f'{kind_key}: max abs err {err:.3e} (scale {scale:.3e})'
    got = summarize(kind_key.split(':', 1)[-1], act)
    scale = max(ref[1], 1.0)
    err = np.abs(got - ref).max()
    # per-element errors of size <= atol with random signs sum to ~atol*sqrt(n) in a summary
    tol = atol * max(1.0, np.sqrt(act.size)) + rtol * scale * 4
    return '' if err <= tol else f'{kind_key}: summary {got} != {ref}'


def bn_invariant_keys(cfg: dict) -> set:
    """Parameters whose exact gradient is 0 because a training-mode BatchNorm follows them
    (per-column shift/scale invariance): fp32 rounding noise is all their gradient holds, and
    Adam turns its sign into +-lr updates in the reference itself. Their post-Adam values are
    therefore only comparable to ~steps*lr; BN running means downstream of them inherit it.
      * mlp Linear biases before a BN (Tower.py:16-17), feature_bn.bias (GenericTower.py:234
        feeds mlp.0 -> BN), dense Linear(1, D) weight+bias (GenericTower.py:221),
      * last encoder layer norm2 weight+bias (its output columns go straight into feature_bn).
    """
    out = set()
    for tname, t in cfg['two_tower'].items():
        p = f'{tname}.'
        idx = 0
        for _ in t['mlp_hidden_dim']:
            out.add(f'{p}mlp.mlp.{idx}.bias')
            out.add(f'{p}mlp.mlp.{idx + 1}.running_mean')
            idx += 4
        out.add(f'{p}feature_bn.bias')
        out.add(f'{p}feature_bn.running_mean')
        out.add(f'{p}feature_bn.running_var')  # scale-invariant inputs (dense weight, norm2.weight)
        for f in t.get('dense_features') or []:
            if f['dim'] == 1:
                out.add(f'{p}embeddings.{f["name"]}.0.weight')
                out.add(f'{p}embeddings.{f["name"]}.0.bias')
        if t.get('sequence_features'):
            nl = (t.get('transformer_parameters') or {}).get('n_layers', 1)
            lp = f'{p}seq_encoder.transformer_backbone.layers.{nl - 1}.norm2.'
            out.update({lp + 'weight', lp + 'bias'})
    return out


def final_atol(key: str, cfg: dict, meta: dict) -> float:
    if key in bn_invariant_keys(cfg):
        return 2.5 * meta['steps'] * meta['lr']
    return 5e-5
