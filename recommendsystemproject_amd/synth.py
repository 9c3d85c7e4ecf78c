"""Synthetic MovieLens-shaped batches and seeded weights (numpy PCG64; host side).

The reference trains on MovieLens-1M pickles that are not in this image, so every workload here
is synthetic data with the shape of the reference's batch dict (SURVEY.md §8a "Batch-dict type",
§8d recipe):

    {'user_tower': {'sparse': int64 [B,S], 'dense': float32 [B,Dn],
                    'sequence': {name: int64 [B,L] or [B,L,T]}},
     'item_tower': {...same...},
     'hard_negatives'?: [N x item-tower dict]}

Column layout follows RecommendationDataset._build_feature_matrices
(project/utils/DataLoader.py:129-207): non-pooled sparse features become the columns of
'sparse' in config order, pooled sparse features and sequence features go to the 'sequence'
dict, dense features become the columns of 'dense'. Sequences are right-padded with 0 the way
project/datacleaning/parsing.py:205-209 builds `hist_movie_ids`.

This module is shared by tests/, bench.py and the golden-fixture generator so the same seed
always yields the same batch.
"""
from __future__ import annotations

import numpy as np

TAGS = 3  # genre lists are padded to 3 (parsing.py:116-121)


def tower_layout(tower_cfg: dict) -> dict:
    """feature_column_mapping exactly as RecommendationDataset builds it
    (project/utils/DataLoader.py:138-207)."""
    mapping = {'sparse': {}, 'dense': {}, 'sequence': {}}
    col = 0
    for feat in tower_cfg.get('sparse_features') or []:
        if 'pooling' in feat:
            mapping['sequence'][feat['name']] = feat['name']
        else:
            mapping['sparse'][feat['name']] = col
            col += 1
    for i, feat in enumerate(tower_cfg.get('dense_features') or []):
        mapping['dense'][feat['name']] = i
    for feat in tower_cfg.get('sequence_features') or []:
        mapping['sequence'][feat['name']] = feat['name']
    return mapping


def _seq_len(tower_cfg: dict) -> int:
    return int((tower_cfg.get('transformer_parameters') or {}).get('max_seq_len', 20))


def _tags_for(rng, valid: np.ndarray, vocab: int) -> np.ndarray:
    """[...] bool -> [..., TAGS] tag lists with 1-3 tags from [1, min(18, vocab-1)], 0-padded."""
    hi = max(1, min(18, vocab - 1))
    n = rng.integers(1, TAGS + 1, size=valid.shape)
    tags = rng.integers(1, hi + 1, size=valid.shape + (TAGS,))
    keep = (np.arange(TAGS) < n[..., None]) & valid[..., None]
    return np.where(keep, tags, 0).astype(np.int64)


def _ids(rng, V: int, size, zipf: float | None) -> np.ndarray:
    """Ids in [1, V-1]: uniform, or Zipf(alpha) ranks scattered over the table by a
    multiplicative hash (SURVEY §8d's skewed variant: a few hot rows, a long cold tail)."""
    if not zipf:
        return rng.integers(1, V, size=size)
    z = rng.zipf(zipf, size=size).astype(np.uint64) - np.uint64(1)
    return ((z * np.uint64(2654435761)) % np.uint64(max(V - 1, 1))).astype(np.int64) + 1


def make_tower_batch(tower_cfg: dict, B: int, rng: np.random.Generator,
                     synth_cfg: dict | None = None, seq_len: int | None = None,
                     seq_valid: np.ndarray | None = None, ids_override: dict | None = None) -> dict:
    """One tower's batch dict. `seq_valid` [B] forces history lengths (edge cases);
    `ids_override` {feature name: int64 [B]} forces single-value ids (e.g. collisions)."""
    synth_cfg = synth_cfg or {}
    bags = synth_cfg.get('bags', {})
    zipf = synth_cfg.get('zipf')
    out: dict = {}
    sparse_cols = []
    seq: dict = {}
    for feat in tower_cfg.get('sparse_features') or []:
        name, V = feat['name'], int(feat['vocab_size'])
        if 'pooling' in feat:
            spec = bags.get(name)
            if spec is None:  # multi-valued categorical (genre_ids): 1..3 tags, padded to 3
                seq[name] = _tags_for(rng, np.ones(B, bool), V)
            else:  # long bag (C3 hist_item_ids): k ~ U{min_valid..length}, right-padded with 0
                Lb = int(spec['length'])
                k = rng.integers(int(spec.get('min_valid', 0)), Lb + 1, size=B)
                ids = _ids(rng, V, (B, Lb), zipf)
                seq[name] = np.where(np.arange(Lb)[None, :] < k[:, None], ids, 0).astype(np.int64)
        else:
            col = (_ids(rng, V, B, zipf) if V >= 1000 else rng.integers(1, V, size=B)).astype(np.int64)
            if ids_override and name in ids_override:
                col = np.asarray(ids_override[name], dtype=np.int64)
            sparse_cols.append(col)
    if sparse_cols:
        out['sparse'] = np.stack(sparse_cols, axis=1)
    dense = [np.log1p(rng.integers(0, 2000, size=B)).astype(np.float32)
             for _ in tower_cfg.get('dense_features') or []]
    if dense:
        out['dense'] = np.stack(dense, axis=1)
    seq_feats = tower_cfg.get('sequence_features') or []
    if seq_feats:
        L = seq_len or _seq_len(tower_cfg)
        k = rng.integers(0, L + 1, size=B) if seq_valid is None else np.asarray(seq_valid)
        valid = np.arange(L)[None, :] < k[:, None]
        for feat in seq_feats:
            name, V = feat['name'], int(feat['vocab_size'])
            if 'pooling' in feat:
                seq[name] = _tags_for(rng, valid, V)
            else:
                ids = _ids(rng, V, (B, L), zipf)
                seq[name] = np.where(valid, ids, 0).astype(np.int64)
    if seq:
        out['sequence'] = seq
    return out


def make_batch(cfg: dict, B: int, seed: int, seq_len: int | None = None, n_hard: int = 0,
               edge_cases: bool = False) -> dict:
    """Full two-tower batch (numpy). With `edge_cases`, row 0 has an all-padding history
     and rows 1..3 share one item id (off-diagonal collisions, T12)."""
    rng = np.random.default_rng(seed)
    tt = cfg['two_tower']
    synth_cfg = cfg.get('synthetic', {})
    ut, it = tt['user_tower'], tt['item_tower']
    seq_valid = None
    if edge_cases and ut.get('sequence_features'):
        L = seq_len or _seq_len(ut)
        seq_valid = rng.integers(0, L + 1, size=B)
        seq_valid[0] = 0
        seq_valid[min(4, B - 1)] = L
    user = make_tower_batch(ut, B, rng, synth_cfg, seq_len, seq_valid)
    override = None
    if edge_cases:
        first = next(f for f in it['sparse_features'] if 'pooling' not in f)
        ids = rng.integers(1, int(first['vocab_size']), size=B).astype(np.int64)
        ids[1:4] = ids[1]
        override = {first['name']: ids}
    item = make_tower_batch(it, B, rng, synth_cfg, ids_override=override)
    batch = {'user_tower': user, 'item_tower': item}
    if n_hard:
        batch['hard_negatives'] = [make_tower_batch(it, B, rng, synth_cfg) for _ in range(n_hard)]
    return batch


def make_state(shapes: dict, seed: int) -> dict:
    """Seeded weights for a reference-layout state_dict ({key: shape}); the same dict loads into
    the reference modules and into ours (same keys). Embedding tables of sequence
    features get a zero padding row (SequenceFeatureProcessor.py:22-29 / T3); tower tables keep a
    non-zero row 0 (GenericTower.py:43-51 / T1)."""
    rng = np.random.default_rng(seed)
    out = {}
    for key, shape in shapes.items():
        shape = tuple(shape)
        if key.endswith('num_batches_tracked'):
            out[key] = np.zeros(shape, np.int64)
        elif key.endswith('running_mean'):
            out[key] = np.zeros(shape, np.float32)
        elif key.endswith('running_var'):
            out[key] = np.ones(shape, np.float32)
        elif len(shape) == 2 and (('.embeddings.' in key and not key.endswith('.0.weight'))
                                  or key.endswith('pos_emb.weight')):
            w = rng.uniform(-0.5, 0.5, size=shape).astype(np.float32)
            if '.feature_embedder.embeddings.' in key:
                w[0] = 0.0
            out[key] = w
        elif len(shape) == 2:
            bound = 1.0 / np.sqrt(shape[1])
            out[key] = rng.uniform(-bound, bound, size=shape).astype(np.float32) * 1.5
        elif key.endswith('weight'):
            out[key] = (1.0 + rng.uniform(-0.1, 0.1, size=shape)).astype(np.float32)
        else:
            out[key] = rng.uniform(-0.1, 0.1, size=shape).astype(np.float32)
    return out


def batch_to_torch(batch, device=None):
    """numpy batch dict -> torch tensors (int64 ids, float32 dense), recursively."""
    import torch
    if isinstance(batch, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(batch))
        return t.to(device) if device is not None else t
    if isinstance(batch, dict):
        return {k: batch_to_torch(v, device) for k, v in batch.items()}
    if isinstance(batch, list):
        return [batch_to_torch(v, device) for v in batch]
    return batch
