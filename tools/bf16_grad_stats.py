"""Measure the bf16 compute mode against the fp32 oracle (tests/bf16_check.py): per-tensor
relative gradient error vs 4u sqrt(depth), regression slope z-scores, embedding / logit errors and
the per-row loss bias, for C2 (B = 1024), C3 capped (B = 1024) and C5 capped (B = 256, N = 10).

    python tools/bf16_grad_stats.py [case ...]   -> one JSON line per case
    case: c2 | c3 | c5 | gold:<fixture> (tests/golden/<fixture>.npz, its first batch), optionally
          followed by @ENV=VALUE,... (switches for that case only; DTYPE=fp32 runs the control)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

import bf16_check as bc  # noqa: E402
from recommendsystemproject_amd import precision  # noqa: E402

CASES = {'c2': ('c2', 1024, None, 0), 'c3': ('c3', 1024, 1_000_000, 0), 'c5': ('c5', 256, 1_000_000, 10)}


def cfg_of(name, cap):
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', f'{name}.yaml')))
    for t in cfg['two_tower'].values():
        t['dropout'] = 0.0
        t.get('transformer_parameters', {})['dropout'] = 0.0
        if cap:
            for f in (t.get('sparse_features') or []) + (t.get('sequence_features') or []):
                f['vocab_size'] = min(int(f['vocab_size']), cap)
    return cfg


def main():
    names = sys.argv[1:] or list(CASES)
    precision.set_compute_dtype('bf16')
    dev = torch.device('cuda:0')
    for spec in names:
        # case[@ENV=VALUE,...]: the environment switches apply to this case only
        n, _, envs = spec.partition('@')
        for kv in filter(None, envs.split(',')):
            k, _, v = kv.partition('=')
            os.environ[k] = v
        precision.set_compute_dtype(os.environ.get('DTYPE', 'bf16'))  # DTYPE=fp32: the control
        if n.startswith('gold:'):  # a golden fixture's config, weights and first batch
            import golden_util as gu
            from oracle.twotower_oracle import model_state_shapes
            from recommendsystemproject_amd import synth
            cfg, meta, data = gu.load(os.path.join(ROOT, 'tests', 'golden', n[5:] + '.npz'))
            shapes = {k: s for k, s, _ in model_state_shapes(cfg)}
            b0 = gu.batches(meta, data)[0]
            B = len(b0['item_tower']['sparse'])
            r = bc.bf16_vs_oracle(cfg, B, dev, 0, state=synth.make_state(shapes, seed=meta['weight_seed']),
                                  batch=b0, T=meta['temperature'])
        else:
            name, B, cap, N = CASES[n]
            cfg = cfg_of(name, cap)
            r = bc.bf16_vs_oracle(cfg, B, dev, seed=61, n_neg=N)
        h, f = r['hip'], r['ref']
        T = float(meta['temperature']) if n.startswith('gold:') else float(cfg['train']['temperature'])
        ok = f['logits'] > -1e8
        d = bc.row_losses(h['logits']) - bc.row_losses(f['logits'])
        stats = bc.grad_stats(h['grads'], f['grads'], cfg, f['kappa'], B)
        out = dict(case=spec, B=B, depth=bc.depth(cfg), rel_tol=bc.rel_tol(cfg),
                   emb_err={k: float((h[k] - f[k]).abs().max()) for k in ('U', 'I', 'H') if f[k] is not None},
                   logit_err=float((h['logits'][ok] - f['logits'][ok]).abs().max()),
                   tol_logit=(2 * 4 * bc.U_BF16 + 2 * bc.U_BF16) / T,
                   loss=(h['loss'], f['loss']), bias_mean=float(d.mean()), bias_se=float(d.std() / np.sqrt(B)),
                   worst_rel=max(s['rel'] for s in stats), worst_z=max(abs(s['z']) for s in stats),
                   grads=sorted(stats, key=lambda s: -s['rel']), fails=bc.check_grads(h['grads'], f['grads'], cfg, f['kappa'], B))
        print(json.dumps(out), flush=True)
        del r
        torch.cuda.empty_cache()
        for kv in filter(None, envs.split(',')):
            os.environ.pop(kv.partition('=')[0], None)


if __name__ == '__main__':
    main()
