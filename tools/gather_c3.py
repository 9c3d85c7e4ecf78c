"""Composition of C3's two forward gathers (profiling tool): rs_gather_fwd on the exact segment
lists of the user and item towers (functions.tower_segments on a synthetic C3 batch), and on each
segment alone, with HIP events, cold (8 rotating batches: rows from HBM) and warm (one batch
re-gathered: rows on chip, as after the step's catch-up).

    python tools/gather_c3.py [--batches 8]
"""
import argparse
import json
import os
import sys

import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommendsystemproject_amd import _hip, ops, synth  # noqa: E402
from recommendsystemproject_amd.functions import tower_segments  # noqa: E402
from recommendsystemproject_amd.project.models.TwoTower.GenericTower import GenericTower  # noqa: E402


def timed(fn, n, it=40):
    for i in range(3):
        fn(i % n)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(it):
        fn(i % n)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', type=int, default=8)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    cfg = yaml.safe_load(open(os.path.join(ROOT, 'configs', 'c3.yaml')))
    B = int(cfg['train']['batch_size'])
    torch.manual_seed(0)
    for name in ('user_tower', 'item_tower'):
        tcfg = cfg['two_tower'][name]
        with torch.device(dev):
            tower = GenericTower(cfg, name)
        mapping = synth.tower_layout(tcfg)
        batches = [synth.batch_to_torch(synth.make_batch(cfg, B, seed=1000 + i), dev)[name] for i in range(a.batches)]
        plans = []
        for b in batches:
            segs, pp, keep, col = tower_segments(tower, b, mapping)
            plans.append((segs, keep, col))
        col = plans[0][2]
        out = torch.empty(B, col, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        nseg = len(plans[0][0])

        cases = [('all', list(range(nseg)))] + [(f'seg{i}:kind{int(plans[0][0][i].kind)}:D{int(plans[0][0][i].dim)}:'
                                               f'V{int(plans[0][0][i].vocab)}:bag{int(plans[0][0][i].bag)}', [i])
                                              for i in range(nseg)]
        st = ops.stream()
        for label, idx in cases:
            # the launch arguments built once per batch: the timed loop is one ctypes call per launch
            arrs = [ops.segments_array([plans[k][0][i] for i in idx]) for k in range(a.batches)]

            def go(k):
                _hip.call('rs_gather_fwd', arrs[k], len(idx), B, out.data_ptr(), out.stride(0), err.data_ptr(), st)
            for temp, n in (('cold', a.batches), ('warm', 1)):
                torch.cuda._sleep(int(2.4e9 * 0.005))  # the host ahead of the GPU
                us = timed(go, n)
                print(json.dumps({'tower': name, 'case': label, 'temperature': temp, 'us': round(us, 2)}), flush=True)
        del tower, batches, plans
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
