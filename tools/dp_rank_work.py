"""Per-rank lazy-table work of the C4 step (C3 data-parallel) at W ranks, timed on ONE GPU.

After the exchange, what a rank does on the three large tables per step depends on the mode
(DESIGN.md §6):
  * replicated: every rank sorts, catches up, segment-sums and Adam-steps the UNION of all
    ranks' lookups (W x 204,800 history ids, W x 4,096 user and item ids);
  * row-sharded (default at W >= 4): the pooled history sorts the union's ids mapped to this
    rank's rows (rs_shard_map_ids: other ranks' rows sort last and are skipped) and catches up,
    segment-sums and Adam-steps only its own ~1/W of the rows; a single-id table (all-to-all)
    sorts its own 4,096 ids and the ~4,096 distinct ids it receives, and works on the latter.
This script builds those calls with synthetic uniform ids (rows ~7 optimizer steps stale, as in
the bench's 8 cycled batches) and times sort + catch-up + segment sum + Adam with HIP events,
median of 5 repetitions. The collectives themselves are not included (sizes in DESIGN.md §6).

  python tools/dp_rank_work.py [W ...]      (default: 1 2 4 8)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import _hip  # noqa: E402

DEV = torch.device('cuda:0')
B, L, D = 4096, 50, 128
LR, B1, B2, EPS = 1e-3, 0.9, 0.999, 1e-8
CAP = 64
T_STEP = 20  # optimizer steps taken; rows last stepped 1..7 steps ago


class Table:
    def __init__(self, V, gen):
        self.V = V
        self.p = torch.randn(V, D, device=DEV, generator=gen) * 0.01
        self.m = torch.randn(V, D, device=DEV, generator=gen) * 1e-3
        self.v = torch.rand(V, D, device=DEV, generator=gen) * 1e-6
        self.g = torch.zeros(V, D, device=DEV)
        # last[V][2] = (moments' step, parameters' step), both the row's last Adam step here
        self.last0 = torch.randint(T_STEP - 7, T_STEP, (V, 1), device=DEV, generator=gen,
                                   dtype=torch.int32).expand(V, 2).contiguous()
        self.last = self.last0.clone()


def _st():
    return torch.cuda.current_stream().cuda_stream


def sort(ids, rows, bag, vocab, id_bytes=8):
    n = rows * bag
    keys = torch.empty(n, dtype=torch.int32, device=DEV)
    vals = torch.empty(n, dtype=torch.int32, device=DEV)
    wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, vocab))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_lookup_sort', ids.data_ptr(), id_bytes, rows, bag, bag, vocab, keys.data_ptr(), vals.data_ptr(),
              ws.data_ptr(), _st())
    return keys, vals


def rows_work(t, keys, vals, n, bag, mode, step, consts, dout):
    hyper = (B1, B2, EPS, 0.0)
    _hip.call('rs_sorted_catchup', keys.data_ptr(), n, D, t.p.data_ptr(), t.m.data_ptr(), t.v.data_ptr(),
              t.last.data_ptr(), step.data_ptr(), consts.data_ptr(), *hyper, _st())
    ws = torch.empty(int(_hip.lib().rs_segsum_ws_bytes(n, D)) // 4 + 1, dtype=torch.int32, device=DEV)
    _hip.call('rs_segsum', keys.data_ptr(), vals.data_ptr(), n, bag, mode, -1, dout.data_ptr(), D, D,
              t.g.data_ptr(), 0, ws.data_ptr(), _st())
    _hip.call('rs_sorted_adam', keys.data_ptr(), n, D, t.p.data_ptr(), t.g.data_ptr(), t.m.data_ptr(),
              t.v.data_ptr(), t.last.data_ptr(), None, 0, step.data_ptr(), consts.data_ptr(), *hyper, 1.0, None,
              _st())


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
    gen = torch.Generator(device=DEV).manual_seed(0)
    hist, user, item = Table(10_000_000, gen), Table(1_000_000, gen), Table(10_000_000, gen)
    step = torch.zeros((), dtype=torch.int64, device=DEV)
    consts = torch.zeros(CAP, 2, device=DEV)
    consts.view(torch.int32)[0, 0] = CAP
    for _ in range(T_STEP):
        _hip.call('rs_adam_prepare', step.data_ptr(), consts.data_ptr(), CAP, LR, B1, B2, _st())
    step_keep = step.clone()
    print(f'{"W":>3} {"mode":>11} {"sort":>7} {"rows":>7} {"total ms":>9}  (per rank, per step)')
    for W in worlds:
        rng = np.random.default_rng(W)
        h_ids = torch.as_tensor(rng.integers(1, hist.V, (W * B, L)), device=DEV)
        u_ids = torch.as_tensor(rng.integers(0, user.V, (W * B, 1)), device=DEV)
        i_ids = torch.as_tensor(rng.integers(0, item.V, (W * B, 1)), device=DEV)
        dout_bag = torch.randn(W * B, D, device=DEV) * 1e-3
        for mode in (['replicated'] if W == 1 else ['replicated', 'sharded']):
            res = []
            for rep in range(5):
                step.copy_(step_keep)
                for t in (hist, user, item):
                    t.last.copy_(t.last0)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                torch.cuda.synchronize()
                ev[0].record()
                sorted_calls = []
                if mode == 'replicated':
                    for t, ids, bag, md in ((hist, h_ids, L, 1), (user, u_ids, 1, 0), (item, i_ids, 1, 0)):
                        k, v = sort(ids, W * B, bag, t.V)
                        sorted_calls.append((t, k, v, W * B * bag, bag, md))
                else:
                    # pooled history: the union's ids mapped to this rank's local rows
                    loc = torch.empty(W * B * L, dtype=torch.int64, device=DEV)
                    err = torch.zeros(1, dtype=torch.int32, device=DEV)
                    ids32 = h_ids.to(torch.int32).reshape(-1)
                    _hip.call('rs_shard_map_ids', ids32.data_ptr(), ids32.numel(), hist.V, W, 0, loc.data_ptr(),
                              err.data_ptr(), _st())
                    k, v = sort(loc, W * B, L, (hist.V + W - 1) // W)
                    sorted_calls.append((hist, k, v, W * B * L, L, 1))
                    # single-id tables (all-to-all): own ids sorted for the buckets, then the ~B
                    # distinct ids received as owner
                    for t, ids in ((user, u_ids), (item, i_ids)):
                        sort(ids[:B], B, 1, t.V)
                        k, v = sort(ids[B:2 * B] if W > 1 else ids[:B], B, 1, t.V)
                        sorted_calls.append((t, k, v, B, 1, 0))
                ev[1].record()
                for t, k, v, n, bag, md in sorted_calls:
                    rows_work(t, k, v, n, bag, md, step, consts, dout_bag if bag > 1 else dout_bag[:n])
                ev[2].record()
                torch.cuda.synchronize()
                res.append((ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])))
            s_ms, r_ms = np.median([r[0] for r in res]), np.median([r[1] for r in res])
            print(f'{W:>3} {mode:>11} {s_ms:7.3f} {r_ms:7.3f} {s_ms + r_ms:9.3f}', flush=True)


if __name__ == '__main__':
    main()
