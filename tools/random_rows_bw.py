"""Random-row read ceiling on one MI355X for the C3 history gather's access pattern: 204,800
lookups of 512-byte rows (fp32 x 128) from a 10M-row table, 8 rotating id sets (no Infinity-Cache
reuse), timed with HIP events. Compares torch.index_select and torch.embedding_bag (ATen kernels,
not ours) with rs_gather_fwd's own pooled launch figure in DESIGN.md §5.

    python tools/random_rows_bw.py
"""
import json

import torch


def timed(fn, it=20):
    for _ in range(3):
        fn(0)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(it):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = torch.device('cuda:0')
    V, D, B, L = 10_000_000, 128, 4096, 50
    table = torch.randn(V, D, device=dev)
    ids = [torch.randint(0, V, (B * L,), device=dev) for _ in range(8)]
    out = torch.empty(B * L, D, device=dev)
    bag = torch.empty(B, D, device=dev)
    offs = torch.arange(0, B * L, L, device=dev)
    res = {}
    ms = timed(lambda i: torch.index_select(table, 0, ids[i % 8], out=out))
    res['index_select_rows_TBps_read'] = round(B * L * D * 4 / ms / 1e9, 2)
    res['index_select_us'] = round(ms * 1e3, 1)
    ms = timed(lambda i: bag.copy_(torch.nn.functional.embedding_bag(ids[i % 8], table, offs, mode='mean')))
    res['embedding_bag_mean_TBps_read'] = round(B * L * D * 4 / ms / 1e9, 2)
    res['embedding_bag_us'] = round(ms * 1e3, 1)
    srt = [torch.sort(x).values for x in ids]
    ms = timed(lambda i: torch.index_select(table, 0, srt[i % 8], out=out))
    res['index_select_sorted_ids_TBps_read'] = round(B * L * D * 4 / ms / 1e9, 2)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
