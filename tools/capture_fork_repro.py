"""Bisect a hipGraph capture crash with a forked side stream (GPU box).
Usage: python tools/capture_fork_repro.py <variant>"""
import sys

import torch

sys.path.insert(0, '.')
from recommendsystemproject_amd import _hip  # noqa: E402

v = sys.argv[1]
dev = torch.device('cuda:0')
side = torch.cuda.Stream()
ids = torch.randint(0, 1000000, (4096, 50), device=dev)
x = torch.randn(1 << 20, device=dev)


def sort_on_side(cur):
    n = ids.numel()
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    vals = torch.empty(n, dtype=torch.int32, device=dev)
    wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, 1000000))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev)
    side.wait_stream(cur)
    _hip.call('rs_lookup_sort', ids.data_ptr(), 8, 4096, 50, 50, 1000000, keys.data_ptr(),
              vals.data_ptr(), ws.data_ptr(), side.cuda_stream)
    return keys, vals, ws


class Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a):
        cur = torch.cuda.current_stream()
        ctx.held = [sort_on_side(cur) for _ in range(3)]
        return a * 2

    @staticmethod
    def backward(ctx, g):
        for _ in ctx.held:
            torch.cuda.current_stream().wait_stream(side)
        return g * 2


w = torch.randn(1024, device=dev, requires_grad=True)


tower = torch.cuda.Stream()


def body():
    cur = torch.cuda.current_stream()
    if v in ('nested', 'nested2'):
        # the model's pattern: item tower on a side stream forks the sort stream from there, the
        # user tower forks it from the capture stream; joins in the backward order
        tower.wait_stream(cur)
        with torch.cuda.stream(tower):
            h1 = sort_on_side(tower)
            y1 = x * 2
        h2 = sort_on_side(cur)
        y2 = x * 3
        if v == 'nested':
            with torch.cuda.stream(tower):
                tower.wait_stream(side)
                y1 = y1 + 1
        cur.wait_stream(side)
        y2 = y2 + 1
        cur.wait_stream(tower)
        return y1, y2, h1, h2
    if v == 'fork_fresh':  # one level: a stream made here forks from the capturing stream and joins back
        a_st = torch.cuda.Stream()
        a_st.wait_stream(cur)
        with torch.cuda.stream(a_st):
            y1 = x * 2
        cur.wait_stream(a_st)
        return y1
    if v in ('chain', 'chain_fresh', 'chain_dj'):
        # a fork of a fork: cur -> A, A -> B, B joined into A, A joined into cur (the user tower on
        # its own stream forking its per-table lookup stream: TwoTowerModel RSYS_USER_STREAM=1)
        a_st = tower if v == 'chain' else torch.cuda.Stream()  # chain_fresh / chain_dj: new streams
        a_st.wait_stream(cur)
        with torch.cuda.stream(a_st):
            y1 = x * 2
            b_st = side if v == 'chain' else torch.cuda.Stream()
            b_st.wait_stream(a_st)
            with torch.cuda.stream(b_st):
                y2 = x * 3
            a_st.wait_stream(b_st)
            y1 = y1 + y2
        cur.wait_stream(a_st)
        if v == 'chain_dj':  # the grandchild also joined straight into the origin
            cur.wait_stream(b_st)
        return y1, y2
    if v == 'autograd':
        y = Fn.apply(w)
        y.sum().backward()
        return y
    y = x * 2
    n = ids.numel()
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    vals = torch.empty(n, dtype=torch.int32, device=dev)
    wsb = int(_hip.lib().rs_lookup_sort_ws_bytes(n, 1000000))
    ws = torch.empty(wsb // 4 + 1, dtype=torch.int32, device=dev)
    side.wait_stream(cur)
    if v == 'torch':
        with torch.cuda.stream(side):
            z = x + 1
    else:
        _hip.call('rs_lookup_sort', ids.data_ptr(), 8, 4096, 50, 50, 1000000, keys.data_ptr(),
                  vals.data_ptr(), ws.data_ptr(), side.cuda_stream)
    y = y * 3
    cur.wait_stream(side)
    return y, keys, vals, ws


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g, capture_error_mode='thread_local'):
    out = body()
g.replay()
torch.cuda.synchronize()
print('ok', v, flush=True)
