"""Time the encoder attention forward / backward at the C2 shape with HIP events.

    python tools/attn_time.py [B] [L] [p] [fp32|bf16]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import ops, precision  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
    precision.set_compute_dtype(sys.argv[4] if len(sys.argv) > 4 else 'bf16')
    d, H = 64, 4
    dev = torch.device('cuda:0')
    qkv = torch.randn(B * L, 3 * d, device=dev)
    if ops.qkv_bf16_ok(L, d, H, B * L):
        qkv = qkv.to(torch.bfloat16)
    lens = (torch.full((B,), L, device=dev) if os.environ.get('FULL') == '1'
            else torch.randint(0, L + 1, (B,), device=dev))
    seq = (torch.arange(L, device=dev)[None, :] < lens[:, None]).long()
    key_pad, _ = ops.seq_mask(seq, 0)
    key = torch.tensor([5, 1], dtype=torch.int64, device=dev)
    dout = torch.randn(B * L, d, device=dev)
    out, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 3)
    ops.attn_bwd(qkv, key_pad, out, dout, lse, B, L, d, H, p, key, 3)
    n = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record()
    for _ in range(n):
        ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 3)
    ev[1].record()
    for _ in range(n):
        ops.attn_bwd(qkv, key_pad, out, dout, lse, B, L, d, H, p, key, 3)
    ev[2].record()
    torch.cuda.synchronize()
    print(json.dumps({'attn_fwd_us': round(ev[0].elapsed_time(ev[1]) / n * 1e3, 1),
                      'attn_bwd_us': round(ev[1].elapsed_time(ev[2]) / n * 1e3, 1)}))


if __name__ == '__main__':
    main()
