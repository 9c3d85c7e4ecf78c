"""Run the encoder attention forward + backward a few times at the C2 shape (for rocprofv3 --pmc).

    python tools/attn_one.py [B] [L] [p] [fp32|bf16]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendsystemproject_amd import ops, precision  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
    precision.set_compute_dtype(sys.argv[4] if len(sys.argv) > 4 else 'fp32')
    d, H = 64, 4
    dev = torch.device('cuda:0')
    qkv = torch.randn(B * L, 3 * d, device=dev)
    if ops.qkv_bf16_ok(L, d, H, B * L):  # the bf16 mode's qkv storage (RS_ATTN_QKV_BF16)
        qkv = qkv.to(torch.bfloat16)
    lens = torch.randint(0, L + 1, (B,), device=dev)
    seq = (torch.arange(L, device=dev)[None, :] < lens[:, None]).long()
    key_pad, _ = ops.seq_mask(seq, 0)
    key = torch.tensor([5, 1], dtype=torch.int64, device=dev)
    dout = torch.randn(B * L, d, device=dev)
    for _ in range(3):
        out, lse = ops.attn_fwd(qkv, key_pad, B, L, d, H, p, key, 3)
        ops.attn_bwd(qkv, key_pad, out, dout, lse, B, L, d, H, p, key, 3)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
