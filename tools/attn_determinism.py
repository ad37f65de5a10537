#!/usr/bin/env python
"""Determinism of the attention backward: one forward, then N backwards (alternating with / without the fused bias
column sums) on the same inputs; counts outputs that differ from the first. python tools/attn_determinism.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

K.load()
dev = "cuda"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for (B, T, H, p) in [(2, 256, 4, 0.1), (2, 256, 4, 0.0), (8, 1024, 12, 0.1)]:
    C, D = H * 64, 64
    g = torch.Generator(device=dev).manual_seed(77)
    qkv = (torch.randn(B * T, 3 * C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    K.attn_fwd(qkv, out, lse, B, T, H, D, p, 5)
    outs = []
    for r in range(3):
        o2 = torch.empty_like(out)
        K.attn_fwd(qkv, o2, torch.empty_like(lse), B, T, H, D, p, 5)
        outs.append(o2)
    dout = (torch.randn(B * T, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    ref, bad = None, 0
    for i in range(n):
        delta = torch.empty(B * H, T, device=dev)
        d = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
        cs = torch.empty(B * T // 32, 3 * C, device=dev) if i % 2 else None
        K.attn_bwd(qkv, out, dout, lse, delta, d, B, T, H, D, p, 5, colsum=cs)
        torch.cuda.synchronize()
        if ref is None:
            ref = d
        elif not torch.equal(d, ref):
            bad += 1
            diff = (d.float() - ref.float()).abs()
            idx = torch.nonzero(diff.view(B * T, 3, C).amax(-1) > 0)
            print(f"  run {i}: {int((diff > 0).sum())} elements differ, (token, q/k/v) e.g. {idx[:4].tolist()}")
    fbad = sum(int(not torch.equal(o, out)) for o in outs)
    print(f"B={B} T={T} H={H} p={p}: backward {bad}/{n - 1} differ, forward {fbad}/3 differ", flush=True)
