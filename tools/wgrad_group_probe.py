#!/usr/bin/env python
"""Prices a grouped weight-gradient launch before building one: the four block weight gradients of a GPT-2 124M layer
(qkv 2304x768, proj 768x768, fc1 3072x768, fc2 768x3072 over 65536 tokens) as four launches at their default split-K
factors (what the step runs: each one round of ~250 blocks + its reduction) against ONE launch of the same total tile
count and per-block depth (9216 x 768 = 108 tiles, 7 splits = 756 blocks, ~3 rounds, one reduction). HIP events,
interleaved rounds, median."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
Mt = 65536
g = torch.Generator(device=dev).manual_seed(0)
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
data = {}
for n, (m, nn) in shapes.items():
    A = (torch.randn(Mt, m, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    B = torch.randn(Mt, nn, device=dev, generator=g).to(torch.bfloat16)
    C = torch.empty(m, nn, device=dev)
    data[n] = (m, nn, A, B, C, K.wgrad_splits(m, nn, Mt))
ws = torch.empty(32 * 3072 * 768, device=dev)
GA = (torch.randn(Mt, 9216, device=dev, generator=g) * 0.1).to(torch.bfloat16)
GB = torch.randn(Mt, 768, device=dev, generator=g).to(torch.bfloat16)
GC = torch.empty(9216, 768, device=dev)


def four():
    for n, (m, nn, A, B, C, sp) in data.items():
        K.gemm_wgrad(m, nn, Mt, A, m, B, nn, C, nn, accumulate=False, workspace=ws, splits=sp)


def grouped(sp):
    K.gemm_wgrad(9216, 768, Mt, GA, 9216, GB, 768, GC, 768, accumulate=False, workspace=ws, splits=sp)


cases = {"four launches (default splits " + ",".join(str(v[5]) for v in data.values()) + ")": four,
         "one launch 9216x768, 7 splits": lambda: grouped(7),
         "one launch 9216x768, 9 splits": lambda: grouped(9),
         "one launch 9216x768, 4 splits": lambda: grouped(4)}
times = {k: [] for k in cases}
for f in cases.values():
    f()
torch.cuda.synchronize()
for _ in range(7):
    for k, f in cases.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _r in range(5):
            f()
        e.record()
        torch.cuda.synchronize()
        times[k].append(s.elapsed_time(e) / 5 * 1e3)
flop = 2 * Mt * sum(m * n for m, n, *_ in data.values())
for k, v in times.items():
    t = sorted(v)[3]
    print(f"{k:45s} {t:8.1f} us  {flop / t / 1e6:7.0f} TF", flush=True)
