"""Split-K sweep of the weight-gradient GEMM (gemm_wgrad: 256x256 slabs + fixed-order reduce) on the
GPT-2 124M step shapes (K = 65536 tokens), against the factor `_lib.wgrad_splits` picks.

    python tools/wgrad_splits_sweep.py

Each candidate is timed with HIP events (slab GEMM + reduce, accumulate into C as the step does),
interleaved over 3 passes; the minimum per candidate is printed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402
from kbench import timeit, PEAK  # noqa: E402

dev = "cuda"
# SWEEP_SCHED=512: the engine's bf16 slabs (K.SCHED_BF16_SLABS)
SCHED = int(os.environ.get("SWEEP_SCHED", "0"))


def main(M=65536, C=768):
    shapes = [("qkv", 3 * C, C), ("proj", C, C), ("fc1", 4 * C, C), ("fc2", C, 4 * C), ("lm_head", 50432, C)]
    for name, m, n in shapes:
        tiles = (m // 256) * (n // 256)
        pick = K.wgrad_splits(m, n, M)
        cands = sorted({s for s in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 14, 16, 18, 19, 20, 24, 28, 32)
                        if M // s >= 256 and tiles * s <= 4 * 256} | {pick})
        A = torch.randn(M, m, device=dev).to(torch.bfloat16)
        B = torch.randn(M, n, device=dev).to(torch.bfloat16)
        Cm = torch.zeros(m, n, device=dev)
        ws = torch.empty(max(cands) * m * n, device=dev)
        best = {}
        for _ in range(3):
            for s in cands:
                ms = timeit(lambda: K.gemm_wgrad(m, n, M, A, m, B, n, Cm, n, accumulate=True, workspace=ws,  # noqa
                                                 splits=s, sched=SCHED), reps=10)
                best[s] = min(best.get(s, 1e9), ms)
        line = " ".join(f"{s}:{best[s]*1e3:.0f}" for s in cands)
        top = min(best, key=best.get)
        tf = 2.0 * m * n * M / best[top] / 1e9
        print(f"{name:8s} {m}x{n} tiles={tiles:4d} pick={pick} ({best[pick]*1e3:.0f} us) best={top} "
              f"({best[top]*1e3:.0f} us, {tf:.0f} TF, {tf/PEAK*100:.1f}%) | us per split: {line}", flush=True)
        del A, B, Cm, ws


if __name__ == "__main__":
    main()
