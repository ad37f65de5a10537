"""Does the cross-entropy pass run faster on logits still held by the 256 MB MALL (Infinity Cache)?

The lm_head forward writes 6.6 GB of bf16 logits that xent reads straight back (2.4 ms, HBM-bound). Run both in row
chunks small enough for a chunk's logits to stay in the MALL (R rows x 50432 x 2 B: 1024 rows = 103 MB) and time the
GEMM and xent launches of the chunked sequence against the whole-batch pair, HIP events.

    python tools/mall_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"


def main():
    M, C, V, Vp = 65536, 768, 50257, 50432
    g = torch.Generator(device=dev).manual_seed(0)
    lnf = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    wte = (torch.randn(Vp, C, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    logits = torch.empty(M, Vp, device=dev, dtype=torch.bfloat16)
    dlogits = torch.empty(M, Vp, device=dev, dtype=torch.bfloat16)
    labels = torch.randint(0, V, (M,), device=dev, generator=g)
    loss_rows = torch.empty(M, device=dev)
    lse = torch.empty(M, device=dev)
    loss = torch.empty(1, device=dev)
    inv = torch.empty(1, device=dev)

    def gemm(r0, R):
        K.gemm(0, K.EPI_BF16, R, Vp, C, lnf[r0:], C, wte, C, logits[r0:], Vp)

    def xent(r0, R):
        K.xent_fwd(logits[r0:], Vp, labels[r0:], loss_rows[r0:], lse[r0:], dlogits[r0:], Vp, R, V, loss, inv)

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def run(R):
        evs = []
        for r0 in range(0, M, R):
            e0, e1, e2 = ev(), ev(), ev()
            e0.record()
            gemm(r0, R)
            e1.record()
            xent(r0, R)
            e2.record()
            evs.append((e0, e1, e2))
        torch.cuda.synchronize()
        tg = sum(a.elapsed_time(b) for a, b, _ in evs)
        tx = sum(b.elapsed_time(c) for _, b, c in evs)
        return tg, tx, evs[0][0].elapsed_time(evs[-1][2])

    for R in (M, 8192, 4096, 2048, 1024, M):
        run(R)  # warm
        res = [run(R) for _ in range(3)]
        tg, tx, tt = (min(r[i] for r in res) for i in range(3))
        print(f"rows/chunk {R:6d}: lm_head fwd {tg:7.3f} ms  xent {tx:7.3f} ms  total {tt:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
