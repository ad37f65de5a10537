#!/usr/bin/env python
"""A/B of GEMM schedules on the GPT-2 124M step shapes (B=64, T=1024): gpt2mi_gemm sched variants timed in
interleaved rounds with HIP events (random data).  python tools/gemm_ab.py [impl_a impl_b ...]  (default 0 6:
the persistent ping-pong schedule vs the one-tile-per-block kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
PEAK = 2516.6


def main():
    impls = [int(a) for a in sys.argv[1:]] or [0, 6]
    M, C, Vp = 65536, 768, 50432
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
    # (N, bias?, epilogue, K): forward shapes (K = C) and the dgrads that run in the forward layout against W^T
    shapes = {
        "lm_head fwd": (Vp, None, K.EPI_BF16, C),
        "qkv fwd +bias": (3 * C, True, K.EPI_BF16, C),
        "fc1 fwd gelu+drop": (4 * C, True, K.EPI_GELU, C),
        "proj dgrad": (C, None, K.EPI_BF16, C),
        "qkv dgrad": (C, None, K.EPI_BF16, 3 * C),
        "fc1 dgrad": (C, None, K.EPI_BF16, 4 * C),
        "lm_head dgrad": (C, None, K.EPI_BF16, Vp),
        "fc2 fwd +resid+drop": (C, True, K.EPI_RESID, 4 * C),
        "proj fwd +resid+drop": (C, True, K.EPI_RESID, C),
        "fc2 dgrad gelu-bwd": (4 * C, None, K.EPI_GELU_BWD, C),
    }
    if os.environ.get("GEMM_AB_SHAPES"):
        shapes = {k: v for k, v in shapes.items() if any(s in k for s in os.environ["GEMM_AB_SHAPES"].split(","))}
    bufs = {}
    xs = {}
    for name, (N, has_bias, epi, Kd) in shapes.items():
        if Kd not in xs:
            xs[Kd] = rnd(M, Kd)
        W = rnd(N, Kd, sc=0.05)
        bias = torch.randn(N, device=dev) if has_bias else None
        # EPI_RESID: fp32 out = resid + drop(acc + bias); EPI_GELU_BWD: bf16 out = acc * aux (the stored GELU derivative)
        out = torch.empty(M, N, dtype=torch.float32 if epi == K.EPI_RESID else torch.bfloat16, device=dev)
        aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev) if epi in (K.EPI_GELU, K.EPI_GELU_BWD) else None
        if epi == K.EPI_GELU_BWD:
            aux.copy_(rnd(M, N))
        resid = torch.randn(M, N, device=dev) if epi == K.EPI_RESID else None
        bufs[name] = (N, W, bias, out, aux, resid, epi, Kd)
    res = {(n, i): [] for n in shapes for i in impls}
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(5):
        for name, (N, W, bias, out, aux, resid, epi, Kd) in bufs.items():
            for impl in impls:
                xa = xs[Kd]
                drop = 0.1 if epi in (K.EPI_GELU, K.EPI_RESID) else 0.0
                fn = lambda: K.gemm(K.FWD, epi, M, N, Kd, xa, Kd, W, Kd, out, N, bias=bias, resid=resid,  # noqa: E731
                                    aux=aux, ldaux=N if aux is not None else 0, p_drop=drop, seed=5, sched=impl)
                fn()
                s, e = ev(), ev()
                s.record()
                for _r in range(10):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[(name, impl)].append(s.elapsed_time(e) / 10)
    for name, (N, *_r) in bufs.items():
        Kd = bufs[name][-1]
        line = f"{name:20s}"
        for impl in impls:
            t = sorted(res[(name, impl)])[2]
            line += f"  impl{impl}: {t * 1e3:8.1f} us {2 * M * N * Kd / t / 1e9:7.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
