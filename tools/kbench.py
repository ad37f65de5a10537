"""Kernel micro-benchmarks on the MI355X (HIP events; random data; interleaved repeats).

    python tools/kbench.py [attn] [gemm] [mem]

Shapes are those of the GPT-2 124M step at B=64, T=1024 (M = 65536 tokens)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
PEAK = 2516.6


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def attn(B=64, T=1024, H=12, p=0.0):
    D = 64
    C = H * D
    qkv = (torch.randn(B * T, 3 * C, device=dev) * 0.5).to(torch.bfloat16)
    out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B * H, T, device=dev)
    dout = torch.randn(B * T, C, device=dev).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B * H, T, device=dev)
    fl = 4.0 * B * H * (T * (T + 1) / 2) * D
    f = timeit(lambda: K.attn_fwd(qkv, out, lse, B, T, H, D, p, 1))
    b = timeit(lambda: K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, D, p, 1))
    print(f"attn p={p}: fwd {f:.3f} ms {fl/f/1e9:.0f} TF | bwd {b:.3f} ms {2.5*fl/b/1e9:.0f} TF(2.5x fwd flop)")


def gemm(M=65536, sched=0):
    C = 768
    shapes = [
        ("qkv fwd", 0, K.EPI_BF16, M, 3 * C, C),
        ("fc1 fwd gelu", 0, K.EPI_GELU, M, 4 * C, C),
        ("fc2 fwd resid", 0, K.EPI_RESID, M, C, 4 * C),
        ("proj fwd resid", 0, K.EPI_RESID, M, C, C),
        ("lm_head fwd", 0, K.EPI_BF16, M, 50432, C),
        ("fc2 dgrad gelu", 1, K.EPI_GELU_BWD, M, 4 * C, C),
        ("qkv dgrad", 1, K.EPI_BF16, M, C, 3 * C),
        ("lm dgrad", 1, K.EPI_BF16, M, C, 50432),
        ("fc1 wgrad", 2, K.EPI_ATOMIC, 4 * C, C, M),
        ("fc2 wgrad", 2, K.EPI_ATOMIC, C, 4 * C, M),
        ("proj wgrad", 2, K.EPI_ATOMIC, C, C, M),
        ("qkv wgrad", 2, K.EPI_ATOMIC, 3 * C, C, M),
        ("lm wgrad", 2, K.EPI_F32, 50432, C, M),
    ]
    for name, lay, epi, m, n, k in shapes:
        if lay == 0:
            A = torch.randn(m, k, device=dev).to(torch.bfloat16); lda = k
            Bm = torch.randn(n, k, device=dev).to(torch.bfloat16); ldb = k
        elif lay == 1:
            A = torch.randn(m, k, device=dev).to(torch.bfloat16); lda = k
            Bm = torch.randn(k, n, device=dev).to(torch.bfloat16); ldb = n
        else:
            A = torch.randn(k, m, device=dev).to(torch.bfloat16); lda = m
            Bm = torch.randn(k, n, device=dev).to(torch.bfloat16); ldb = n
        out_f32 = epi in (K.EPI_F32, K.EPI_ATOMIC, K.EPI_RESID)
        Cm = torch.zeros(m, n, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        bias = torch.zeros(n, device=dev)
        resid = torch.zeros(m, n, device=dev) if epi == K.EPI_RESID else None
        aux = torch.zeros(m, n, device=dev, dtype=torch.bfloat16) if epi in (K.EPI_GELU, K.EPI_GELU_BWD) else None
        splits = 4 if epi == K.EPI_ATOMIC else 1
        if lay == 2 and m % 256 == 0:
            sp = K.wgrad_splits(m, n, k)
            wsb = torch.empty(max(4, sp * m * n if sp > 1 else 4), device=dev)
            fn = lambda: K.gemm_wgrad(m, n, k, A, lda, Bm, ldb, Cm, n, workspace=wsb, splits=sp, sched=sched)  # noqa
        else:
            fn = lambda: K.gemm(lay, epi, m, n, k, A, lda, Bm, ldb, Cm, n, bias=bias if lay == 0 else None,  # noqa
                                resid=resid, aux=aux, ldaux=n, splits=splits,
                                p_drop=0.1 if epi in (K.EPI_GELU, K.EPI_RESID) else 0.0, seed=7, sched=sched)
        ms = timeit(fn, reps=10)
        tf = 2.0 * m * n * k / ms / 1e9
        print(f"{name:16s} M={m:6d} N={n:6d} K={k:6d}: {ms:7.3f} ms {tf:6.0f} TF ({tf/PEAK*100:4.1f}%)")
        del A, Bm, Cm, resid, aux
    # hipBLASLt reference point for the same plain shape (not used by the product path)
    A = torch.randn(M, C, device=dev).to(torch.bfloat16)
    W = torch.randn(50304, C, device=dev).to(torch.bfloat16)
    ms = timeit(lambda: A @ W.t(), reps=10)
    print(f"[torch/hipBLASLt reference] lm_head fwd: {ms:.3f} ms {2.0*M*50304*C/ms/1e9:.0f} TF")
    W = torch.randn(4 * C, C, device=dev).to(torch.bfloat16)
    ms = timeit(lambda: A @ W.t(), reps=10)
    print(f"[torch/hipBLASLt reference] fc1 fwd: {ms:.3f} ms {2.0*M*4*C*C/ms/1e9:.0f} TF")


def mem(M=65536, C=768, Vp=50432, V=50257):
    """Bandwidth-bound kernels at their step shapes; GB/s from algorithmic bytes."""
    g = torch.Generator(device=dev).manual_seed(0)
    logits = (torch.randn(M, Vp, device=dev, generator=g) * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (M,), device=dev, generator=g)
    dl = torch.empty_like(logits)
    lr, lse = torch.empty(M, device=dev), torch.empty(M, device=dev)
    loss, ic = torch.empty(1, device=dev), torch.empty(1, device=dev)
    ms = timeit(lambda: K.xent_fwd(logits, Vp, labels, lr, lse, dl, Vp, M, V, loss, ic), reps=10)
    print(f"xent             {ms:7.3f} ms {4.0 * M * Vp / ms / 1e6:6.0f} GB/s")
    del logits, dl
    x = torch.randn(M, C, device=dev, generator=g)
    w, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    y = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    ms = timeit(lambda: K.layernorm_fwd(x, w, b, y, None, mean, rstd, M, C, 1e-5), reps=20)
    print(f"ln fwd           {ms:7.3f} ms {(6.0 * M * C + 8 * M) / ms / 1e6:6.0f} GB/s")
    dy = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    dres = torch.zeros(M, C, device=dev)
    dw, db, dbo = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    ob = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    ms = timeit(lambda: K.layernorm_bwd(x, w, mean, rstd, dy, dres, dw, db, ob, dbo, M, C, 0.1, 7), reps=20)
    print(f"ln bwd           {ms:7.3f} ms {16.0 * M * C / ms / 1e6:6.0f} GB/s (16 B/element)")
    del x, dy, dres, ob, y
    n = 124475904
    pp, gg, m1, v1 = (torch.randn(n, device=dev, generator=g) for _ in range(4))
    v1.abs_()
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    part = torch.empty(K.norm_partials_size(), device=dev)
    gn = torch.empty(1, device=dev)
    ms = timeit(lambda: K.adamw(pp, gg, m1, v1, pb, n, 1e-4, 0.1, 0.9, 0.95, 1e-8, 1, 1.0, part, gn), reps=10)
    print(f"adamw            {ms:7.3f} ms {30.0 * n / ms / 1e6:6.0f} GB/s (30 B/param)")


if __name__ == "__main__":
    what = sys.argv[1:] or ["attn", "gemm"]
    K.load()
    if "attn" in what:
        attn(p=0.0)
        attn(p=0.1)
    if "mem" in what:
        mem()
    if "gemm" in what:
        impls = [int(a[5:]) for a in sys.argv[1:] if a.startswith("impl=")] or [0, 2]
        for impl in impls:
            print(f"--- gemm impl {impl} ({ {0: 'ping-pong 256x256', 1: '128x128 only', 2: '2-stage 256x256'}[impl] })")
            gemm(sched=impl)
