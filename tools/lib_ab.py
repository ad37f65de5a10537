#!/usr/bin/env python
"""A/B of library builds (same C ABI) on the GPT-2 124M weight-gradient shapes (K = 65536 tokens): every
library in argv is loaded side by side with ctypes, outputs are compared bitwise against the first, and
the wgrad GEMM (gpt2mi_gemm_wgrad, the split-K choice of _lib.wgrad_splits) is timed in interleaved rounds.

    python tools/lib_ab.py libA.so libB.so ...
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"


def bind(path, _n=[0]):
    # a private copy per argument, so the same library can be listed twice with different settings
    import shutil
    import tempfile
    _n[0] += 1
    cp = os.path.join(tempfile.mkdtemp(), f"lib{_n[0]}.so")
    shutil.copy(path, cp)
    lib = ctypes.CDLL(cp)
    for name, args in K._SIGS.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = K._RESTYPES.get(name, ctypes.c_int)
    return lib


def _sched(lib):
    return getattr(lib, "sched", 0)


def main():
    libs = [bind(p) for p in sys.argv[1:]]
    # LIB_AB_IMPLS=0,2: the GEMM sched argument per library (the same .so may be listed twice)
    impls = [int(v) for v in os.environ.get("LIB_AB_IMPLS", "").split(",") if v]
    for lib, impl in zip(libs, impls):
        lib.sched = impl
    Mt, C, Vp = 65536, 768, 50432
    shapes = {"lm_head wgrad": (Vp, C), "qkv wgrad": (3 * C, C), "fc1 wgrad": (4 * C, C), "fc2 wgrad": (C, 4 * C),
              "proj wgrad": (C, C)}
    g = torch.Generator(device=dev).manual_seed(0)
    st = torch.cuda.current_stream().cuda_stream
    data = {}
    for name, (m, n) in shapes.items():
        A = (torch.randn(Mt, m, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        B = (torch.randn(Mt, n, device=dev, generator=g)).to(torch.bfloat16)
        sp = K.wgrad_splits(m, n, Mt)
        ws = torch.empty(max(sp * m * n, 4), device=dev)
        data[name] = (m, n, A, B, sp, ws)
    if os.environ.get("LIB_AB_OP") == "gemm":
        return gemm_mode(libs, g, st)
    if os.environ.get("LIB_AB_OP") == "attn":
        return attn_mode(libs, g, st)
    if os.environ.get("LIB_AB_OP") == "adamw":
        return adamw_mode(libs, g, st)
    if os.environ.get("LIB_AB_OP") == "xent":
        return xent_mode(libs, g, st)
    if os.environ.get("LIB_AB_OP") == "embed":
        return embed_mode(libs, g, st)
    outs = {}
    for i, lib in enumerate(libs):
        for name, (m, n, A, B, sp, ws) in data.items():
            Cm = torch.zeros(m, n, device=dev)
            rc = lib.gpt2mi_gemm_wgrad(m, n, Mt, A.data_ptr(), m, B.data_ptr(), n, Cm.data_ptr(), n, 0, 1.0, None,
                                       ws.data_ptr(), ws.numel(), sp, _sched(lib), st)
            assert rc == 0, (i, name, rc)
            outs[(i, name)] = Cm
    torch.cuda.synchronize()
    for name in shapes:
        for i in range(1, len(libs)):
            if not torch.equal(outs[(0, name)], outs[(i, name)]):
                d = (outs[(0, name)] - outs[(i, name)]).abs().max().item()
                print(f"MISMATCH lib{i} {name}: max diff {d}")
    times = {k: [] for k in outs}
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(5):
        for name, (m, n, A, B, sp, ws) in data.items():
            for i, lib in enumerate(libs):
                Cm = outs[(i, name)]
                fn = lambda: lib.gpt2mi_gemm_wgrad(m, n, Mt, A.data_ptr(), m, B.data_ptr(), n, Cm.data_ptr(), n, 1,  # noqa
                                                   1.0, None, ws.data_ptr(), ws.numel(), sp, _sched(lib), st)
                fn()
                s, e = ev(), ev()
                s.record()
                for _r in range(5):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[(i, name)].append(s.elapsed_time(e) / 5)
    for name, (m, n, *_r) in data.items():
        line = f"{name:14s}"
        for i in range(len(libs)):
            t = sorted(times[(i, name)])[2]
            line += f"  lib{i}: {t * 1e3:8.1f} us {2 * m * n * Mt / t / 1e9:6.0f} TF"
        print(line, flush=True)


def gemm_mode(libs, g, st):
    """LIB_AB_OP=gemm: forward / dgrad layouts (gpt2mi_gemm, BF16 epilogue) on the lm_head and K=768 shapes."""
    Mt, C, Vp = 65536, 768, 50432
    # name: (layout, N, K, epilogue); the fused-epilogue shapes run as in the step (bias, p = 0.1)
    shapes = {"lm_head fwd": (0, Vp, C, K.EPI_BF16), "lm_head dgrad": (1, C, Vp, K.EPI_BF16),
              "qkv fwd": (0, 3 * C, C, K.EPI_BF16), "fc1 dgrad": (1, C, 4 * C, K.EPI_BF16),
              "fc1 gelu": (0, 4 * C, C, K.EPI_GELU), "fc2dg gelubwd": (0, 4 * C, C, K.EPI_GELU_BWD),
              "proj resid": (0, C, C, K.EPI_RESID), "fc2 resid": (0, C, 4 * C, K.EPI_RESID),
              # the fc1 shape with cheaper epilogues: prices the GELU math and the dropout hash of "fc1 gelu"
              "fc1shape bf16": (0, 4 * C, C, K.EPI_BF16), "fc1shape gelu nodrop": (0, 4 * C, C, K.EPI_GELU)}
    if os.environ.get("GEMM_AB_SHAPES"):
        shapes = {k: v for k, v in shapes.items() if any(t in k for t in os.environ["GEMM_AB_SHAPES"].split(","))}
    data = {}
    for name, (lay, n, k, epi) in shapes.items():
        A = (torch.randn(Mt, k, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        B = (torch.randn(n, k, device=dev, generator=g) if lay == 0 else
             torch.randn(k, n, device=dev, generator=g)).to(torch.bfloat16)
        out = torch.empty(Mt, n, dtype=torch.float32 if epi == K.EPI_RESID else torch.bfloat16, device=dev)
        bias = torch.randn(n, device=dev, generator=g) if epi != K.EPI_BF16 else None
        resid = torch.randn(Mt, n, device=dev, generator=g) if epi == K.EPI_RESID else None
        aux = torch.randn(Mt, n, device=dev, generator=g).to(torch.bfloat16) if epi in (K.EPI_GELU, K.EPI_GELU_BWD) else None
        data[name] = (lay, n, k, A, B, out, epi, bias, resid, aux)
    # outputs of every library vs the first: C bitwise, the fused bias grad (atomics: any order) to 1e-5
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    for name, (lay, n, k, A, B, out, epi, bias, resid, aux) in data.items():
        ref = None
        for i, lib in enumerate(libs):
            o = torch.empty_like(out)
            db = torch.zeros(n, device=dev) if epi == K.EPI_GELU_BWD else None
            pd = 0.1 if epi in (K.EPI_GELU, K.EPI_RESID) and "nodrop" not in name else 0.0
            a2 = aux.clone() if aux is not None else None
            assert lib.gpt2mi_gemm(lay, epi, Mt, n, k, A.data_ptr(), k, B.data_ptr(), k if lay == 0 else n, o.data_ptr(),
                                   n, ptr(bias), ptr(resid), ptr(a2), n if aux is not None else 0, 1.0, None, 0, 1, pd,
                                   5, ptr(db), _sched(lib), st) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = (o, a2, db)
                continue
            if not torch.equal(o, ref[0]) or (a2 is not None and not torch.equal(a2, ref[1])):
                print(f"MISMATCH lib{i} {name}", flush=True)
            if db is not None and not torch.allclose(db, ref[2], rtol=1e-4, atol=1e-4 * ref[2].abs().max().item()):
                print(f"MISMATCH lib{i} {name} dbias: {(db - ref[2]).abs().max().item()}", flush=True)
    times = {(i, n): [] for i in range(len(libs)) for n in shapes}
    # LIB_AB_STAGGER="0;8000;6000,4": GPT2MI_PP_STAGGER per library ("<ns>[,<groups>]", read per call)
    stag = [v for v in os.environ.get("LIB_AB_STAGGER", "").split(";") if v]
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    dbs = {name: torch.zeros(v[1], device=dev) for name, v in data.items() if v[6] == K.EPI_GELU_BWD}
    # LIB_AB_HOG=<blocks>: every timed batch runs beside tools/ab/libhog.so's CU hog (that many CUs held for 3 ms on a
    # side stream, as RCCL kernels hold them in a data-parallel step)
    hog_blocks = int(os.environ.get("LIB_AB_HOG", "0"))
    if hog_blocks:
        hog = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab", "libhog.so"))
        hog.hog.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p]
        side = torch.cuda.Stream()
    for _ in range(5):
        for name, (lay, n, k, A, B, out, epi, bias, resid, aux) in data.items():
            ldb = k if lay == 0 else n
            pd = 0.1 if epi in (K.EPI_GELU, K.EPI_RESID) and "nodrop" not in name else 0.0
            for i, lib in enumerate(libs):
                if stag:
                    os.environ["GPT2MI_PP_STAGGER"] = stag[i]
                fn = lambda: lib.gpt2mi_gemm(lay, epi, Mt, n, k, A.data_ptr(), k, B.data_ptr(), ldb,  # noqa: E731
                                             out.data_ptr(), n, ptr(bias), ptr(resid), ptr(aux), n if aux is not None else 0,
                                             1.0, None, 0, 1, pd, 5, ptr(dbs.get(name)), _sched(lib), st)
                assert fn() == 0
                s, e = ev(), ev()
                if hog_blocks:
                    torch.cuda.synchronize()
                    assert hog.hog(hog_blocks, 3_000_000, side.cuda_stream) == 0
                s.record()
                for _r in range(5):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[(i, name)].append(s.elapsed_time(e) / 5)
    for name, (lay, n, k, *_r) in data.items():
        line = f"{name:15s}"
        for i in range(len(libs)):
            t = sorted(times[(i, name)])[2]
            line += f"  lib{i}: {t * 1e3:8.1f} us {2 * n * k * Mt / t / 1e9:6.0f} TF"
        print(line, flush=True)


def attn_mode(libs, g, st):
    """LIB_AB_OP=attn: attention forward / backward at cfg 2 (B=64, T=1024, H=12, D=64, dropout 0.1); outputs
    compared bitwise against the first library."""
    B, T, H, D = 64, 1024, 12, 64
    C = H * D
    pd = float(os.environ.get("LIB_AB_PDROP", "0.1"))
    qkv = (torch.randn(B * T, 3 * C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dout = (torch.randn(B * T, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    res = []
    for lib in libs:
        out = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * H * T, device=dev)
        delta = torch.empty(B * H * T, device=dev)
        dqkv = torch.empty(B * T, 3 * C, dtype=torch.bfloat16, device=dev)
        res.append((out, lse, delta, dqkv))
    fwd = lambda lib, r: lib.gpt2mi_attn_fwd(qkv.data_ptr(), r[0].data_ptr(), r[1].data_ptr(), B, T, H, D, pd,  # noqa
                                              7, st)
    bwd = lambda lib, r: lib.gpt2mi_attn_bwd(qkv.data_ptr(), r[0].data_ptr(), dout.data_ptr(), r[1].data_ptr(),  # noqa
                                              r[2].data_ptr(), r[3].data_ptr(), None, B, T, H, D, pd, 7, st)
    for lib, r in zip(libs, res):
        assert fwd(lib, r) == 0 and bwd(lib, r) == 0
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        for k, name in enumerate(("out", "lse", "delta", "dqkv")):
            if not torch.equal(res[0][k], res[i][k]):
                print(f"MISMATCH lib{i} {name}")
    times = {(i, n): [] for i in range(len(libs)) for n in ("fwd", "bwd")}
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(5):
        for i, (lib, r) in enumerate(zip(libs, res)):
            for n, fn in (("fwd", fwd), ("bwd", bwd)):
                s, e = ev(), ev()
                s.record()
                for _r in range(10):
                    fn(lib, r)
                e.record()
                torch.cuda.synchronize()
                times[(i, n)].append(s.elapsed_time(e) / 10)
    for n in ("fwd", "bwd"):
        line = f"attn {n:10s}"
        for i in range(len(libs)):
            line += f"  lib{i}: {sorted(times[(i, n)])[2] * 1e3:8.1f} us"
        print(line, flush=True)



def adamw_mode(libs, g, st):
    """LIB_AB_OP=adamw: the fused AdamW over the 124M arena (with the bf16 shadow and the grad-norm partials);
    parameters / moments / shadow compared bitwise against the first library after one step."""
    n = 124_475_904
    p0 = torch.randn(n, device=dev, generator=g)
    gr = torch.randn(n, device=dev, generator=g) * 1e-3
    res = []
    for lib in libs:
        p, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
        part = torch.empty(4096, device=dev)
        gn = torch.empty(1, device=dev)
        res.append((p, m, v, pb, part, gn))
    step = lambda lib, r: lib.gpt2mi_adamw(r[0].data_ptr(), gr.data_ptr(), r[1].data_ptr(), r[2].data_ptr(),  # noqa
                                           r[3].data_ptr(), n, 1e-4, 0.1, 0.9, 0.95, 1e-8, 1, 1.0, r[4].data_ptr(),
                                           r[5].data_ptr(), st)
    for lib, r in zip(libs, res):
        assert step(lib, r) == 0
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        for k, name in enumerate(("p", "m", "v", "shadow")):
            if not torch.equal(res[0][k], res[i][k]):
                print(f"MISMATCH lib{i} {name}")
        print(f"grad norm lib0 {res[0][5].item():.7g} lib{i} {res[i][5].item():.7g}")
    times = {i: [] for i in range(len(libs))}
    for _ in range(5):
        for i, (lib, r) in enumerate(zip(libs, res)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _r in range(5):
                step(lib, r)
            e.record()
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / 5)
    print("adamw " + "  ".join(f"lib{i}: {sorted(t)[2] * 1e3:8.1f} us" for i, t in times.items()), flush=True)


def xent_mode(libs, g, st):
    """LIB_AB_OP=xent: the register-resident cross-entropy (loss rows, lse, bf16 dlogits) at cfg 2's head
    (65536 rows of 50257 logits, row stride 50304); outputs compared bitwise against the first library."""
    M, V, ld = 65536, 50257, 50304
    logits = (torch.randn(M, ld, device=dev, generator=g) * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (M,), device=dev, generator=g)
    labels[::97] = -100
    res = []
    for lib in libs:
        res.append((torch.empty(M, device=dev), torch.empty(M, device=dev), torch.empty_like(logits),
                    torch.empty(1, device=dev), torch.empty(1, device=dev)))
    run = lambda lib, r: lib.gpt2mi_xent_fwd(logits.data_ptr(), ld, labels.data_ptr(), r[0].data_ptr(),  # noqa
                                             r[1].data_ptr(), r[2].data_ptr(), ld, M, V, -100, r[3].data_ptr(),
                                             r[4].data_ptr(), st)
    for lib, r in zip(libs, res):
        assert run(lib, r) == 0
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        for k, name in enumerate(("loss_rows", "lse", "dlogits", "loss")):
            if not torch.equal(res[0][k], res[i][k]):
                print(f"MISMATCH lib{i} {name}")
    times = {i: [] for i in range(len(libs))}
    for _ in range(5):
        for i, (lib, r) in enumerate(zip(libs, res)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _r in range(5):
                run(lib, r)
            e.record()
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / 5)
    gb = 2 * 2 * M * ld / 1e9
    print("xent " + "  ".join(f"lib{i}: {sorted(t)[2] * 1e3:8.1f} us {gb / sorted(t)[2]:5.2f} TB/s"
                              for i, t in times.items()), flush=True)


def embed_mode(libs, g, st):
    """LIB_AB_OP=embed: the embedding backward at cfg 2 (B=64, T=1024, C=768, dropout 0.1): dwpe compared bitwise
    against the first library, dwte (fp32 atomics, any order) to 1e-5."""
    B, T, C, V = 64, 1024, 768, 50257
    idx = torch.randint(0, V, (B * T,), device=dev, generator=g)
    dres = torch.randn(B * T, C, device=dev, generator=g)
    res = [(torch.zeros(V, C, device=dev), torch.zeros(T, C, device=dev)) for _ in libs]
    run = lambda lib, r: lib.gpt2mi_embed_bwd(idx.data_ptr(), dres.data_ptr(), r[0].data_ptr(), r[1].data_ptr(),  # noqa
                                              B, T, T, C, 0.1, 77, st)
    for lib, r in zip(libs, res):
        assert run(lib, r) == 0
    torch.cuda.synchronize()
    for i in range(1, len(libs)):
        if not torch.equal(res[0][1], res[i][1]):
            print(f"MISMATCH lib{i} dwpe")
        if not torch.allclose(res[0][0], res[i][0], rtol=1e-5, atol=1e-6):
            print(f"MISMATCH lib{i} dwte {(res[0][0] - res[i][0]).abs().max().item()}")
    times = {i: [] for i in range(len(libs))}
    for _ in range(5):
        for i, (lib, r) in enumerate(zip(libs, res)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _r in range(5):
                run(lib, r)
            e.record()
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / 5)
    print("embed_bwd " + "  ".join(f"lib{i}: {sorted(t)[2] * 1e3:8.1f} us" for i, t in times.items()), flush=True)


if __name__ == "__main__":
    main()
