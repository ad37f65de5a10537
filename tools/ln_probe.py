"""LayerNorm backward at cfg 2 (M = 65536, C = 768, bf16 dy, dropout 0.1 on the emitted branch grad): the full
call (LN param grads + the next branch's bias grad, column sums reduced by one atomic per column per block) against
the same call without those column-sum outputs, to price the reduction.

    python tools/ln_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"


def main(M=65536, C=768):
    libs = os.environ.get("LN_LIBS")
    if libs:  # A/B of library builds: the full call in each, interleaved
        return ab(libs.split(","), M, C)
    x = torch.randn(M, C, device=dev)
    w = torch.randn(C, device=dev)
    mean, rstd = torch.randn(M, device=dev), torch.rand(M, device=dev) + 0.5
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, C, device=dev)
    dw, db, dbo = (torch.zeros(C, device=dev) for _ in range(3))
    ob = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    cases = {"full": (dw, db, dbo), "no dbias_out": (dw, db, None), "no column sums": (None, None, None)}
    t = {k: [] for k in cases}
    for _ in range(5):
        for k, (a, b, c) in cases.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _r in range(10):
                K.layernorm_bwd(x, w, mean, rstd, dy, dres, a, b, ob, c, M, C, 0.1, 7)
            e.record()
            torch.cuda.synchronize()
            t[k].append(s.elapsed_time(e) / 10 * 1e3)
    print("ln_bwd " + "  ".join(f"{k}: {sorted(v)[2]:.1f} us" for k, v in t.items()), flush=True)


def ab(paths, M, C):
    import ctypes
    libs = []
    for path in paths:
        lib = ctypes.CDLL(path)
        lib.gpt2mi_layernorm_bwd.argtypes = K._SIGS["gpt2mi_layernorm_bwd"]
        libs.append(lib)
    x = torch.randn(M, C, device=dev)
    w = torch.randn(C, device=dev)
    mean, rstd = torch.randn(M, device=dev), torch.rand(M, device=dev) + 0.5
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, C, device=dev)
    dw, db, dbo = (torch.zeros(C, device=dev) for _ in range(3))
    ob = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    t = {i: [] for i in range(len(libs))}
    for _ in range(5):
        for i, lib in enumerate(libs):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _r in range(10):
                lib.gpt2mi_layernorm_bwd(x.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(), dy.data_ptr(),
                                         dres.data_ptr(), dw.data_ptr(), db.data_ptr(), ob.data_ptr(), dbo.data_ptr(),
                                         M, C, 0.1, 7, 0, st)
            e.record()
            torch.cuda.synchronize()
            t[i].append(s.elapsed_time(e) / 10 * 1e3)
    print("ln_bwd " + "  ".join(f"lib{i}: {sorted(v)[2]:.1f} us" for i, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
