#!/usr/bin/env python
"""Numerics of the GELU_BWD epilogue variants at the fc2 dgrad shape (M = 65536, N = 3072, K = 768): each library's
output and fused bias gradient against a float64 reference of bf16(round_bf16(dY . W) * derivative) (the rounding
the reference's autocast dgrad applies before the GELU backward), and against the product library.

    python tools/aux_check.py tools/ab/lib_base.so tools/ab/lib_auxlds.so
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lib_ab import bind  # noqa: E402

dev = "cuda"


def main():
    libs = [bind(p) for p in sys.argv[1:]]
    M, N, K = 65536, 3072, 768
    g = torch.Generator(device=dev).manual_seed(3)
    A = (torch.randn(M, K, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    aux = (torch.rand(M, N, device=dev, generator=g) * 1.2).to(torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    y = A.double() @ B.double().t()
    ref_r = (y.to(torch.bfloat16).double() * aux.double())  # rounded dgrad output first (autocast)
    ref_u = (y * aux.double())
    outs = []
    for i, lib in enumerate(libs):
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        db = torch.zeros(N, device=dev)
        assert lib.gpt2mi_gemm(0, 4, M, N, K, A.data_ptr(), K, B.data_ptr(), K, o.data_ptr(), N, None, None,
                               aux.data_ptr(), N, 1.0, None, 0, 1, 0.0, 5, db.data_ptr(), 0, st) == 0
        torch.cuda.synchronize()
        od = o.double()
        scale = ref_u.abs().max().item()
        e_r = ((od - ref_r).abs().max().item()) / scale
        e_u = ((od - ref_u).abs().max().item()) / scale
        rel_r = ((od - ref_r).abs() / ref_r.abs().clamp_min(1e-30)).max().item()
        dbr = od.sum(0)
        print(f"lib{i}: max|o - bf16-rounded ref| / max|ref| {e_r:.2e} (elementwise rel {rel_r:.2e}), vs unrounded "
              f"{e_u:.2e}; fused dbias vs column sums of o: {((db.double() - dbr).abs().max() / dbr.abs().max()).item():.2e}",
              flush=True)
        outs.append(o)
    for i in range(1, len(outs)):
        d = (outs[i].double() - outs[0].double()).abs()
        print(f"lib{i} vs lib0: {int((d > 0).sum().item())} of {M * N} elements differ, max {d.max().item():.3e}",
              flush=True)


if __name__ == "__main__":
    main()
