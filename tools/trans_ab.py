"""A/B of the 256x256 ping-pong GEMM on k-contiguous vs m-contiguous (transposed, the weight-gradient layout)
operands at one shape: C[M,N] fp32 = A.B^T over K, 3 rounds of 256 tiles, no split-K, so the two differ only in
the operand layout (ds_read_b128 vs ds_read_b64_tr_b16 fragments). Interleaved rounds, HIP events.

    python tools/trans_ab.py [K]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    Kd = int(sys.argv[1]) if len(sys.argv) > 1 else 21824
    M, N = 65536, 768
    a_kc = (torch.randn(M, Kd, device=dev) * 0.5).to(torch.bfloat16)
    b_kc = (torch.randn(N, Kd, device=dev) * 0.5).to(torch.bfloat16)
    a_mc = a_kc.t().contiguous()
    b_mc = b_kc.t().contiguous()
    c1 = torch.empty(M, N, device=dev)
    c2 = torch.empty(M, N, device=dev)
    fl = 2.0 * M * N * Kd
    kc = lambda: K.gemm(K.FWD, K.EPI_F32, M, N, Kd, a_kc, Kd, b_kc, Kd, c1, N)  # noqa: E731
    mc = lambda: K.gemm_wgrad(M, N, Kd, a_mc, M, b_mc, N, c2, N, accumulate=False, splits=1)  # noqa: E731
    # one operand transposed (layout 1: A k-contiguous, B m-contiguous)
    c3 = torch.empty(M, N, device=dev)
    kb = lambda: K.gemm(1, K.EPI_F32, M, N, Kd, a_kc, Kd, b_mc, N, c3, N)  # noqa: E731
    res = {"kc": [], "mc": [], "kc_a_mc_b": []}
    for _ in range(4):
        res["kc"].append(timeit(kc))
        res["mc"].append(timeit(mc))
        res["kc_a_mc_b"].append(timeit(kb))
    torch.cuda.synchronize()
    err = max((c1 - c2).abs().max().item(), (c1 - c3).abs().max().item())
    for k, v in res.items():
        best = min(v)
        print(f"{k}: {' '.join(f'{x:.3f}' for x in v)} ms  best {fl / best / 1e9:.0f} TF/s ({fl / best / 1e9 / 2516.6:.1%})")
    print(f"max |kc - mc| = {err:.3e}")


if __name__ == "__main__":
    main()
