"""The lm_head weight-gradient K-range of one split (65536 / 3 tokens) in its two operand layouts, HIP events:
  both m-contiguous (the step's form: dW[Vp][C] = dlogits^T . lnf, A = dlogits [K][Vp], B = lnf [K][C]) against
  one k-contiguous (dW^T[C][Vp] = lnf^T . dlogits: A = lnf^T [C][K] k-contiguous, B = dlogits [K][Vp]).

    python tools/lmwg_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"


def timeit(fn, reps=5):
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
    Vp, C, Kd = 50432, 768, 21824
    dl = (torch.randn(Kd, Vp, device=dev) * 0.01).to(torch.bfloat16)
    x = (torch.randn(Kd, C, device=dev)).to(torch.bfloat16)
    xt = x.t().contiguous()
    w1 = torch.empty(Vp, C, device=dev)
    w2 = torch.empty(C, Vp, device=dev)
    fl = 2.0 * Vp * C * Kd
    both = lambda: K.gemm_wgrad(Vp, C, Kd, dl, Vp, x, C, w1, C, accumulate=False, splits=1)  # noqa: E731
    one = lambda: K.gemm(1, K.EPI_F32, C, Vp, Kd, xt, Kd, dl, Vp, w2, Vp)  # noqa: E731
    res = {"both m-contiguous": [], "A k-contiguous": []}
    for _ in range(4):
        res["both m-contiguous"].append(timeit(both))
        res["A k-contiguous"].append(timeit(one))
    torch.cuda.synchronize()
    err = (w1 - w2.t()).abs().max().item()
    for k, v in res.items():
        b = min(v)
        print(f"{k:18s}: {' '.join(f'{t:.3f}' for t in v)} ms  best {fl / b / 1e9:.0f} TF/s")
    print(f"max |dW - (dW^T)^T| = {err:.3e}")


if __name__ == "__main__":
    main()
