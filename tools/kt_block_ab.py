"""The block weight gradients (qkv, proj, fc1, fc2 at cfg 2: 65 536 tokens) in the two operand layouts, HIP events:
  both token-major (the step's form: gemm_wgrad, dW = dY^T . X, both operands read by ds_read_b64_tr_b16) against
  the transposed-X form (gemm_wgrad_kt: X^T staged once, dW^T = X^T . dY in layout 1, transposing split-K reduce),
  timed with and without the transpose of X (a producer that writes X^T itself would pay only its extra stores).

    python tools/kt_block_ab.py
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
    return s.elapsed_time(e) / reps * 1e3


def main():
    Mt, C = 65536, 768
    shapes = {"qkv": (3 * C, C), "proj": (C, C), "fc1": (4 * C, C), "fc2": (C, 4 * C)}
    for name, (M, N) in shapes.items():
        dy = (torch.randn(Mt, M, device=dev) * 0.01).to(torch.bfloat16)
        x = torch.randn(Mt, N, device=dev).to(torch.bfloat16)
        xt = torch.empty(N, Mt, device=dev, dtype=torch.bfloat16)
        s = K.wgrad_splits(M, N, Mt)
        ws = torch.empty(s * M * N + 4096, device=dev)
        w1 = torch.zeros(M, N, device=dev)
        w2 = torch.zeros(M, N, device=dev)
        both = lambda: K.gemm_wgrad(M, N, Mt, dy, M, x, N, w1, N, accumulate=False, workspace=ws, splits=s)  # noqa
        tr = lambda: K.transpose_bf16(x, xt, Mt, N)  # noqa: E731
        kt = lambda: K.gemm_wgrad_kt(M, N, Mt, dy, M, xt, Mt, w2, N, accumulate=False, workspace=ws, splits=s)  # noqa

        def kt_tr():
            tr()
            kt()

        res = {"both token-major": [], "transpose + kt": [], "kt only": [], "transpose only": []}
        for _ in range(4):
            res["both token-major"].append(timeit(both))
            res["transpose + kt"].append(timeit(kt_tr))
            res["kt only"].append(timeit(kt))
            res["transpose only"].append(timeit(tr))
        torch.cuda.synchronize()
        both()
        kt_tr()
        torch.cuda.synchronize()
        same = torch.equal(w1, w2)
        fl = 2.0 * M * N * Mt
        print(f"{name}: M={M} N={N} splits={s} same bits: {same}")
        for k, v in res.items():
            b = min(v)
            tf = f"{fl / b / 1e6:.0f} TF/s" if k != "transpose only" else ""
            print(f"  {k:18s}: {' '.join(f'{t:.1f}' for t in v)} us  best {b:.1f} {tf}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
