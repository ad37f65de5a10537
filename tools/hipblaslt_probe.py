"""Reference point, not product code: torch (hipBLASLt) on the step's plain GEMM shapes, HIP-event timed,
next to the same shapes through libgpt2mi. Run under rocprofv3 --kernel-trace to see hipBLASLt's kernel names.

    python tools/hipblaslt_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
M, C, Vp = 65536, 768, 50432


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def r(*s):
    return (torch.randn(*s, device=dev) * 0.5).to(torch.bfloat16)


K.load()
# (name, M, N, K): out[M,N] = A[M,K] . W[N,K]^T   (forward layout; dgrads run against the transposed shadow)
shapes = [("lm_head fwd", M, Vp, C), ("qkv fwd", M, 3 * C, C), ("fc1 fwd (plain)", M, 4 * C, C),
          ("proj fwd (plain)", M, C, C), ("lm dgrad", M, C, Vp), ("qkv dgrad", M, C, 3 * C),
          ("fc1 dgrad", M, C, 4 * C)]
for name, m, n, k in shapes:
    a, w = r(m, k), r(n, k)
    out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
    t_blt = timeit(lambda: torch.mm(a, w.t(), out=out))
    t_own = timeit(lambda: K.gemm(K.FWD, K.EPI_BF16, m, n, k, a, k, w, k, out, n))
    f = 2.0 * m * n * k
    print(f"{name:18s} hipBLASLt {t_blt:7.3f} ms {f / t_blt / 1e9:6.0f} TF | libgpt2mi {t_own:7.3f} ms {f / t_own / 1e9:6.0f} TF")
    del a, w, out

# weight gradients dW[m_out, n_in] = dY^T . X over K = M tokens (both operands token-major: the transposed layout)
for name, mo, ni in (("lm_head wgrad", Vp, C), ("qkv wgrad", 3 * C, C), ("fc1 wgrad", 4 * C, C), ("fc2 wgrad", C, 4 * C)):
    dy, x = r(M, mo), r(M, ni)
    out = torch.empty(mo, ni, dtype=torch.bfloat16, device=dev)
    t_blt = timeit(lambda: torch.mm(dy.t(), x, out=out))
    sp = K.wgrad_splits(mo, ni, M)
    ws = torch.empty(sp * mo * ni, device=dev)
    acc = torch.zeros(mo, ni, device=dev)
    t_own = timeit(lambda: K.gemm_wgrad(mo, ni, M, dy, mo, x, ni, acc, ni, True, 1.0, None, ws, sp))
    f = 2.0 * M * mo * ni
    print(f"{name:18s} hipBLASLt {t_blt:7.3f} ms {f / t_blt / 1e9:6.0f} TF | libgpt2mi {t_own:7.3f} ms {f / t_own / 1e9:6.0f} TF")
    del dy, x, out, ws, acc
