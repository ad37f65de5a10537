"""GEMM A/B probe on the MI355X: interleaved rounds of each kernel implementation on the same random
operands, one process (cdna_hip_programming.md §5.4 rule 24). Shapes: square 8192^3 (the guide's
reference point) and the GPT-2 step's extreme shapes.

    python tools/gemm_probe.py [impl,impl,...] [shape names]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
SHAPES = {
    # name: (layout, epilogue, M, N, K)
    "sq8k_fwd": (0, K.EPI_BF16, 8192, 8192, 8192),
    "sq8k_dgrad": (1, K.EPI_BF16, 8192, 8192, 8192),
    "lm_fwd": (0, K.EPI_BF16, 65536, 50432, 768),
    "lm_dgrad": (1, K.EPI_BF16, 65536, 768, 50432),
    "fc1_gelu": (0, K.EPI_GELU, 65536, 3072, 768),
    "fc2_resid": (0, K.EPI_RESID, 65536, 768, 3072),
    "qkv_fwd": (0, K.EPI_BF16, 65536, 2304, 768),
    "fc2_dgelu": (1, K.EPI_GELU_BWD, 65536, 3072, 768),
    "fc1_dgrad": (1, K.EPI_BF16, 65536, 768, 3072),
    # dgrads as the step runs them (forward layout against the transposed weight shadow)
    "fc2_dgelu0": (0, K.EPI_GELU_BWD, 65536, 3072, 768),
    "proj_dgrad0": (0, K.EPI_BF16, 65536, 768, 768),
    "qkv_dgrad0": (0, K.EPI_BF16, 65536, 768, 2304),
    "proj_resid": (0, K.EPI_RESID, 65536, 768, 768),
    # weight gradients (layout 2 through gemm_wgrad: split-K slabs + deterministic reduce)
    "lm_wgrad": (2, K.EPI_F32, 50432, 768, 65536),
    "fc1_wgrad": (2, K.EPI_F32, 3072, 768, 65536),
    "qkv_wgrad": (2, K.EPI_F32, 2304, 768, 65536),
    "proj_wgrad": (2, K.EPI_F32, 768, 768, 65536),
    "sq8k_wgrad": (2, K.EPI_F32, 8192, 8192, 8192),
    # per-tile fixed cost: the same 2304 x 65536 output at three depths
    "qkv_k768": (0, K.EPI_BF16, 65536, 2304, 768),
    "qkv_k1536": (0, K.EPI_BF16, 65536, 2304, 1536),
    "qkv_k3072": (0, K.EPI_BF16, 65536, 2304, 3072),
    "qkv_k768_f32": (0, K.EPI_F32, 65536, 2304, 768),
    # per-tile fixed cost on the lm_head width: the same 65536 x 50432 output at three depths
    "lm_k128": (0, K.EPI_BF16, 65536, 50432, 128),
    "lm_k256": (0, K.EPI_BF16, 65536, 50432, 256),
    "lm_k512": (0, K.EPI_BF16, 65536, 50432, 512),
}


def make(layout, epi, M, N, Kd, sched=0):
    if layout == 2:
        A = (torch.rand(Kd, M, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(Kd, N, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.zeros(M, N, device=dev)
        sp = K.wgrad_splits(M, N, Kd)
        ws = torch.empty(max(4, sp * M * N if sp > 1 else 4), device=dev)
        return lambda: K.gemm_wgrad(M, N, Kd, A, M, B, N, C, N, workspace=ws, splits=sp, sched=sched)
    A = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16) if layout == 0 else \
        (torch.rand(Kd, N, device=dev) * 2 - 1).to(torch.bfloat16)
    f32 = epi in (K.EPI_F32, K.EPI_RESID)
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    bias = torch.zeros(N, device=dev) if layout == 0 else None
    resid = torch.zeros(M, N, device=dev) if epi == K.EPI_RESID else None
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi in (K.EPI_GELU, K.EPI_GELU_BWD) else None
    ldb = Kd if layout == 0 else N
    return lambda: K.gemm(layout, epi, M, N, Kd, A, Kd, B, ldb, C, N, bias=bias, resid=resid, aux=aux, ldaux=N,
                          sched=sched)


def main():
    impls = [0, 2]
    names = []
    for a in sys.argv[1:]:
        if a[0].isdigit():
            impls = [int(x) for x in a.split(",")]
        else:
            names.append(a)
    names = names or list(SHAPES)
    K.load()
    for name in names:
        layout, epi, M, N, Kd = SHAPES[name]
        fns = {i: make(layout, epi, M, N, Kd, sched=i) for i in impls}
        flop = 2.0 * M * N * Kd
        reps = max(3, int(2e13 / flop))
        res = {i: [] for i in impls}
        for rnd in range(5):
            for i in impls:
                fn = fns[i]
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[i].append(s.elapsed_time(e) / reps)
        line = f"{name:11s} M={M} N={N} K={Kd}:"
        for i in impls:
            ms = sorted(res[i])[len(res[i]) // 2]
            line += f"  impl{i} {ms:7.3f} ms {flop / ms / 1e9:6.0f} TF"
        print(line, flush=True)




def hipblaslt_reference():
    """torch.matmul (hipBLASLt) on the lm_head shapes, same random data style (reference points only)."""
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    cases = {
        "lm_fwd": (lambda a, b: a @ b.t(), r(65536, 768), r(50432, 768)),
        "lm_dgrad": (lambda a, b: a @ b, r(65536, 50432), r(50432, 768)),
        "lm_wgrad": (lambda a, b: a.t() @ b, r(65536, 50432), r(65536, 768)),
    }
    for name, (f, a, b) in cases.items():
        f(a, b)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            f(a, b)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        print(f"[hipBLASLt] {name}: {ms:.3f} ms {2 * 65536 * 50432 * 768 / ms / 1e9:.0f} TF", flush=True)
        del a, b


if __name__ == "__main__":
    if "blaslt" in sys.argv[1:]:
        K.load()
        hipblaslt_reference()
    else:
        main()
