"""Launch ONE of bench.py's probed kernels a few times on step-shaped inputs (GPT-2 124M, B=64, T=1024,
dropout 0.1), for the rocprofv3 --pmc traffic passes (tools/pmc_traffic.sh -> profiles/traffic.json).

    python tools/kernel_one.py <lm_head_fwd|lm_head_dgrad|lm_head_wgrad|fc1_fwd|proj_fwd|fc2_fwd|qkv_fwd|fc2_dgrad|
                                attn_fwd|attn_bwd|wgrad> [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
# the weight gradients as the engine launches them under autocast: fp32 split-K slabs since round 4
# (Engine.WGRAD_BF16_SLABS = False; KERNEL_ONE_BF16_SLABS=1: the opt-in bf16 slabs)
SLABS = K.SCHED_BF16_SLABS if os.environ.get("KERNEL_ONE_BF16_SLABS") == "1" else 0
M, C, Vp, V, B, T, H = 65536, 768, 50432, 50257, 64, 1024, 12


def r(*s):
    return (torch.randn(*s, device=dev) * 0.5).to(torch.bfloat16)


def make(name):
    if name == "lm_head_fwd":
        a, w, out = r(M, C), r(Vp, C), torch.empty(M, Vp, dtype=torch.bfloat16, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_BF16, M, Vp, C, a, C, w, C, out, Vp)
    if name == "lm_head_dgrad":  # forward layout against the transposed wte shadow
        dl, wt, out = r(M, Vp), r(C, Vp), torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_BF16, M, C, Vp, dl, Vp, wt, Vp, out, C)
    if name in ("lm_head_wgrad", "lm_head_wgrad_kt"):  # the step's form: lnf transposed once, gpt2mi_gemm_wgrad_kt
        dl, x, g = r(M, Vp), r(M, C), torch.zeros(Vp, C, device=dev)
        xt = torch.empty(C, M, dtype=torch.bfloat16, device=dev)
        sp = K.wgrad_splits(Vp, C, M)
        ws = torch.empty(sp * Vp * C, device=dev)

        def run():
            K.transpose_bf16(x, xt, M, C, C, M)
            K.gemm_wgrad_kt(Vp, C, M, dl, Vp, xt, M, g, C, workspace=ws, splits=sp, sched=SLABS)
        return run
    if name == "lm_head_wgrad_old":
        dl, x, g = r(M, Vp), r(M, C), torch.zeros(Vp, C, device=dev)
        sp = K.wgrad_splits(Vp, C, M)
        ws = torch.empty(sp * Vp * C, device=dev)
        return lambda: K.gemm_wgrad(Vp, C, M, dl, Vp, x, C, g, C, workspace=ws, splits=sp, sched=SLABS)
    if name == "fc1_fwd":
        a, w = r(M, C), r(4 * C, C)
        bias = torch.zeros(4 * C, device=dev)
        h, dg = (torch.empty(M, 4 * C, dtype=torch.bfloat16, device=dev) for _ in range(2))
        return lambda: K.gemm(K.FWD, K.EPI_GELU, M, 4 * C, C, a, C, w, C, h, 4 * C, bias=bias, aux=dg, ldaux=4 * C,
                              p_drop=0.1, seed=3)
    if name == "proj_fwd":  # fp32 residual + dropout epilogue, K = 768
        a, w, res = r(M, C), r(C, C), torch.randn(M, C, device=dev)
        bias, out = torch.zeros(C, device=dev), torch.empty(M, C, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_RESID, M, C, C, a, C, w, C, out, C, bias=bias, resid=res, p_drop=0.1, seed=4)
    if name == "fc2_fwd":  # fp32 residual + dropout epilogue, K = 3072
        a, w, res = r(M, 4 * C), r(C, 4 * C), torch.randn(M, C, device=dev)
        bias, out = torch.zeros(C, device=dev), torch.empty(M, C, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_RESID, M, C, 4 * C, a, 4 * C, w, 4 * C, out, C, bias=bias, resid=res,
                              p_drop=0.1, seed=4)
    if name == "qkv_fwd":
        a, w, bias = r(M, C), r(3 * C, C), torch.zeros(3 * C, device=dev)
        out = torch.empty(M, 3 * C, dtype=torch.bfloat16, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_BF16, M, 3 * C, C, a, C, w, C, out, 3 * C, bias=bias)
    if name == "fc2_dgrad":  # GELU-derivative epilogue + fused fc1 bias grad (forward layout against W^T)
        dy, wt, dg = r(M, C), r(4 * C, C), r(M, 4 * C)
        out, db = torch.empty(M, 4 * C, dtype=torch.bfloat16, device=dev), torch.zeros(4 * C, device=dev)
        return lambda: K.gemm(K.FWD, K.EPI_GELU_BWD, M, 4 * C, C, dy, C, wt, C, out, 4 * C, aux=dg, ldaux=4 * C,
                              dbias=db)
    if name == "attn_fwd":
        qkv, out = r(M, 3 * C), torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B * H, T, device=dev)
        p = float(os.environ.get("ATTN_P", "0.1"))
        return lambda: K.attn_fwd(qkv, out, lse, B, T, H, C // H, p, 5)
    if name == "attn_bwd":  # dQ (+ delta) then dK/dV
        qkv, out, dout = r(M, 3 * C), r(M, C), r(M, C)
        lse = torch.randn(B * H, T, device=dev).abs() + 5.0
        delta = torch.empty(B * H, T, device=dev)
        dqkv = torch.empty(M, 3 * C, dtype=torch.bfloat16, device=dev)
        p = float(os.environ.get("ATTN_P", "0.1"))
        return lambda: K.attn_bwd(qkv, out, dout, lse, delta, dqkv, B, T, H, C // H, p, 5)
    if name == "wgrad":  # one step's weight gradients: 12 x (fc2 + fc1, proj + qkv grouped) + the tied lm_head
        pairs = [[(C, 4 * C), (4 * C, C)], [(C, C), (3 * C, C)]]  # as Engine._block_bwd groups them (round 6)
        shapes = [sh for pr in pairs for sh in pr] + [(Vp, C)]
        ops = {(m, n): (r(M, m), r(M, n), torch.zeros(m, n, device=dev)) for m, n in set(shapes)}
        ws = torch.empty(max([K.wgrad_splits(Vp, C, M) * Vp * C] +
                             [K.wgrad_group_splits(pr, M) * sum(m * n for m, n in pr) for pr in pairs]), device=dev)
        xt = torch.empty(C, M, dtype=torch.bfloat16, device=dev)
        grouped = not SLABS  # the opt-in bf16 slabs keep the four launches

        def run():  # the lm_head as the step runs it: lnf transposed, gpt2mi_gemm_wgrad_kt
            a, x, g = ops[(Vp, C)]
            K.transpose_bf16(x, xt, M, C, C, M)
            K.gemm_wgrad_kt(Vp, C, M, a, Vp, xt, M, g, C, workspace=ws, splits=K.wgrad_splits(Vp, C, M), sched=SLABS)
            for _ in range(12):
                for pr in pairs:
                    if grouped:
                        K.gemm_wgrad_grouped([(m, n, ops[(m, n)][0], m, ops[(m, n)][1], n, ops[(m, n)][2])
                                              for m, n in pr], M, workspace=ws, splits=K.wgrad_group_splits(pr, M))
                    else:
                        for m, n in pr:
                            a, x, g = ops[(m, n)]
                            K.gemm_wgrad(m, n, M, a, m, x, n, g, n, workspace=ws, splits=K.wgrad_splits(m, n, M),
                                         sched=SLABS)
        return run
    raise SystemExit(f"unknown kernel {name}")


if __name__ == "__main__":
    K.load()
    fn = make(sys.argv[1])
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
        fn()
    torch.cuda.synchronize()
