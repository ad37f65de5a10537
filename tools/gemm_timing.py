"""Per-block phase timing of the ping-pong GEMM (s_memtime stamps; see PP_STAMP in gemm_pp.hip).

    make -C gpt_2_distributed_amd/csrc timing   # builds tools/ab/lib_timing.so with -DGEMM_PP_TIMING
    GPT2MI_LIB=tools/ab/lib_timing.so python tools/gemm_timing.py [M N K]

Prints, in s_memtime ticks and us (at the measured tick rate), the average prologue (first operands
landed), main loop, epilogue, and the gap between consecutive blocks on one CU."""
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd import _lib as K  # noqa: E402

dev = "cuda"
M, N, Kd = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (65536, 50432, 768)
K.load()
A = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
nblk = (M // 256) * (N // 256)
ts = torch.zeros(nblk * 6, dtype=torch.int64, device=dev)
for _ in range(3):
    K.gemm(0, K.EPI_BF16, M, N, Kd, A, Kd, B, Kd, C, N, aux=ts, ldaux=N)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
K.gemm(0, K.EPI_BF16, M, N, Kd, A, Kd, B, Kd, C, N, aux=ts, ldaux=N)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1)
t = ts.view(nblk, 6).cpu().tolist()
# s_memtime is per-XCD (not synchronized across XCDs): calibrate the tick on each XCD's span ~ the kernel
by_xcc = defaultdict(list)
for r in t:
    by_xcc[r[5] & 0xF].append(r)
spans = {x: max(r[3] for r in v) - min(r[0] for r in v) for x, v in by_xcc.items()}
rate = sum(spans.values()) / len(spans) / (ms * 1e-3)
us = 1e6 / rate
pro = sum(r[1] - r[0] for r in t) / nblk
main = sum(r[2] - r[1] for r in t) / nblk
epi = sum(r[3] - r[2] for r in t) / nblk
busy = sum(r[3] - r[0] for r in t) * us * 1e-3  # block-ms
# HW_ID (gfx9): wave_id[3:0], simd_id[5:4], pipe[7:6], cu_id[11:8], sh_id[12], se_id[15:13]
per_cu = defaultdict(list)
for r in t:
    per_cu[(r[5] & 0xF, (r[4] >> 8) & 0xFF)].append((r[0], r[3]))
gaps = []
for v in per_cu.values():
    v.sort()
    gaps += [b[0] - a[1] for a, b in zip(v, v[1:])]
gap = sum(gaps) / max(1, len(gaps))
print(f"M={M} N={N} K={Kd}: {ms:.3f} ms, {nblk} blocks on {len(per_cu)} CUs ({len(by_xcc)} XCDs), "
      f"tick {us * 1e3:.3f} ns, mean blocks in flight {busy / ms:.1f}")
print(f"  prologue {pro * us:6.2f} us | main {main * us:6.2f} us | epilogue {epi * us:6.2f} us | "
      f"gap between blocks on a CU {gap * us:6.2f} us")
