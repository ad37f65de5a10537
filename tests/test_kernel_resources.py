"""Register budget of the hand-scheduled kernels (CPU: cross-compiles for gfx950, no GPU).

The ping-pong GEMM and the attention kernels count their own LDS-DMA instructions with literal
`s_waitcnt vmcnt(N)`; a register spill adds scratch memory operations to that counter and silently
breaks the accounting (and costs HBM round trips). Every kernel must compile with zero scratch, no
spills, and the occupancy its launch bounds promise."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpt_2_distributed_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# source -> {kernel-name substring: minimum occupancy (waves/SIMD)}
EXPECT = {
    "gemm_pp.hip": {"gemm_pp_kernel": 2},
    "attention.hip": {"attn_fwd_kernel": 3, "attn_bwd_dkdv_kernel": 3, "attn_bwd_dq_kernel": 3},
}


def _resources(src, extra=()):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", f"-I{CSRC}/../../include", *extra, "-c",
           os.path.join(CSRC, src), "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    kernels, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill): (\S+)", line)
        if not m:
            continue
        key, val = m.groups()
        if key == "Function Name":
            name = val
            kernels[name] = {}
        elif name:
            kernels[name][key] = int(val)
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src", sorted(EXPECT))
def test_no_scratch_and_occupancy(src):
    extra = {"attention.hip": ("-fno-honor-nans", "-fno-slp-vectorize"),  # as the Makefile builds them
             "gemm_pp.hip": ("-fno-slp-vectorize",)}.get(src, ())
    kernels = _resources(src, extra)
    for sub, occ in EXPECT[src].items():
        found = {k: v for k, v in kernels.items() if sub in k}
        assert found, f"{sub} not found in {src}"
        for k, v in found.items():
            assert v["ScratchSize [bytes/lane]"] == 0, f"{k}: scratch {v}"
            assert v["VGPRs Spill"] == 0, f"{k}: spills {v}"  # (SGPR spills go to VGPR lanes: no memory)
            assert v["Occupancy [waves/SIMD]"] >= occ, f"{k}: occupancy {v}"
