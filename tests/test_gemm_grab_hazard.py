"""The persistent GEMM's work-queue grab (gemm_pp.hip, DYN variants) on the code hipcc actually emits (CPU only).

The grab is a returning `global_atomic_add` issued from inline asm, so that no compiler-inserted `s_waitcnt vmcnt(0)`
drains the LDS-DMAs in flight behind it; its return VGPR is written asynchronously and only the kernel's own counted
waits retire it. The compiler does not know that: if register allocation ever copied, moved, read or reused that VGPR
before a `vmcnt(0)` retires the atomic, a tile would be lost or run twice without any spill showing. This
test compiles gemm_pp.hip to device assembly with the Makefile's flags and walks the control-flow graph of every DYN
kernel from each returning atomic: on every path, no instruction may touch the return register before an
`s_waitcnt` with `vmcnt(0)`.

The scheme also assumes that workgroups with equal `blockIdx.x % 8` share an XCD (speed only, never correctness:
each label's counter is private to its blocks, wherever they run)."""
import os
import re
import shutil
import subprocess

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpt_2_distributed_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _asm():
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", f"-I{CSRC}/../../include",
           "-fno-slp-vectorize", "--cuda-device-only", "-S", os.path.join(CSRC, "gemm_pp.hip"), "-o", "-"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout


def _functions(asm):
    funcs, cur, name = {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name, cur = m.group(1), []
            funcs[name] = cur
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        s = line.split(";")[0].strip()
        if s:
            cur.append(s)
    return funcs


def _regs(ins):
    """VGPR numbers an instruction names (operands only)."""
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return set()
    ops = parts[1]
    regs = {int(r) for r in re.findall(r"(?<![\w\[])v(\d+)\b", ops)}
    for a, b in re.findall(r"(?<!\w)v\[(\d+):(\d+)\]", ops):
        regs.update(range(int(a), int(b) + 1))
    return regs


def _cfg(body):
    """label -> instructions, and the label that follows each label in the text (fall-through)."""
    blocks, order, cur = {"__entry": []}, ["__entry"], "__entry"
    for s in body:
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        if s.startswith("."):
            continue
        blocks[cur].append(s)
    fall = {lab: (order[i + 1] if i + 1 < len(order) else None) for i, lab in enumerate(order)}
    return blocks, fall


def _vmcnt0(s):
    return s.startswith("s_waitcnt") and re.search(r"vmcnt\(0\)", s) is not None


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
def test_work_queue_grab_register_untouched_until_retired():
    funcs = _functions(_asm())
    # template arguments <A_T, B_T, EPI, MAP, PERSIST, BND, DYN, GRP>: DYN = 1 (GRP = 0, the single-problem kernels)
    dyn = {n: b for n, b in funcs.items()
           if re.search(r"gemm_pp_kernelILb[01]ELb[01]ELi\d+ELi\d+ELb[01]ELb[01]ELb1ELb0E", n)}
    assert dyn, "no DYN (work-queue) kernel found"
    checked = 0
    for name, body in dyn.items():
        blocks, fall = _cfg(body)
        for lab, ins in blocks.items():
            for k, s in enumerate(ins):
                if not (s.startswith("global_atomic_add ") and " sc0" in s):
                    continue
                dst = int(re.match(r"global_atomic_add v(\d+),", s).group(1))
                checked += 1
                # walk every path from the instruction after the atomic to the first vmcnt(0)
                stack, seen = [(lab, k + 1)], set()
                while stack:
                    b, i = stack.pop()
                    if (b, i) in seen:
                        continue
                    seen.add((b, i))
                    seq = blocks[b]
                    done = False
                    for j in range(i, len(seq)):
                        t = seq[j]
                        if _vmcnt0(t) or t.startswith("s_endpgm"):
                            done = True
                            break
                        assert dst not in _regs(t), (
                            f"{name}: v{dst} (work-queue grab in flight) touched by '{t}' before vmcnt(0)")
                        if t.startswith("s_cbranch"):
                            stack.append((t.split()[1], 0))
                        elif t.startswith("s_branch"):
                            stack.append((t.split()[1], 0))
                            done = True
                            break
                    if not done and fall[b]:
                        stack.append((fall[b], 0))
    assert checked >= len(dyn), f"expected a returning grab atomic in each of {len(dyn)} DYN kernels, found {checked}"
