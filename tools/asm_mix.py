#!/usr/bin/env python
"""Instruction mix per basic block of one kernel in a hipcc -S listing (loop bodies are the blocks a
later branch jumps back to).  python tools/asm_mix.py file.s kernel_substring"""
import collections
import re
import sys


def classify(op):
    for pre, k in (("v_mfma", "mfma"), ("v_exp", "exp"), ("v_mul_lo_u32", "mul_lo"), ("v_cvt_pk_bf16", "cvt_pk"),
                   ("v_cndmask", "cndmask"), ("v_cmp", "vcmp"), ("v_mov", "mov"), ("v_accvgpr", "accmov"),
                   ("v_permlane", "permlane"), ("v_pk_", "vpk"), ("v_", "valu"), ("s_waitcnt", "wait"),
                   ("s_barrier", "barrier"), ("s_", "salu"), ("ds_", "ds"), ("buffer_", "vmem"), ("global_", "vmem")):
        if op.startswith(pre):
            return k
    return op


def main(path, key):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\w+:", l) and key in l)
    blocks, cur, name = [], [], "entry"
    for l in lines[start + 1:]:
        t = l.strip()
        if t.startswith("s_endpgm"):
            break
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        if not t or t.startswith((";", ".")):
            continue
        cur.append(t)
    blocks.append((name, cur))
    order = [b[0] for b in blocks]
    for i, (n, body) in enumerate(blocks):
        tgts = [re.findall(r"(\.LBB\w+)", x) for x in body if x.startswith("s_cbranch") or x.startswith("s_branch")]
        back = any(t in order[:i + 1] for ts in tgts for t in ts)
        c = collections.Counter(classify(x.split()[0]) for x in body)
        print(f"{n:14s} {len(body):5d} {'LOOP' if back else '    '} " + " ".join(f"{k}={v}" for k, v in c.most_common()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
