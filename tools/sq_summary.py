#!/usr/bin/env python
"""Derived SQ metrics per kernel from tools/pmc_sq.sh output directories (rocprofv3 --pmc csv; per-launch
averages, the cold first launch dropped):
  cyc        = GRBM_GUI_ACTIVE / 8                                  GPU-active cycles of one XCD (the counter is
                                                                    summed over the 8 XCDs); clock = cyc / duration
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (cyc * 1024)              share of the 1024 SIMDs' cycles the MFMA pipe
                                                                    is busy (16 cycles per v_mfma_f32_16x16x32_bf16,
                                                                    summed over SIMDs). Against the 2.4 GHz peak the
                                                                    kernel reaches mfma_busy * clock / 2.4
  valu_busy  = SQ_ACTIVE_INST_VALU * 4 / (cyc * 1024)                VALU issue (quad-cycle counter)
  wait_any   = SQ_WAIT_ANY / SQ_WAVE_CYCLES                          share of wave lifetime waiting (any reason)
  wait_inst  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES                     ... waiting on s_waitcnt (memory / LDS)
  lds_conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE               LDS bank-conflict cycles per active cycle
  mfma/valu/lds/salu instructions per launch
    python tools/sq_summary.py <outdir>/<probe> [...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                agg[(name, "DURATION_NS")].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    out = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        v = v[1:] if len(v) > 1 else v
        out[k][c] = sum(v) / len(v)
    return out


def main():
    for d in sys.argv[1:]:
        data = load(d)
        for k, c in sorted(data.items()):
            if "gpt2mi" not in k and "gemm" not in k and "attn" not in k and "splitk" not in k:
                continue
            g = c.get("GRBM_GUI_ACTIVE") or c.get("GRBM_COUNT")
            if not g:
                continue
            cyc = g / 8
            simd = cyc * 1024
            dur = c.get("DURATION_NS", 0)
            row = {
                "us": dur / 1e3,
                "clock_ghz": cyc / dur if dur else 0.0,
                "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd,
                "valu_busy": c.get("SQ_ACTIVE_INST_VALU", 0) * 4 / simd,
                "wait_any": c.get("SQ_WAIT_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)),
                "wait_inst": c.get("SQ_WAIT_INST_ANY", 0) / max(1, c.get("SQ_WAVE_CYCLES", 1)),
                "lds_conf": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c.get("SQ_LDS_IDX_ACTIVE", 1)),
            }
            print(f"{os.path.basename(d.rstrip('/'))}: {k[:90]}")
            print("   " + "  ".join(f"{n} {v:.3f}" for n, v in row.items())
                  + f"  | insts mfma {c.get('SQ_INSTS_MFMA', 0):.3g} valu {c.get('SQ_INSTS_VALU', 0):.3g}"
                  + f" lds {c.get('SQ_INSTS_LDS', 0):.3g} salu {c.get('SQ_INSTS_SALU', 0):.3g}"
                  + f" xcd_cycles {cyc:.4g}")


if __name__ == "__main__":
    main()
