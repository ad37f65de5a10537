#!/bin/bash
# SQ issue/wait counters of one kernel_one.py probe, two rocprofv3 --pmc passes (<= 8 SQ counters each).
#   bash tools/pmc_sq.sh <probe> <outdir>
set -e
export TMPDIR=/tmp
P=$1; OUT=$2
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/a -o run --output-format csv -- python tools/kernel_one.py $P 3 > $OUT/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA GRBM_COUNT -d $OUT/b -o run --output-format csv -- python tools/kernel_one.py $P 3 > $OUT/b.log 2>&1
