#!/bin/bash
# Builds the wgrad ablation libraries (gemm256.hip with -DWG_ABL=n: 1 no MFMA, 2 no fragment reads, 4 no
# next-tile DMA) into tools/ab/ for tools/lib_ab.py:  bash tools/wgrad_ablation.sh 0 1 2 4 6
set -e
cd "$(dirname "$0")/../gpt_2_distributed_amd/csrc"
make -s -j8
mkdir -p ../../tools/ab
OBJS="build/runtime.cpp.o build/norm_embed.hip.o build/xent_adamw.hip.o build/gemm.hip.o build/gemm_pp.hip.o build/attention.hip.o build/fp32.hip.o build/transpose.hip.o build/aux_ops.hip.o"
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Wall -Wno-unused-function -I../../include \
    -DGPT2MI_AB_BUILD -DWG_ABL=$n -c gemm256.hip -o build/gemm256_abl$n.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/ab/lib_abl$n.so $OBJS build/gemm256_abl$n.o
done
ls -la ../../tools/ab
