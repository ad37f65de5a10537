#!/bin/bash
# Builds an A/B library variant into tools/ab/lib_<name>.so: the tree's objects with ONE source file recompiled
# with extra flags (e.g. -DSOME_EXPERIMENT), for tools/lib_ab.py.
#   bash tools/variant_lib.sh <name> <source.hip> [flags...]
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../gpt_2_distributed_amd/csrc"
make -s -j8
mkdir -p ../../tools/ab
OBJS=""
for f in runtime.cpp norm_embed.hip xent_adamw.hip gemm.hip gemm256.hip gemm_pp.hip attention.hip fp32.hip transpose.hip aux_ops.hip; do
  [ "$f" = "$SRC" ] || OBJS="$OBJS build/$f.o"
done
EXTRA=""; [ "$SRC" = attention.hip ] && EXTRA="-fno-honor-nans -fno-slp-vectorize"
[ "$SRC" = gemm_pp.hip ] && EXTRA="-fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++20 -Wall -Wno-unused-function -I../../include -DGPT2MI_AB_BUILD $EXTRA "$@" \
  -c "$SRC" -o "build/${SRC}_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "../../tools/ab/lib_$NAME.so" $OBJS "build/${SRC}_$NAME.o"
echo "tools/ab/lib_$NAME.so"
