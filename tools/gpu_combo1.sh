#!/bin/bash
# one GPU session: the bench matrix (tools/gpu_bench_matrix.sh), then the tile-group A/B
TAG=${TAG:-r3b} bash tools/gpu_bench_matrix.sh || exit $?
bash tools/gpu_ab_gm.sh
