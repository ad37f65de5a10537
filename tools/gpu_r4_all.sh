#!/bin/bash
# tests (tools/gpu_r4_tests.sh) then the bench lines + rocprof (tools/gpu_r4_bench.sh) in one call; the benches run after
# a test FAILURE (not after a time limit, abort or fault: then nothing more runs on the GPU)
TAG=${TAG:-r4x}
TAG=$TAG bash tools/gpu_r4_tests.sh
rc=$?
case $rc in 0|1) ;; *) echo "tests rc=$rc: stopping"; exit $rc ;; esac
TAG=$TAG PROF=${PROF:-1} bash tools/gpu_r4_bench.sh || exit $?
exit $rc
