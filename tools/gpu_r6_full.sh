#!/bin/bash
# Round 6: the whole GPU test suite + smoke, the default bench, BASELINE cfg 5 as SURVEY specifies it (GPT-2 1.5B, FSDP,
# B = 32, grad_accum 4; resharded = the default, and resident) on one forced-RCCL rank, and rocprof summaries of the default bench and
# of GPT-2 1.5B at B = 8 -> gpurun_out/$TAG/
set -o pipefail
T=${TAG:-r6e}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
run() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  grep '^{' $O/$name.log | tail -1 > $O/$name.json
  echo "$name rc=$rc $(cut -c1-240 $O/$name.json)"
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29581"
run bench 300 python bench.py || exit $?
if [ -n "$WRAPPED" ]; then  # the one-rank DDP / FSDP overhead against the same call's bench
  run ddp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel ddp || exit $?
  run fsdp1 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp || exit $?
  run fsdp1_resident 300 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp --resident || exit $?
  run bench_again 300 python bench.py --no-cpu-baseline || exit $?
fi
if [ -n "$MODELS" ]; then  # BASELINE cfgs 4 / 5 on one forced-RCCL rank: FULL_SHARD (the default) and resident
  run m350_fsdp 400 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp --model 350M \
    --batch 32 --steps 6 --warmup 2 || exit $?
  run m15b_fsdp_ga4 600 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp --model 1.5B \
    --batch 32 --grad_accum 4 --steps 4 --warmup 2 || exit $?
  run m15b_fsdp_ga4_resident 600 env GPT2MI_FORCE_COLLECTIVES=1 $TR bench.py --no-cpu-baseline --parallel fsdp \
    --resident --model 1.5B --batch 32 --grad_accum 4 --steps 4 --warmup 2 || exit $?
fi
if [ -n "$PMC" ]; then  # HBM traffic of the bench's dominant (weight-gradient) family -> profiles/traffic.json
  PROBES=wgrad timeout -k 10 400 bash tools/pmc_traffic.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
  cp profiles/traffic.json $O/traffic.json; tail -2 $O/pmc.log
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 5 --warmup 3 \
    --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
  python tools/rocpd_stats.py $O/prof/run_results.db $O/kernel_stats.csv && \
    python tools/prof_summary.py $O/kernel_stats.csv 8 > $O/summary.txt 2>&1; head -30 $O/summary.txt
fi
if [ -n "$PROF15" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof15 -o run -- python bench.py --model 1.5B --batch 8 \
    --steps 3 --warmup 2 --no-cpu-baseline > $O/prof15.log 2>&1 || exit $?
  grep '^{' $O/prof15.log | tail -1 > $O/m15b8.json
  python tools/rocpd_stats.py $O/prof15/run_results.db $O/kernel_stats15.csv && \
    python tools/prof_summary.py $O/kernel_stats15.csv 5 > $O/summary15.txt 2>&1; head -30 $O/summary15.txt
fi
if [ -n "$TRAIN" ]; then  # the reference trainer's loop end to end on synthetic Zipf shards: the loss curve
  timeout -k 10 600 python -m gpt_2_distributed_amd.train_gpt2_distributed --synthetic 4 --synthetic_tokens 20000000 \
    --seq_len 1024 --batch 16 --grad_accum_steps 4 --max_steps 300 --log_every 10 --save_every 100000 --lr 6e-4 \
    --workers 2 --save_dir /tmp/ckpt_train > $O/train_curve.log 2>&1 || { tail -20 $O/train_curve.log; exit 1; }
  grep '^{' $O/train_curve.log | python -c "import json,sys; r=[json.loads(l) for l in sys.stdin]; print('train', [(d['step'], d['loss']) for d in r][::3], 'tok/s', r[-1]['tok_per_s_node'])"
fi
if [ -n "$PROFW" ]; then  # rocprof of the one-rank wrapped lines (forced RCCL collectives): where the wrapper's time goes
  for v in "ddp:--parallel ddp" "fsdp:--parallel fsdp" "fsdpres:--parallel fsdp --resident"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 300 env GPT2MI_FORCE_COLLECTIVES=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 \
      MASTER_PORT=29591 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run -- python bench.py --steps 5 \
      --warmup 3 --no-cpu-baseline $args > $O/prof_$name.log 2>&1 || exit $?
    python tools/rocpd_stats.py $O/prof_$name/run_results.db $O/kernel_stats_$name.csv && \
      python tools/prof_summary.py $O/kernel_stats_$name.csv 8 > $O/summary_$name.txt 2>&1
    echo "== $name"; head -8 $O/summary_$name.txt; tail -1 $O/summary_$name.txt
  done
fi
