#!/usr/bin/env python
"""All-reduce bus bandwidth at the DDP step's bucket sizes, for the first multi-GPU run (RCCL over xGMI).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29600 \
        tools/rccl_busbw.py [--backend nccl] [--sizes-mb 1,4,28,157,498] [--iters 20]

Prints one JSON line per size on rank 0: algbw = bytes / time, busbw = algbw * 2 (W - 1) / W (the ring all-reduce's
per-GPU traffic, the figure nccl-tests reports), time = max over ranks. Sizes: 28 MB = one GPT2Block bucket of the 124M
grad arena (fp32), 157 MB = the embedding bucket (wte + wpe), 498 MB = the whole arena. Run it once with RCCL's
defaults and once per channel setting tried (e.g. NCCL_MIN_NCHANNELS=32, NCCL_DEBUG=INFO shows the channels RCCL
built); `--backend gloo` runs it on the CPU.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--sizes-mb", default="1,4,28,157,498")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    gpu = args.backend == "nccl"
    if gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    dev = torch.device("cuda") if gpu else torch.device("cpu")

    def sync():
        if gpu:
            torch.cuda.synchronize()

    for mb in (float(s) for s in args.sizes_mb.split(",") if s):
        n = max(1, int(mb * 1e6) // 4)
        x = torch.ones(n, dtype=torch.float32, device=dev)
        for _ in range(args.warmup):
            dist.all_reduce(x)
        sync()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            dist.all_reduce(x)
        sync()
        dt = torch.tensor([(time.perf_counter() - t0) / args.iters], dtype=torch.float64, device=dev)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        # x was summed iters + warmup times starting from ones: every element is world ** (iters + warmup), so a
        # wrong reduction shows up without a second buffer (checked while that stays finite)
        k = args.iters + args.warmup
        if world ** k < 1e30:
            assert torch.all(x == float(world) ** k), "all-reduce result"
        t = float(dt.item())
        alg = 4 * n / t / 1e9
        if rank == 0:
            print(json.dumps({"size_mb": round(4 * n / 1e6, 3), "world": world, "backend": args.backend,
                              "ms": round(t * 1e3, 4), "algbw_GBps": round(alg, 2),
                              "busbw_GBps": round(alg * 2 * (world - 1) / max(world, 1), 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
