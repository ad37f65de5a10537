#!/usr/bin/env python
"""Benchmark: GPT-2 training step (fwd + bwd + grad all-reduce + AdamW) on N MI355X GPUs.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU, RCCL). W untimed warm-up steps, then EXACTLY K steps
bracketed by barrier + synchronize, wall time = MAX over ranks; rank 0 prints ONE JSON line.

Workload = BASELINE.json config 2/3: GPT-2 124M (12L/768d/12H, V=50257), B=64 sequences per GPU,
T=1024, bf16 compute (autocast numerics), fp32 master weights, fused AdamW (lr 1e-4, wd 0.1,
betas 0.9/0.95), dropout 0.1 as the reference's default config (model.py:47-51), grad_accum 1.
Data: synthetic uniform token batches already resident in HBM (no network).

Also reported:
  mfu          tok/s * 854,438,400 FLOP/token / (N * 2.5166e15)   (bf16 dense peak)
  roofline     for the dominant kernel (the tied lm_head GEMMs are the largest launches): algorithmic
               FLOP per launch / average launch time measured live with HIP events on the launch stream
  kernels      the same for every probed launch family
Probed launches: every launch of the probed families in every --probe-every'th timed step (default 5: steps 0, 5, 10,
15 of the default 20), so each launch of a step is sampled equally often. Each probed launch costs two event
records inside the timed region: probing all ≈ 76 launches of every step (rounds 1-4) cost 58.68 vs 58.49 ms per step
at every 5th step and 58.42 with the first step alone (profiles/r4pr/, same box, alternating runs).
  cpu_baseline the oracle (CPU restatement of the reference step, oracle/train_ref.py) timed on this
               host's cores on a bounded sample (rank 0, N = 1 only)
"""
import argparse
import contextlib
import json
import os
import sys
import time

# kernel arguments in device memory (set before the HIP runtime starts; an entry-point setting, see
# gpt_2_distributed_amd/__init__.py and INTEGRATION.md §4)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import torch  # noqa: E402
import torch.distributed as dist

PEAK_BF16_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12  # 2516.6 dense bf16 (MI355X_MICROARCH.md)
METRIC = "train tokens/sec (whole node) + MFU, GPT-2 124M B=64 T=1024 at 1/2/4/8 MI355X"  # BASELINE.json


def metric_name(model, B, T, parallel, wrapped, GA):
    """BASELINE.json's metric string for its headline configuration (124M, B=64, T=1024); the same metric named for
    the configuration actually run otherwise (BASELINE cfgs 4 / 5: 350M / 1.5B under FSDP, accumulation)."""
    if model == "124M" and B == 64 and T == 1024 and GA == 1 and not (wrapped and parallel == "fsdp"):
        return METRIC
    return (f"train tokens/sec (whole node) + MFU, GPT-2 {model} B={B} T={T}"
            + (f" x{GA} accumulated" if GA > 1 else "") + (" FSDP" if wrapped and parallel == "fsdp" else ""))


def flops_per_token(cfg, T):
    C, L, V = cfg.n_embd, cfg.n_layer, cfg.vocab_size
    return 6 * (L * 12 * C * C + V * C) + 12 * L * T * C


def cpu_baseline(batch=4, seq_len=1024, steps=3):
    """The oracle's fp32 CPU step on BASELINE cfg 1's shape (124M, B=4, T=1024; bounded sample: 3 timed
    steps after 1 warm-up step, about 15-30 s of CPU work)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracle import model_ref, train_ref
    cfg = model_ref.Cfg(resid_pdrop=0.0, attn_pdrop=0.0, n_positions=seq_len)
    g = torch.Generator().manual_seed(0)
    data = [(torch.randint(0, cfg.vocab_size, (batch, seq_len), generator=g),
             torch.randint(0, cfg.vocab_size, (batch, seq_len), generator=g)) for _ in range(steps + 1)]
    params = model_ref.init_params(cfg)
    train_ref.run(cfg, data[:1], 1, params=params)  # warm-up (allocations, thread pool)
    t0 = time.perf_counter()
    train_ref.run(cfg, data[1:], steps, params=params)
    dt = time.perf_counter() - t0
    return {"value": round(steps * batch * seq_len / dt, 2), "unit": "tokens/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle/train_ref.py fp32 fwd+bwd+AdamW, 124M, B={batch}, T={seq_len}, {steps} timed steps "
                      f"({dt:.1f} s) after 1 warm-up"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--model", default="124M")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    # BASELINE configs 4-5 (350M / 1.5B under FSDP, 1.5B with gradient accumulation); a "step" is then one
    # optimizer step over grad_accum micro-batches of --batch sequences per rank
    ap.add_argument("--parallel", choices=["ddp", "fsdp"], default="ddp", help="multi-rank wrapper (N > 1)")
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--resident", action="store_true",
                    help="--parallel fsdp: keep gathered units resident (default: reshard after forward, FULL_SHARD's "
                         "memory behaviour as in the reference)")
    ap.add_argument("--reshard", action="store_true", help="--parallel fsdp: the default (kept for older scripts)")
    ap.add_argument("--probe-every", type=int, default=5,
                    help="time the probed kernel launches (HIP events) in every N-th timed step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from gpt_2_distributed_amd.parallel import init_distributed, local_device_index, use_collectives
    local_rank = local_device_index()
    # a torchrun launch of one rank with GPT2MI_FORCE_COLLECTIVES=1 runs the wrapper and its RCCL calls too
    wrapped = world > 1 or ("WORLD_SIZE" in os.environ and use_collectives(world))
    if wrapped:
        init_distributed()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from gpt_2_distributed_amd.model import GPT2, GPT2Config, MODEL_SIZES
    cfg = GPT2Config(**MODEL_SIZES[args.model], n_positions=args.seq_len, resid_pdrop=args.dropout,
                     attn_pdrop=args.dropout)
    model = GPT2(cfg).to(dev)
    model.train()
    if wrapped:
        from gpt_2_distributed_amd.parallel import DistributedDataParallel, ShardedDataParallel
        wrap = ShardedDataParallel if args.parallel == "fsdp" else DistributedDataParallel
        # the embeddings' all-reduce (DDP) / reduce-scatter (FSDP) runs under the optimizer step of every other range
        extra = dict(reshard_after_forward=not args.resident) if args.parallel == "fsdp" else {}
        ddp = wrap(model, bucket_mb=args.bucket_mb, overlap_optimizer=True, **extra)
        opt = ddp.configure_optimizers(learning_rate=1e-4)
        fwd = ddp
    else:
        opt = model.configure_optimizers(learning_rate=1e-4)
        fwd = model
    eng = model.engine()

    B, T = args.batch, args.seq_len
    g = torch.Generator().manual_seed(1234 + rank)
    batches = []
    for _ in range(4):
        t = torch.randint(0, cfg.vocab_size, (B, T + 1), generator=g)
        batches.append((t[:, :-1].contiguous().to(dev), t[:, 1:].contiguous().to(dev)))

    GA = args.grad_accum

    def step(i):
        # the reference loop (:400-425) runs every micro-step's backward synced; the resident wrappers skip the
        # collective on all but the last one (no_sync: the same sums), the resharded FSDP reduce-scatters every one
        # as the reference does (its gradients do not outlive their unit's backward)
        sync_each = args.parallel == "fsdp" and not args.resident
        for a in range(GA):
            x, y = batches[(i * GA + a) % len(batches)]
            ctx = fwd.no_sync() if (a + 1 < GA and hasattr(fwd, "no_sync") and not sync_each) \
                else contextlib.nullcontext()
            with ctx:
                with torch.autocast("cuda", dtype=torch.bfloat16):  # the reference trainer's step (:404)
                    _, loss = fwd(x, labels=y)
                    loss = loss / GA
                loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    for i in range(args.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    if wrapped:
        dist.barrier()
    probes = ["lm_head_fwd", "lm_head_dgrad", "lm_head_wgrad", "fc1_fwd", "attn_fwd", "wgrad"]
    armed = {p: [] for p in probes}
    every = max(1, args.probe_every)
    torch.cuda.synchronize()
    if wrapped:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        eng.probes = armed if i % every == 0 else {}  # the sampled steps record events around every probed launch
        loss = step(i)
    torch.cuda.synchronize()
    if wrapped:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.probes = {}
    dt_t = torch.tensor([dt], device=dev)
    if wrapped:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    final_loss = float(loss.item())

    M = B * T
    C, V, H = cfg.n_embd, cfg.vocab_size, cfg.n_head
    kflops = {
        "lm_head_fwd": 2.0 * M * V * C, "lm_head_dgrad": 2.0 * M * V * C, "lm_head_wgrad": 2.0 * M * V * C,
        "fc1_fwd": 2.0 * M * 4 * C * C, "attn_fwd": 4.0 * B * H * (T * (T + 1) / 2) * (C // H),
        # the weight-gradient family (the tied lm_head + every block's qkv / proj / fc1 / fc2 weight gradients, each
        # launch with its split-K reduction; 1 + L launches a step since round 6, a block's four grouped in one, 1 + 4L
        # before): the average algorithmic FLOPs of a launch = the step's weight-gradient FLOPs / its launches
        "wgrad": (2.0 * M * V * C + cfg.n_layer * 2.0 * M * 12 * C * C)
        / max(1.0, len(armed["wgrad"]) / len(range(0, args.steps, every))),
    }
    kernels = {}
    for name, evs in armed.items():
        if not evs:
            continue
        ms = sum(s.elapsed_time(e) for s, e in evs) / len(evs)
        tf = kflops[name] / (ms * 1e-3) / 1e12
        kernels[name] = {"avg_ms": round(ms, 4), "launches": len(evs), "tflops": round(tf, 1),
                         "frac_of_peak": round(tf / PEAK_BF16_TFLOPS, 4)}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["launches"] / max(1, args.steps)) \
        if kernels else None
    # roofline.traffic: the HBM bytes per launch of the dominant kernel from the PMC passes of THIS configuration
    # (tools/pmc_traffic.sh -> profiles/traffic.json, collected at BASELINE cfg 2: 124M, B=64, T=1024); null for any
    # other configuration (no PMC pass of its shapes), with the configuration the file's numbers belong to named
    traffic, traffic_src = None, None
    tpath = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    cfg2 = args.model == "124M" and B == 64 and T == 1024
    if dom and os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get(dom, {}).get("hbm_bytes_per_launch") if cfg2 else None
        except Exception:
            traffic = None
        traffic_src = ("profiles/traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this configuration "
                       "(124M, B=64, T=1024)" if traffic is not None else
                       "null: profiles/traffic.json holds PMC passes of 124M, B=64, T=1024 only, not of this "
                       "configuration's shapes")
    roofline = None
    if dom:
        k = kernels[dom]
        roofline = {"kernel": dom, "bound": "mfma", "achieved": k["tflops"], "peak": round(PEAK_BF16_TFLOPS, 1),
                    "unit": "TFLOP/s", "frac": k["frac_of_peak"], "traffic": traffic, "traffic_source": traffic_src,
                    "algorithmic_flop_per_launch": kflops[dom]}

    tokens = world * B * T * GA * args.steps
    tok_s = tokens / dt
    fpt = flops_per_token(cfg, T)
    out = {
        "metric": metric_name(args.model, B, T, args.parallel, wrapped, GA),
        "value": round(tok_s, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (uniform random tokens, resident in HBM)",
        "config": {"workload": f"GPT-2 {args.model} training step: fwd+loss+bwd+AdamW"
                               + ({"ddp": " + bucketed grad all-reduce in the backward",
                                   "fsdp": " + per-block FSDP all-gather / reduce-scatter"
                                   + (", resident units" if args.resident else ", resharded after forward")}[args.parallel]
                                  if wrapped else "")
                               + f", dropout {args.dropout}" + (f", {GA} accumulated micro-batches" if GA > 1 else ""),
                   "model": f"GPT-2 {args.model}", "global_batch": B * world * GA, "seq_len": T,
                   "parallelism": f"{'fsdp' if args.parallel == 'fsdp' and wrapped else 'dp'}{world}"},
        "mfu": round(tok_s * fpt / (world * PEAK_BF16_TFLOPS * 1e12), 4),
        "flop_per_token": fpt,
        "final_loss": round(final_loss * GA, 4),
        # peak HBM allocated on this rank (torch's caching allocator: activations, arenas, collective buffers)
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
        "roofline": roofline,
        "kernels": kernels,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(seq_len=T)
        except Exception as e:  # reported, never fatal to the GPU measurement
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if wrapped:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
