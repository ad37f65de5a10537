#!/usr/bin/env python
"""Training CLI with the reference's flags (`/root/reference/train_gpt2_distributed.py:282-310`).

    python -m gpt_2_distributed_amd.train_gpt2_distributed --data_dir DIR [--training_mode local|ddp|fsdp]
        [--device cuda] [--seq_len 1024] [--batch 4] [--grad_accum_steps 4] [--epochs 1] [--lr 1e-4]
        [--save_every 1000] [--save_dir ./checkpoints] [--log_dir ./logs] [--workers 2]
    build-side extensions: --model {124M,350M,1.5B} --dropout P --max_steps N --synthetic N_SHARDS
        --resume STEP_DIR --log_every N

Loop semantics follow the reference (:374-457): seed 42; loss/grad_accum; backward; every
grad_accum micro-steps the fused AdamW step (which also yields the clip_grad_norm_(inf) value);
checkpoints every --save_every optimizer steps between barriers. Differences, all deliberate:
  * DDP syncs gradients only on the last micro-step (``no_sync`` elsewhere; same math);
  * logged tok/s is the whole-node SUM and MFU is reported (the reference averages per-GPU tok/s,
    stats_tracker.py:25-34); host syncs happen only on log steps, which also carry the reference's epoch_time and
    memory metrics (gpu_alloc_gb, gpu_reserved_gb, gpu_max_alloc_gb, gpu_utilization_pct, cpu_mb;
    stats_tracker.py:265-364) with its reductions over ranks (no TensorBoard writer);
  * checkpoints are collective-correct under fsdp, and --resume restores model + optimizer + the
    dropout stream + the data position (the reference's load_checkpoint is a stub, :104-111).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import pathlib
import tempfile
import time

import torch
import torch.distributed as dist

from . import dataloader as gpt2_dataloader
from .model import GPT2, GPT2Config, MODEL_SIZES
from .parallel import DistributedDataParallel, FullyShardedDataParallel, init_distributed, is_primary

SEED = 42
PEAK_BF16 = 2.5166e15


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", required=False, help="Path to data directory containing .bin files.")
    p.add_argument("--training_mode", choices=["fsdp", "ddp", "local"], default="local")
    p.add_argument("--device", default="cuda")
    p.add_argument("--seq_len", type=int, default=gpt2_dataloader.DEFAULT_CONTEXT_LENGTH)
    p.add_argument("--batch", type=int, default=gpt2_dataloader.DEFAULT_BATCH_SIZE)
    p.add_argument("--grad_accum_steps", type=int, default=4)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--save_every", type=int, default=1000)
    p.add_argument("--save_dir", type=str, default="./checkpoints")
    p.add_argument("--log_dir", type=str, default="./logs")
    p.add_argument("--workers", type=int, default=gpt2_dataloader.DEFAULT_N_PROCS)
    # build-side extensions
    p.add_argument("--model", choices=sorted(MODEL_SIZES), default="124M")
    p.add_argument("--dropout", type=float, default=None, help="override resid/attn dropout (default: config 0.1)")
    p.add_argument("--max_steps", type=int, default=0, help="stop after N optimizer steps (0 = run all epochs)")
    p.add_argument("--synthetic", type=int, default=0, help="write N synthetic Zipf shards and train on them")
    p.add_argument("--synthetic_tokens", type=int, default=2_000_000)
    p.add_argument("--resume", type=str, default="", help="checkpoint step_XXXXXXX directory to resume from")
    p.add_argument("--log_every", type=int, default=20)
    # fsdp memory behaviour: the reference's FSDP(sharding_strategy=FULL_SHARD) (train_gpt2_distributed.py:156-161)
    # frees each block's gathered parameters after its forward and gathers them again for its backward; that is the
    # default here too. --fsdp_resident keeps every gathered unit until the optimizer step instead (no re-gather in
    # the backward; per-rank memory then does not shrink with the world size: DESIGN.md §5)
    p.add_argument("--fsdp_resident", action="store_true",
                   help="fsdp: keep each gathered unit resident until the optimizer step instead of FULL_SHARD's "
                        "reshard after forward")
    p.add_argument("--fsdp_reshard", action="store_true",
                   help="fsdp: reshard after forward (the default; kept for command lines of earlier rounds)")
    return p


def save_checkpoint(model, opt, step: int, out_dir: str, trainer_state: dict = None):
    """step_{:07d}/model.pt (reference state_dict keys) + optim.pt (train_gpt2_distributed.py:67-101).
    Collective-correct (the reference returns early on non-primary ranks before FSDP's full-state
    all-gather, :81-94): under fsdp every rank joins the parameter gather and writes its optimizer shard
    (optim_rank{r}.pt). trainer.json keeps what an exact resume needs beyond the weights: the dropout
    stream position and the epoch / micro-batch the next step starts from."""
    base = model.module if hasattr(model, "module") else model
    out = os.path.join(out_dir, f"step_{step:07d}")
    sharded = isinstance(model, FullyShardedDataParallel)
    sd = model.state_dict() if sharded else base.state_dict()  # fsdp: a collective on every rank
    if is_primary():
        os.makedirs(out, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in sd.items()}, os.path.join(out, "model.pt"))
        st = dict(trainer_state or {}, step=step, step_seed=base.engine()._step_seed)
        with open(os.path.join(out, "trainer.json"), "w") as f:
            json.dump(st, f)
    if dist.is_initialized():
        dist.barrier()
    osd = opt.state_dict()
    osd = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in osd.items()}
    if sharded:
        torch.save(osd, os.path.join(out, f"optim_rank{dist.get_rank()}.pt"))
    elif is_primary():
        torch.save(osd, os.path.join(out, "optim.pt"))
    if dist.is_initialized():
        dist.barrier()
    return out


def load_checkpoint(model, opt, ckpt_dir: str):
    """Restore what save_checkpoint wrote (the reference's load_checkpoint is a stub, :104-111).
    Returns the trainer state (step, step_seed, epoch, micro)."""
    base = model.module if hasattr(model, "module") else model
    sd = torch.load(os.path.join(ckpt_dir, "model.pt"), map_location="cpu", weights_only=True)
    if isinstance(model, FullyShardedDataParallel):
        model.load_full_state_dict(sd)
    else:
        with torch.no_grad():
            for n, p in base.named_parameters():
                p.copy_(sd[n])
        base.engine().refresh_shadow()
    name = f"optim_rank{dist.get_rank()}.pt" if isinstance(model, FullyShardedDataParallel) else "optim.pt"
    osd = torch.load(os.path.join(ckpt_dir, name), map_location="cpu", weights_only=True)
    opt.load_state_dict(osd)
    st = {"step": int(osd["step"])}
    tpath = os.path.join(ckpt_dir, "trainer.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            st.update(json.load(f))
        base.engine()._step_seed = int(st.get("step_seed", 0))
    return st


def memory_metrics(world: int) -> dict:
    """The reference's memory metrics (stats_tracker.py:265-364: _collect_memory_metrics and its registry entries),
    reduced over ranks as it reduces them: gpu_alloc_gb / gpu_reserved_gb / gpu_utilization_pct averaged, gpu_max_alloc_gb
    the MAX, cpu_mb the SUM (host RSS of every process). GiB = 2^30 bytes, MB = 2^20 as there. Collective: every rank
    calls it (on log steps only)."""
    import psutil
    gib = 1024 ** 3
    alloc = torch.cuda.memory_allocated() / gib
    total = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory / gib
    v = torch.tensor([alloc, torch.cuda.memory_reserved() / gib, alloc / total * 100.0,
                      psutil.Process().memory_info().rss / 2 ** 20], dtype=torch.float64, device="cuda")
    mx = torch.tensor([torch.cuda.max_memory_allocated() / gib], dtype=torch.float64, device="cuda")
    if dist.is_initialized() and world > 1:
        dist.all_reduce(v)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        v[:3] /= world
    v, mx = v.tolist(), mx.item()
    return {"gpu_alloc_gb": round(v[0], 3), "gpu_reserved_gb": round(v[1], 3), "gpu_max_alloc_gb": round(mx, 3),
            "gpu_utilization_pct": round(v[2], 2), "cpu_mb": round(v[3], 1)}


def main(argv=None):
    torch.manual_seed(SEED)
    os.environ.setdefault("PYTORCH_CUDA_ALLOC_CONF", "expandable_segments:True")
    args = build_parser().parse_args(argv)
    if args.training_mode in ("fsdp", "ddp"):
        init_distributed()
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if not torch.cuda.is_available():
        raise ValueError("CUDA is not available.")  # as the reference (:322-323); no CPU path
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    data_dir = args.data_dir
    if args.synthetic:
        from .synthetic import write_shards
        data_dir = data_dir or tempfile.mkdtemp(prefix="gpt2_synth_")
        if is_primary():
            write_shards(data_dir, args.synthetic, args.synthetic_tokens, dist="zipf", seed=1234)
        if dist.is_initialized():
            dist.barrier()
    if not data_dir:
        raise SystemExit("--data_dir is required (or --synthetic N)")
    if is_primary():
        print(f"==> started rank {rank}/{world} on GPU {local_rank} in {args.training_mode.upper()} mode")
        print(f"==> Micro batch: {args.batch}, Gradient accum: {args.grad_accum_steps}")
        print(f"==> Sequence length: {args.seq_len}")

    paths = gpt2_dataloader.get_shard_paths(pathlib.Path(data_dir), split="train")
    ds = gpt2_dataloader.TokenShardDataset(paths, seq_len=args.seq_len, shuffle=True)
    dl = gpt2_dataloader.create_dataloader(ds, batch_size=args.batch, num_workers=args.workers) \
        if args.workers > 0 else None

    over = dict(MODEL_SIZES[args.model])
    if args.dropout is not None:
        over.update(resid_pdrop=args.dropout, attn_pdrop=args.dropout)
    config = dataclasses.replace(GPT2Config(), n_positions=args.seq_len, **over)
    base = GPT2(config).to(device)
    if args.training_mode == "ddp":
        model = DistributedDataParallel(base, overlap_optimizer=True)  # the grad norm comes from the fused AdamW
    elif args.training_mode == "fsdp":
        model = FullyShardedDataParallel(base, overlap_optimizer=True, reshard_after_forward=not args.fsdp_resident)
    else:
        model = base
    optim = model.configure_optimizers(weight_decay=0.1, learning_rate=args.lr, betas=(0.9, 0.95))
    global_step, start_epoch, skip = 0, 0, 0
    # the epoch the DataLoader's persistent workers were spawned with: they keep that dataset copy, so every later
    # epoch replays its order (SURVEY §5 "epoch freeze"); a resumed run must spawn its workers with the same one
    worker_epoch = None
    if args.resume:
        st = load_checkpoint(model, optim, args.resume)
        global_step = st["step"]
        start_epoch, skip = int(st.get("epoch", 0)), int(st.get("micro", 0))
        if st.get("worker_epoch") is not None:
            worker_epoch = int(st["worker_epoch"])
        elif "worker_epoch" not in st and start_epoch > 0:
            # a checkpoint from before worker_epoch was recorded: an uninterrupted run spawned its persistent workers
            # in epoch 0 (the first epoch it iterated), so they replay epoch 0's order in every later epoch
            worker_epoch = 0
    fpt = 6 * (config.n_layer * 12 * config.n_embd ** 2 + config.vocab_size * config.n_embd) + \
        12 * config.n_layer * args.seq_len * config.n_embd
    optim.zero_grad()
    tok_per_step = args.batch * args.grad_accum_steps * args.seq_len * world
    t_last, steps_since = time.perf_counter(), 0
    done, epoch, micro = False, start_epoch, 0
    for epoch in range(start_epoch, args.epochs):
        t_epoch = time.perf_counter()  # the reference's epoch_time (stats_tracker.py:265-275): time in this epoch
        ds.set_epoch(epoch)  # as the reference; persistent workers keep the epoch they were spawned with
        if dl is not None:
            if worker_epoch is None:
                worker_epoch = epoch  # the workers spawn at this epoch's first iteration
            else:
                ds.set_epoch(worker_epoch)  # no effect once they run; a resumed run spawns them with it
        if is_primary():
            print(f"\n==== Epoch {epoch} ====")
        batches = dl if dl is not None else gpt2_dataloader.iter_batches(paths, args.seq_len, args.batch, 1,
                                                                       epoch=epoch)
        micro = 0
        for x, y in batches:
            if skip:  # resume: the micro-batches the checkpointed steps already consumed
                skip -= 1
                micro += 1
                continue
            x = x.to(device, non_blocking=True)
            y = y.to(device, non_blocking=True)
            last = (micro + 1) % args.grad_accum_steps == 0
            # no_sync on the resident wrappers (the same sums, one collective per step); the resharded FSDP syncs every
            # micro-step, as the reference's loop does for every mode (its gradients do not outlive their unit)
            ctx = model.no_sync() if (hasattr(model, "no_sync") and not last
                                      and not getattr(model, "reshard_after_forward", False)) else _Null()
            with ctx:
                with torch.autocast("cuda", dtype=torch.bfloat16):  # as train_gpt2_distributed.py:404
                    _, loss = model(x, labels=y)
                    loss = loss / args.grad_accum_steps
                loss.backward()
            micro += 1
            if not last:
                continue
            optim.step()
            optim.zero_grad()
            global_step += 1
            steps_since += 1
            if global_step % args.log_every == 0 or global_step == 1:
                torch.cuda.synchronize()
                now = time.perf_counter()
                tps = tok_per_step * steps_since / (now - t_last)
                mem = memory_metrics(world)
                if is_primary():
                    print(json.dumps({"step": global_step, "loss": round(loss.item() * args.grad_accum_steps, 5),
                                      "grad_norm": round(float(optim.grad_norm.item()), 5), "lr": args.lr,
                                      "tok_per_s_node": round(tps, 1),
                                      "mfu": round(tps * fpt / (world * PEAK_BF16), 4),
                                      "epoch_time": round(now - t_epoch, 2), **mem}), flush=True)
                t_last, steps_since = now, 0
            if global_step % args.save_every == 0:
                save_checkpoint(model, optim, global_step, args.save_dir,
                                {"epoch": epoch, "micro": micro, "worker_epoch": worker_epoch})
            if args.max_steps and global_step >= args.max_steps:
                done = True
                break
        if done:
            break
    pos = {"epoch": epoch, "micro": micro} if done else {"epoch": args.epochs, "micro": 0}
    pos["worker_epoch"] = worker_epoch
    save_checkpoint(model, optim, global_step, args.save_dir, pos)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    # kernel arguments in device memory (gpt_2_distributed_amd/__init__.py); read when the HIP runtime starts, which
    # has not happened yet (importing torch does not start it); an explicit setting in the environment wins
    os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
    main()
