"""Data parallelism over RCCL (torch.distributed "nccl" = RCCL on ROCm), one process per GPU.

Replaces the reference's ``DDP(model, device_ids=[device])`` / ``FSDP(model, ...)``
(train_gpt2_distributed.py:129-165) and ``init_process_group("nccl")`` (:50-59):

* ``init_distributed()``: same contract as the reference (env:// rendezvous from torchrun,
  ``LOCAL_RANK`` -> device).
* ``DistributedDataParallel(model)``: broadcasts the flat fp32 arena from rank 0 once (C2) and
  all-reduces (average) the flat fp32 grad arena in ``bucket_mb`` buckets. Buckets are issued
  asynchronously from inside the engine's backward, as soon as a contiguous arena range is final
  (blocks finish last-to-first, wte/wpe at the very end), so RCCL runs on its own stream under the
  remaining backward kernels (C4). No per-forward buffer broadcast (C3): there is no mask buffer.
  ``no_sync()`` skips the collective on non-final gradient-accumulation micro-steps.
* ``ShardedDataParallel(model)`` (the ``--training_mode fsdp`` path): ZeRO-style full sharding of
  the optimizer over the same arena — grads are reduce-scattered (each rank receives the average of
  its 1/world slice), AdamW updates only the local slice of master weights and moments, and the
  updated fp32 slice is all-gathered back (C5). The whole model fits one MI355X (288 GB), so
  parameters are not freed between layers; sharding buys optimizer-state memory and halves the
  grad traffic of an all-reduce into RS + AG of the same bytes.

The bucketing logic is engine-agnostic (``BucketedReducer`` takes a flat tensor and ready ranges),
so it is tested on CPU with gloo.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist


def local_device_index() -> int:
    """LOCAL_RANK -> device (train_gpt2_distributed.py:59). GPT2MI_SINGLE_DEVICE=1 puts every rank on
    device 0: a test hook to rehearse the multi-rank path on a one-GPU box (with a gloo backend)."""
    if os.environ.get("GPT2MI_SINGLE_DEVICE") == "1":
        return 0
    return int(os.environ.get("LOCAL_RANK", 0))


def init_distributed() -> None:
    """train_gpt2_distributed.py:50-59: init_process_group("nccl") (= RCCL) + set_device(LOCAL_RANK).
    GPT2MI_DIST_BACKEND overrides the backend (tests)."""
    if dist.is_initialized():
        return
    backend = os.environ.get("GPT2MI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    dist.init_process_group(backend)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_device_index())


def is_primary() -> bool:
    return dist.get_rank() == 0 if dist.is_initialized() else True


class BucketedReducer:
    """Averages a flat gradient tensor across the group in contiguous buckets.

    ``order`` lists (name, lo, hi) ranges of ``flat`` in the order they become final during backward.
    ``mark_ready(name)`` is called when a range is final; once the ready-but-unsent span reaches
    ``bucket_bytes`` (or at ``flush``) an async all-reduce of that span is issued. Ranges must become
    ready so that the unsent span stays contiguous (true for reverse arena order)."""

    def __init__(self, flat: torch.Tensor, order: List[Tuple[str, int, int]], bucket_mb: float = 64.0,
                 group=None, mode: str = "allreduce"):
        self.flat = flat
        self.order = order
        self.index = {n: i for i, (n, _, _) in enumerate(order)}
        self.bucket_elems = int(bucket_mb * 1024 * 1024 / flat.element_size())
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.mode = mode
        self.use_avg = dist.get_backend(group) == "nccl"
        self.reset()

    def reset(self):
        self.next = 0           # next index in `order` not yet marked ready
        self.pending_lo = None  # unsent contiguous span [lo, hi)
        self.pending_hi = None
        self.works = []
        self.post = []          # gloo: spans to rescale after wait

    def mark_ready(self, name: str):
        i = self.index[name]
        if i < self.next:
            return
        while self.next <= i:
            _, lo, hi = self.order[self.next]
            if self.pending_lo is None:
                self.pending_lo, self.pending_hi = lo, hi
            else:
                # ranges arrive in descending arena order
                assert hi <= self.pending_lo + 0 or lo >= self.pending_hi, "non-contiguous ready order"
                self.pending_lo = min(self.pending_lo, lo)
                self.pending_hi = max(self.pending_hi, hi)
            self.next += 1
        if self.pending_hi - self.pending_lo >= self.bucket_elems:
            self._launch()

    def _launch(self):
        if self.pending_lo is None:
            return
        span = self.flat[self.pending_lo:self.pending_hi]
        if self.use_avg:
            w = dist.all_reduce(span, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        else:
            w = dist.all_reduce(span, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self.post.append(span)
        self.works.append(w)
        self.pending_lo = self.pending_hi = None

    def flush(self):
        """Mark everything ready, launch the tail and wait (current stream waits on RCCL)."""
        if self.next < len(self.order):
            self.mark_ready(self.order[-1][0])
        self._launch()
        for w in self.works:
            w.wait()
        for span in self.post:
            span.mul_(1.0 / self.world)
        self.works, self.post = [], []
        self.reset()


class DistributedDataParallel(torch.nn.Module):
    """DDP for the arena model: same call surface as torch DDP for the reference loop."""

    def __init__(self, module, device_ids=None, bucket_mb: float = 64.0, broadcast: bool = True):
        super().__init__()
        self.module = module
        eng = module.engine()
        self.engine = eng
        if broadcast and dist.get_world_size() > 1:
            dist.broadcast(module.arena, src=0)
            eng.refresh_shadow()
        # ready order = reverse arena order; one range per engine "ready" event
        self.reducer = BucketedReducer(eng.grad, self._ready_ranges(module), bucket_mb)
        self._sync = True
        eng.grad_sync = self._on_event

    @staticmethod
    def _ready_ranges(module):
        lay = module.layout
        L = module.config.n_layer
        total = lay.total
        starts = {n: s.offset for n, s in lay.slots.items()}
        order = []
        lnf_lo = starts["transformer.ln_f.weight"]
        order.append(("transformer.ln_f.bias", lnf_lo, total))
        hi = lnf_lo
        for l in reversed(range(L)):
            lo = starts[f"transformer.h.{l}.ln1.weight"]
            order.append((f"transformer.h.{l}.ln1.weight", lo, hi))
            hi = lo
        order.append(("transformer.wte.weight", 0, hi))
        return order

    def _on_event(self, event, name=None):
        if event == "ready" and self._sync:
            self.reducer.mark_ready(name)

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def finish_gradient_sync(self):
        """Wait for every bucket (called by the optimizer step wrapper / trainer)."""
        if self._sync:
            self.reducer.flush()

    def configure_optimizers(self, *a, **kw):
        opt = self.module.configure_optimizers(*a, **kw)
        return _SyncedOptimizer(opt, self)

    def state_dict(self, *a, **kw):
        return self.module.state_dict(*a, **kw)


class _SyncedOptimizer:
    """Optimizer proxy: step() first completes the gradient collective."""

    def __init__(self, opt, ddp):
        self.opt = opt
        self.ddp = ddp

    def step(self, closure=None):
        self.ddp.finish_gradient_sync()
        return self.opt.step(closure)

    def zero_grad(self, set_to_none=True):
        self.opt.zero_grad(set_to_none)

    def __getattr__(self, k):
        return getattr(self.opt, k)


class ShardedDataParallel(DistributedDataParallel):
    """ZeRO-style sharded optimizer over the arena (the build's --training_mode fsdp)."""

    def __init__(self, module, device_ids=None, bucket_mb: float = 64.0):
        super().__init__(module, device_ids, bucket_mb)
        W = dist.get_world_size()
        total = module.layout.total
        per = (total + W - 1) // W
        per = (per + 63) // 64 * 64
        self.per = per
        self.padded = per * W
        r = dist.get_rank()
        self.lo, self.hi = min(r * per, total), min((r + 1) * per, total)
        self.engine.grad_sync = None  # reduce-scatter happens at the end (one fused collective)

    def finish_gradient_sync(self):
        eng = self.engine
        W = dist.get_world_size()
        g = eng.grad
        if g.numel() < self.padded:
            raise RuntimeError("arena must be padded to the shard grid")
        inp = g[:self.padded]
        shard = torch.empty(self.per, dtype=g.dtype, device=g.device)
        op = dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM
        dist.reduce_scatter_tensor(shard, inp, op=op)
        if op == dist.ReduceOp.SUM:
            shard.mul_(1.0 / W)
        g[self.lo:self.hi].copy_(shard[:self.hi - self.lo])

    def configure_optimizers(self, weight_decay=0.1, learning_rate=1e-4, betas=(0.9, 0.95), device_type=None,
                             eps=1e-8):
        from .optim import FusedAdamW
        opt = FusedAdamW(self.module, lr=learning_rate, betas=betas, eps=eps, weight_decay=weight_decay,
                         shard=(self.lo, self.hi))
        return _ShardedOptimizer(opt, self)


class _ShardedOptimizer(_SyncedOptimizer):
    def step(self, closure=None):
        self.ddp.finish_gradient_sync()
        out = self.opt.step(closure)
        # the kernel's norm covers this rank's slice: the clip_grad_norm_ value is the global one
        # (train_gpt2_distributed.py:419-421 on the full grads)
        n2 = self.opt.grad_norm.square()
        dist.all_reduce(n2)
        self.opt.grad_norm.copy_(n2.sqrt())
        # all-gather the updated fp32 master slices, then refresh the bf16 shadow once
        m = self.ddp.module
        arena = m.arena
        shard = torch.zeros(self.ddp.per, dtype=arena.dtype, device=arena.device)
        n = self.ddp.hi - self.ddp.lo
        shard[:n].copy_(arena[self.ddp.lo:self.ddp.hi])
        full = torch.empty(self.ddp.padded, dtype=arena.dtype, device=arena.device)
        dist.all_gather_into_tensor(full, shard)
        arena.copy_(full[:arena.numel()])
        m.engine().refresh_shadow()
        return out
