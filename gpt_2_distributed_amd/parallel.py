"""Data parallelism over RCCL (torch.distributed "nccl" = RCCL on ROCm), one process per GPU.

Replaces the reference's ``DDP(model, device_ids=[device])`` / ``FSDP(model, ...)``
(train_gpt2_distributed.py:129-165) and ``init_process_group("nccl")`` (:50-59):

* ``init_distributed()``: same contract as the reference (env:// rendezvous from torchrun,
  ``LOCAL_RANK`` -> device).
* ``DistributedDataParallel(model)``: broadcasts the flat fp32 arena from rank 0 once (C2) and
  averages the flat fp32 grad arena in ``bucket_mb`` buckets (C4). Buckets are issued asynchronously
  from inside the engine's backward as soon as a contiguous arena range is final (blocks finish
  last-to-first, the embeddings at the very end), so RCCL runs on its own stream under the remaining
  backward kernels, and the backward does not return before every bucket is reduced: ``p.grad`` is the
  global average when ``loss.backward()`` returns, exactly as with torch DDP, so the reference loop's
  ``clip_grad_norm_`` / ``torch.optim.AdamW`` see final gradients. There is no per-forward buffer
  broadcast (C3): the build has no mask buffer. ``no_sync()`` skips the collective on non-final
  gradient-accumulation micro-steps.
* ``FullyShardedDataParallel(model)`` (``--training_mode fsdp``; ``ShardedDataParallel`` is an alias):
  the reference's FULL_SHARD wrapping with one unit per ``GPT2Block`` plus the root (C5). Each unit's
  flat parameter range is sharded 1/world per rank: the fp32 master shard (exposed as the wrapper's
  single ``flat_param``, like FSDP's FlatParameter with use_orig_params=False), its grad and the AdamW
  moments live only on the owning rank. In the forward the engine asks for each unit just before it
  reads it; the wrapper all-gathers that unit in the compute precision (bf16 under autocast, like
  MixedPrecision(param_dtype=bf16)) and has the following units' all-gathers already in flight on RCCL's
  stream (by default every remaining unit's, issued at the first unit: ``prefetch_depth``). In the backward each unit's gradient range is reduce-scattered (bf16
  under autocast, like reduce_dtype=bf16) the moment the engine marks it final, overlapped with the
  remaining backward. MI355X-first difference: a gathered unit stays resident until the next optimizer
  step (288 GB HBM holds every unit of every BASELINE model), so the backward does not re-gather it and
  gradient-accumulation micro-steps gather once per optimizer step; the math is FULL_SHARD's.

Gradient scaling: every collective is a SUM. A synced backward computes its gradients pre-divided by
world (``GradHooks.begin_backward``); gradients accumulated earlier (no_sync micro-steps, or an
accumulation without no_sync) are divided once before it. SUM then yields the average on any backend,
so the gloo-tested path is the RCCL path.

The bucketing / shard planning is engine-agnostic (``BucketedReducer``, ``plan_shards``), so it is
tested on CPU with gloo.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from .engine import GradHooks

SHARD_ALIGN = 64  # elements: 256-B aligned shard chunks (16-B vector kernels, RCCL chunking)


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


def use_collectives(world: int) -> bool:
    """Collectives run when world > 1. GPT2MI_FORCE_COLLECTIVES=1 also runs them in a world of one: a
    one-GPU box then drives the real RCCL calls (async all-reduce from the backward, all-gather /
    reduce-scatter on the wrapper's buffers) that the multi-GPU node runs."""
    return world > 1 or os.environ.get("GPT2MI_FORCE_COLLECTIVES") == "1"


def is_primary() -> bool:
    return dist.get_rank() == 0 if dist.is_initialized() else True


def unit_ranges(layout, n_layer: int) -> List[Tuple[str, int, int]]:
    """The FSDP units / DDP ready ranges of the arena, in arena order: "embed" (wte, wpe), "h.<l>" (one
    GPT2Block each: transformer_auto_wrap_policy({GPT2Block}), train_gpt2_distributed.py:146-161) and
    "head" (ln_f). The root unit of the reference is embed + head (two arena ranges)."""
    starts = {n: s.offset for n, s in layout.slots.items()}
    out = [("embed", 0, starts["transformer.h.0.ln1.weight"])]
    for l in range(n_layer):
        lo = starts[f"transformer.h.{l}.ln1.weight"]
        hi = starts[f"transformer.h.{l+1}.ln1.weight"] if l + 1 < n_layer else starts["transformer.ln_f.weight"]
        out.append((f"h.{l}", lo, hi))
    out.append(("head", starts["transformer.ln_f.weight"], layout.total))
    return out


def backward_order(units):
    """The order the engine marks ranges final: head, h.L-1 .. h.0, embed."""
    return [units[-1]] + list(reversed(units[1:-1])) + [units[0]]


class BucketedReducer:
    """SUM-all-reduces a flat gradient tensor across the group in contiguous buckets.

    ``order`` lists (name, lo, hi) ranges of ``flat`` in the order they become final during backward.
    ``mark_ready(name)`` is called when a range is final; once the ready-but-unsent span reaches
    ``bucket_bytes`` an async all-reduce of that span is issued. ``finish()`` issues the tail and makes
    the caller's stream wait for every bucket. Ranges must become ready so that the unsent span stays
    contiguous (true for reverse arena order)."""

    def __init__(self, flat: torch.Tensor, order: List[Tuple[str, int, int]], bucket_mb: float = 64.0, group=None):
        self.flat = flat
        self.order = order
        self.index = {n: i for i, (n, _, _) in enumerate(order)}
        self.bucket_elems = max(1, int(bucket_mb * 1024 * 1024 / flat.element_size()))
        self.group = group
        self.reset()

    def reset(self):
        self.next = 0           # next index in `order` not yet marked ready
        self.pending_lo = None  # unsent contiguous span [lo, hi)
        self.pending_hi = None
        self.works = []
        self.spans = []         # [lo, hi) of each issued bucket
        self.launched = 0       # buckets issued during the backward (before finish)

    def mark_ready(self, name: str):
        i = self.index[name]
        if i < self.next:
            return
        while self.next <= i:
            _, lo, hi = self.order[self.next]
            if self.pending_lo is None:
                self.pending_lo, self.pending_hi = lo, hi
            else:
                if not (hi <= self.pending_lo or lo >= self.pending_hi):
                    raise RuntimeError("BucketedReducer: overlapping ready ranges")
                if hi != self.pending_lo and lo != self.pending_hi:
                    raise RuntimeError("BucketedReducer: non-contiguous ready order")
                self.pending_lo = min(self.pending_lo, lo)
                self.pending_hi = max(self.pending_hi, hi)
            self.next += 1
        if self.pending_hi - self.pending_lo >= self.bucket_elems:
            self._launch()

    def _launch(self):
        if self.pending_lo is None:
            return
        span = self.flat[self.pending_lo:self.pending_hi]
        self.works.append(dist.all_reduce(span, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.spans.append((self.pending_lo, self.pending_hi))
        self.launched += 1
        self.pending_lo = self.pending_hi = None

    def finish(self, defer_last: bool = False):
        """Issue whatever is left, then make the current stream wait on every bucket (nccl: a stream
        wait, the host does not block; gloo: the host waits). defer_last: the last bucket (the embeddings, final only
        at the end of the backward) is left in flight and returned as (work, lo, hi) for the caller to wait on."""
        if self.next < len(self.order):
            self.mark_ready(self.order[-1][0])
        self._launch()
        works, tail = self.works, None
        if defer_last and works:
            tail = (works[-1],) + self.spans[-1]
            works = works[:-1]
        for w in works:
            w.wait()
        self.reset()
        return tail


class _DPHooks(GradHooks):
    """The gradient side shared by DDP and FSDP: 1/world pre-scaling and the no_sync switch."""

    def __init__(self, engine, world: int):
        self.engine = engine
        self.world = world
        self.coll = use_collectives(world)
        self.sync = True

    def begin_backward(self) -> float:
        if not self.sync or self.world == 1:
            return 1.0
        if self.engine.grad_dirty:  # gradients accumulated before this synced backward: divide them too
            from . import _lib as K
            K.scale_(self.engine.grad, 1.0 / self.world)
        return 1.0 / self.world


class _DDPHooks(_DPHooks):
    def __init__(self, engine, world, reducer):
        super().__init__(engine, world)
        self.reducer = reducer
        # DistributedDataParallel(overlap_optimizer=True) with the fused AdamW: the backward returns with its last bucket
        # (work, lo, hi) still in flight, and the optimizer updates every other range under it (optim.FusedAdamW.step)
        self.defer_tail = False
        self.tail = None

    def take_tail(self):
        t, self.tail = self.tail, None
        return t

    def wait_tail(self):
        """Make the current stream wait for a deferred last bucket (its gradients final from here on)."""
        t = self.take_tail()
        if t is not None:
            t[0].wait()

    def begin_backward(self) -> float:
        self.wait_tail()  # the next backward writes the deferred range again
        if self.sync and self.coll:
            # a backward that raised midway left buckets in flight and `next` past them: wait for those (their
            # spans are re-reduced by this backward anyway) and start over
            for w in self.reducer.works:
                w.wait()
            self.reducer.reset()
        return super().begin_backward()

    def inflight(self) -> bool:
        # from the first bucket on, RCCL runs under the rest of the backward (no persistent GEMM grid there); the
        # lm_head backward and the last blocks' backward before the first full bucket keep the persistent schedule
        # (a host-side event query: a bucket that reads complete is certainly done before anything enqueued now runs)
        return (self.sync and self.coll and any(not w.is_completed() for w in self.reducer.works)) or \
            (self.tail is not None and not self.tail[0].is_completed())

    def ready(self, name):
        if self.sync and self.coll:
            self.reducer.mark_ready(name)

    def end_backward(self):
        if self.sync and self.coll:
            self.tail = self.reducer.finish(defer_last=self.defer_tail)


class DistributedDataParallel(nn.Module):
    """DDP for the arena model: same call surface as torch DDP for the reference loop.

    ``bucket_mb`` defaults to torch DDP's ``bucket_cap_mb`` (25, the reference's DDP(model) at
    train_gpt2_distributed.py:163): at the GPT-2 widths every GPT2Block (28 MB fp32 at 124M) is its own bucket, so
    only the block-0 and embedding buckets follow the last backward kernels. ``overlap_optimizer=True`` (bench.py,
    the trainer): with this wrapper's ``configure_optimizers`` AdamW, the backward returns with the embedding bucket
    still in flight and the optimizer step updates every other range under it — the embedding gradients are then
    final only after ``optimizer.step()`` or ``finish_gradient_sync()`` (torch DDP semantics, the default, make them
    final when ``loss.backward()`` returns)."""

    def __init__(self, module, device_ids=None, bucket_mb: float = 25.0, broadcast: bool = True,
                 overlap_optimizer: bool = False):
        super().__init__()
        self.module = module
        self.overlap_optimizer = overlap_optimizer
        eng = module.engine()
        self.engine = eng
        world = dist.get_world_size()
        if broadcast and use_collectives(world):
            dist.broadcast(module.arena, src=0)
            eng.refresh_shadow()
        units = unit_ranges(module.layout, module.config.n_layer)
        self.reducer = BucketedReducer(eng.grad, backward_order(units), bucket_mb)
        self.hooks = _DDPHooks(eng, world, self.reducer)
        eng.grad_sync = self.hooks

    @contextlib.contextmanager
    def no_sync(self):
        old = self.hooks.sync
        self.hooks.sync = False
        try:
            yield
        finally:
            self.hooks.sync = old

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def finish_gradient_sync(self):
        """Make the gradients final on the current stream: a no-op unless overlap_optimizer left the last bucket in
        flight (the backward itself completes every other bucket)."""
        self.hooks.wait_tail()

    def configure_optimizers(self, *a, **kw):
        opt = self.module.configure_optimizers(*a, **kw)
        if self.overlap_optimizer:
            from .optim import FusedAdamW
            if isinstance(opt, FusedAdamW):  # the only optimizer that waits for a deferred bucket itself
                opt.attach_tail(self.hooks)
                self.hooks.defer_tail = True
        return opt

    def state_dict(self, *a, **kw):
        return self.module.state_dict(*a, **kw)


# --------------------------------------------------------------------------------------------------
# FSDP
# --------------------------------------------------------------------------------------------------
@dataclass
class ShardPlan:
    name: str
    lo: int          # arena range of the unit
    hi: int
    per: int         # elements per rank (padded)
    soff: int        # offset of this unit's chunk in every rank's shard arena

    @property
    def n(self):
        return self.hi - self.lo


def plan_shards(units, world: int, align: int = SHARD_ALIGN) -> Tuple[List[ShardPlan], int]:
    """Every unit's range split into `world` equal chunks of `per` elements (rank r owns unit elements
    [r*per, (r+1)*per), zero-padded past the unit's end); any world size (3, 6, 12 ...) works."""
    plans, off = [], 0
    for name, lo, hi in units:
        per = -(-(hi - lo) // world)
        per = -(-per // align) * align
        plans.append(ShardPlan(name, lo, hi, per, off))
        off += per
    return plans, off


class _FSDPHooks(_DPHooks):
    def __init__(self, fsdp, world):
        super().__init__(fsdp.engine, world)
        self.fsdp = fsdp

    def begin_backward(self) -> float:
        self.fsdp.wait_tail()  # the next backward packs and reduce-scatters the deferred unit again
        return super().begin_backward()

    def ready(self, name):
        if self.sync:
            self.fsdp._reduce_scatter(name)

    def end_backward(self):
        if self.sync:
            self.fsdp._finish_reduce()

    def fwd_unit(self, unit):
        self.fsdp._gather_for(unit)

    def inflight(self) -> bool:
        # an all-gather or reduce-scatter this wrapper issued has not completed yet (a host-side event query: when it
        # reads complete, the collective is certainly done before anything enqueued now runs; while the host runs ahead
        # of the GPU it may read pending for one that will be done by then, which only costs the persistent schedule)
        f = self.fsdp
        if not f.coll:
            return False
        return any(w is not None and u not in f._fenced and not w.is_completed() for u, (w, _) in f._pending.items()) or \
            any(w is not None and not w.is_completed() for _, w, _ in f._rs_works) or \
            (f._tail is not None and f._tail[1] is not None and not f._tail[1].is_completed())


class FullyShardedDataParallel(nn.Module):
    """FULL_SHARD data parallelism over per-GPT2Block units (see the module docstring)."""

    # the forward unit (index in arena order: embed, h.0, h.1, h.2, ...) at which every pending all-gather is waited for
    FENCE_UNIT = 3

    def __init__(self, module, device_ids=None, bucket_mb: float = 64.0, prefetch: bool = True,
                 prefetch_depth: Optional[int] = None, overlap_optimizer: bool = False):
        super().__init__()
        self.module = module
        # overlap_optimizer (with configure_optimizers' ShardedAdamW): the backward returns with the last unit's
        # reduce-scatter (the embeddings, final only after the embedding backward) in flight, and the optimizer updates
        # every other unit under it; flat_param.grad of that unit is final after optimizer.step() or
        # finish_gradient_sync() (by default it is final when loss.backward() returns)
        self.overlap_optimizer = overlap_optimizer
        self._defer_tail = False
        self._tail = None  # (unit, work, out, accumulate) of the deferred reduce-scatter
        eng = module.engine()
        self.engine = eng
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.prefetch = prefetch
        # units gathered ahead of the one being computed (None: every remaining unit at the first unit's forward, so the
        # gathers finish under the first blocks and the rest of the forward runs with no collective in flight; a
        # gathered unit stays resident until the next optimizer step either way, so depth costs no memory)
        self.prefetch_depth = prefetch_depth
        W, r = self.world, self.rank
        self.coll = use_collectives(W)
        if self.coll:
            dist.broadcast(module.arena, src=0)
        self.units = unit_ranges(module.layout, module.config.n_layer)
        self.plans, self.shard_total = plan_shards(self.units, W)
        self.plan = {p.name: p for p in self.plans}
        self.order = [p.name for p in self.plans]  # forward order = arena order
        dev = module.arena.device
        master = torch.zeros(self.shard_total, dtype=torch.float32, device=dev)
        for p in self.plans:  # this rank's chunk of every unit
            a, b = p.lo + r * p.per, min(p.hi, p.lo + (r + 1) * p.per)
            if b > a:
                master[p.soff:p.soff + b - a].copy_(module.arena[a:b])
        # FSDP's FlatParameter (use_orig_params=False): the only parameter the wrapper exposes
        self.flat_param = nn.Parameter(master)
        self.grad_shard = torch.zeros_like(master)
        self._bufs: Dict[tuple, torch.Tensor] = {}
        self._valid: Dict[str, Optional[torch.dtype]] = {u: None for u in self.order}
        self._pending: Dict[str, tuple] = {}       # unit -> (work, dtype) of an in-flight all-gather
        # pending all-gathers the compute stream already waits for (fenced at unit FENCE_UNIT of the forward): no kernel
        # enqueued after the fence can overlap them, so they do not count as in flight for the GEMM schedule
        self._fenced = set()
        self._rs_works: List[tuple] = []            # (unit, work, out) of in-flight reduce-scatters
        # every unit's bf16_chunk == bf16(its flat_param range) (set by our AdamW, which writes them)
        self._bf16_fresh = False
        self._seen_version = None
        self.hooks = _FSDPHooks(self, W)
        # a torch optimizer on flat_param (fused AdamW does not bump its version): every gathered unit goes stale
        from .engine import watch_optimizer_steps
        watch_optimizer_steps(self, [self.flat_param], FullyShardedDataParallel._stale_after_step)
        eng.grad_sync = self.hooks
        eng.param_provider = self.hooks
        eng.zero_grad()
        eng.bind_grads()

    # ---- parameters: the flat shard only (torch optimizers / clip_grad_norm_ see what FSDP exposes) ----
    def parameters(self, recurse: bool = True):
        yield self.flat_param

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):
        yield (prefix + ("." if prefix else "") + "flat_param", self.flat_param)

    def memory_report(self) -> dict:
        """Bytes per rank: sharded state (fp32 master, grad, AdamW moments, bf16 AG source) vs the
        resident compute views (fp32 params, bf16 shadow + transposed shadow, transient fp32 grad arena,
        collective staging). DDP keeps every one of the sharded tensors whole."""
        n_full = self.module.arena.numel()
        sharded = self.shard_total * (4 + 4 + 8 + 2)
        views = n_full * (4 + 2 + 2 + 4)
        staging = sum(t.numel() * t.element_size() for t in self._bufs.values())
        return {"params": n_full, "world": self.world, "sharded_state_bytes": sharded,
                "ddp_equivalent_state_bytes": n_full * (4 + 4 + 8),
                "compute_view_bytes": views, "staging_bytes": staging}

    # ---- buffers ------------------------------------------------------------------------------------
    def _buf(self, kind, unit, dtype, n):
        key = (kind, unit, dtype)
        t = self._bufs.get(key)
        if t is None:
            t = torch.empty(n, dtype=dtype, device=self.flat_param.device)
            self._bufs[key] = t
        return t

    def bf16_chunk(self, unit) -> torch.Tensor:
        """This rank's bf16 shard of ``unit``: its chunk of the unit's all-gather buffer, so the bf16 gather runs in
        place (RCCL copies nothing locally; at one rank the gathered unit IS the shard). The optimizer writes it."""
        p = self.plan[unit]
        return self._buf("ag", unit, torch.bfloat16, p.per * self.world)[self.rank * p.per:(self.rank + 1) * p.per]

    # ---- forward: per-unit all-gather with prefetch ---------------------------------------------------
    def mark_params_updated(self, bf16_fresh: bool):
        """Called after an optimizer step on flat_param (our AdamW also wrote every bf16_chunk)."""
        self._valid = {u: None for u in self.order}
        self._bf16_fresh = bf16_fresh
        self._seen_version = self.flat_param._version

    def _stale_after_step(self):
        self._seen_version = None  # _check_version then treats every gathered unit as stale

    def _check_version(self):
        if self._seen_version is None or self.flat_param._version != self._seen_version:
            # a step we did not see (torch optimizer, load): every gathered unit is stale
            self._valid = {u: None for u in self.order}
            self._bf16_fresh = False
            self._seen_version = self.flat_param._version

    def _issue_gather(self, unit, dtype):
        from . import _lib as K
        p = self.plan[unit]
        out = self._buf("ag", unit, dtype, p.per * self.world)
        if dtype == torch.bfloat16:
            if not self._bf16_fresh:  # a step we did not run (torch optimizer, load): re-round every shard
                fp = self.flat_param.detach()
                for q in self.plans:
                    K.cast_f32_bf16(fp[q.soff:q.soff + q.per], self.bf16_chunk(q.name), q.per)
                self._bf16_fresh = True
            src = self.bf16_chunk(unit)  # in place: a view of out
        else:
            src = self.flat_param.detach()[p.soff:p.soff + p.per]
        if not self.coll:
            if src.data_ptr() != out.data_ptr():
                out.copy_(src)
            work = None
        else:
            work = dist.all_gather_into_tensor(out, src, async_op=True)
        self._pending[unit] = (work, dtype)
        self._fenced.discard(unit)  # a new gather of the unit: not waited for yet

    def _gather_for(self, unit):
        from . import _lib as K
        eng = self.engine
        dtype = eng.compute_dtype()
        self._check_version()
        if self._valid.get(unit) != dtype:
            if unit not in self._pending or self._pending[unit][1] != dtype:
                self._issue_gather(unit, dtype)
        if self.prefetch:  # the next units' all-gathers ride under this unit's compute
            i = self.order.index(unit)
            last = len(self.order) if self.prefetch_depth is None else min(len(self.order), i + 1 + self.prefetch_depth)
            for nxt in self.order[i + 1:last]:
                if self._valid.get(nxt) != dtype and nxt not in self._pending:
                    self._issue_gather(nxt, dtype)
        if self.coll and self.order.index(unit) >= min(self.FENCE_UNIT, len(self.order) - 1):
            # every gather still pending is waited for here (a stream wait): they were issued at the first unit and are
            # done by now at any world size, so this costs nothing, and the rest of the forward's GEMMs keep the static
            # persistent schedule (GradHooks.inflight) instead of the work-queue variant
            for u, (w, _) in self._pending.items():
                if w is not None and u not in self._fenced:
                    w.wait()
                    self._fenced.add(u)
        if self._valid.get(unit) == dtype:
            return
        work, _ = self._pending.pop(unit)
        if work is not None and unit not in self._fenced:
            work.wait()
        self._fenced.discard(unit)
        p = self.plan[unit]
        out = self._buf("ag", unit, dtype, p.per * self.world)
        bf = eng.shadow[p.lo:p.hi] if dtype == torch.bfloat16 else None
        K.fsdp_unpack(out, self.module.arena[p.lo:p.hi], bf, p.n)
        if dtype == torch.bfloat16:
            names = [n for n, s in self.module.layout.slots.items() if p.lo <= s.offset < p.hi]
            eng.refresh_shadowT(names)
        self._valid[unit] = dtype

    # ---- backward: per-unit reduce-scatter as ranges become final ----------------------------------------
    def _reduce_scatter(self, unit):
        from . import _lib as K
        p = self.plan[unit]
        eng = self.engine
        dtype = eng.bwd_act  # reduce_dtype = the compute precision (bf16 under autocast)
        inp = self._buf("rs_in", unit, dtype, p.per * self.world)
        K.fsdp_pack(eng.grad[p.lo:p.hi], inp, p.n, p.per * self.world)
        # in place: this rank's chunk of the packed input receives the reduced shard (RCCL copies nothing locally)
        out = inp[self.rank * p.per:(self.rank + 1) * p.per]
        if not self.coll:
            work = None
        else:
            work = dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, async_op=True)
        self._rs_works.append((unit, work, out))

    def _finish_reduce(self):
        from . import _lib as K
        done = {u for u, _, _ in self._rs_works}
        for u in self.order:  # ranges the engine did not mark (e.g. a sub-module backward): reduce them too
            if u not in done:
                self._reduce_scatter(u)
        # the packed inputs hold this backward's gradients: the full arena restarts from zero (lazily: the next
        # backward's weight-gradient GEMMs write their slots and only the rest is zeroed, Engine.discard_grads)
        self.engine.discard_grads()
        # accumulate only into a gradient the caller still holds: after a torch optimizer's
        # zero_grad(set_to_none=True) flat_param.grad is None and the shard's old values are stale
        acc = self.flat_param.grad is self.grad_shard
        works = self._rs_works
        if self._defer_tail and self.coll and works:
            u, work, out = works[-1]
            self._tail = (u, work, out, acc)
            works = works[:-1]
        for u, work, out in works:
            if work is not None:
                work.wait()
            p = self.plan[u]
            K.fsdp_accum(out, self.grad_shard[p.soff:p.soff + p.per], p.per, accumulate=acc)
        self._rs_works = []
        self.flat_param.grad = self.grad_shard

    def tail_unit(self) -> Optional[str]:
        """The unit whose reduce-scatter overlap_optimizer left in flight (None if none)."""
        return self._tail[0] if self._tail is not None else None

    def wait_tail(self):
        """Complete a deferred reduce-scatter: the current stream waits for it and accumulates its shard."""
        from . import _lib as K
        t, self._tail = self._tail, None
        if t is not None:
            u, work, out, acc = t
            if work is not None:
                work.wait()
            p = self.plan[u]
            K.fsdp_accum(out, self.grad_shard[p.soff:p.soff + p.per], p.per, accumulate=acc)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.hooks.sync
        self.hooks.sync = False
        try:
            yield
        finally:
            self.hooks.sync = old

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def finish_gradient_sync(self):
        """Make the gradient shard final on the current stream: a no-op unless overlap_optimizer left the last unit's
        reduce-scatter in flight (the backward itself completes every other one)."""
        self.wait_tail()

    def zero_grad(self, set_to_none: bool = True):
        from . import _lib as K
        self.wait_tail()  # its accumulate writes the shard; its reduce-scatter the unit's packing buffer
        if set_to_none:  # the next backward writes the shard instead of adding to it (_finish_reduce)
            self.flat_param.grad = None
        else:
            K.zero_(self.grad_shard)
            self.flat_param.grad = self.grad_shard
        self.engine.discard_grads()

    def configure_optimizers(self, weight_decay=0.1, learning_rate=1e-4, betas=(0.9, 0.95), device_type=None,
                             eps=1e-8):
        from .optim import ShardedAdamW
        self._defer_tail = self.overlap_optimizer  # ShardedAdamW.step waits for the deferred unit itself
        return ShardedAdamW(self, lr=learning_rate, betas=betas, eps=eps, weight_decay=weight_decay)

    # ---- full state (checkpointing): collective, every rank calls --------------------------------------
    @torch.no_grad()
    def full_arena(self) -> torch.Tensor:
        """The fp32 master parameters of every unit, all-gathered (FULL_STATE_DICT; fixes the reference's
        rank-0-only early return before this collective, train_gpt2_distributed.py:81-94)."""
        arena = torch.zeros_like(self.module.arena)
        for p in self.plans:
            src = self.flat_param.detach()[p.soff:p.soff + p.per]
            out = torch.empty(p.per * self.world, dtype=torch.float32, device=arena.device)
            if not self.coll:
                out.copy_(src)
            else:
                dist.all_gather_into_tensor(out, src)
            arena[p.lo:p.hi].copy_(out[:p.n])
        return arena

    def state_dict(self, *a, **kw):
        arena = self.full_arena()
        lay = self.module.layout
        return {n: lay.view(arena, n).clone() for n in self.module.state_dict()
                if n in lay.slots} | ({"lm_head.weight": lay.view(arena, "transformer.wte.weight").clone()}
                                      if "lm_head.weight" in self.module.state_dict() else {})

    @torch.no_grad()
    def load_full_state_dict(self, sd):
        m = self.module
        for n, p in m.named_parameters():
            p.copy_(sd[n])
        for pl in self.plans:
            a, b = pl.lo + self.rank * pl.per, min(pl.hi, pl.lo + (self.rank + 1) * pl.per)
            chunk = self.flat_param.detach()[pl.soff:pl.soff + pl.per]
            chunk.zero_()
            if b > a:
                chunk[:b - a].copy_(m.arena[a:b])
        self.mark_params_updated(False)
        self._seen_version = None  # force a refresh at the next forward


ShardedDataParallel = FullyShardedDataParallel
