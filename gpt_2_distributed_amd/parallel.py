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
  stream, as many as fit a byte budget of gathered output (``prefetch_bytes``, like FSDP's ``limit_all_gathers``
  rate limiter; ``prefetch_depth`` caps it by a unit count). In the backward each unit's gradient range is reduce-scattered (bf16
  under autocast, like reduce_dtype=bf16) the moment the engine marks it final, overlapped with the
  remaining backward. By default (``reshard_after_forward=True``, torch FSDP's FULL_SHARD default, which the
  reference runs) each block unit's gathered parameters are released after its forward and gathered again for
  its backward, so per-rank memory falls with the world size. ``reshard_after_forward=False`` is the MI355X
  resident mode: a gathered unit stays until the next optimizer step (288 GB HBM holds every unit of every
  BASELINE model), so the backward does not re-gather it and gradient-accumulation micro-steps gather once per
  optimizer step; the math is FULL_SHARD's either way.

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

    def bwd_unit(self, unit):
        if self.fsdp.store is not None:
            self.fsdp._bwd_unit(unit)

    def inflight(self) -> bool:
        # an all-gather or reduce-scatter this wrapper issued has not completed yet (a host-side event query: when it
        # reads complete, the collective is certainly done before anything enqueued now runs; while the host runs ahead
        # of the GPU it may read pending for one that will be done by then, which only costs the persistent schedule)
        f = self.fsdp
        if not f.coll:
            return False
        return any(w is not None and u not in f._fenced and not w.is_completed() for u, (w, *_) in f._pending.items()) or \
            any(w is not None and not w.is_completed() for _, w, _ in f._rs_works) or \
            (f._tail is not None and f._tail[1] is not None and not f._tail[1].is_completed())


def fsdp_memory_plan(units, world: int, reshard: bool) -> dict:
    """Per-rank bytes of FullyShardedDataParallel over ``units`` (unit_ranges) at ``world`` ranks, bf16 autocast:
    sharded state (fp32 master, grad, two AdamW moments, bf16 shard: 18 B per sharded element), compute views and
    collective staging. Resident: every unit's views (12 B/param: fp32 params + bf16 shadow + W^T + fp32 grads) and
    every unit's bf16 gather / reduce-scatter buffers. reshard_after_forward: the root unit's views, _ReshardStore's
    P_SLOTS parameter slots (8 B/param of a block) and G_SLOTS gradient slots (4 B), STAGE_SLOTS-deep bf16 gather and
    reduce-scatter rings of one block plus the root's own buffers, and a bf16 reduce-scatter output per unit."""
    plans, shard_total = plan_shards(units, world)
    sharded = shard_total * (4 + 4 + 8 + 2)
    total = units[-1][2]
    if not reshard:
        views = total * (4 + 2 + 2 + 4)
        # each unit's bf16 gather buffer less this rank's chunk of it (the bf16 shard, in the sharded state) + its bf16
        # reduce-scatter input
        staging = sum(p.per * (world - 1) * 2 + p.per * world * 2 for p in plans)
    else:
        root = [p for p in plans if p.name in ("embed", "head")]
        blocks = [p for p in plans if p.name not in ("embed", "head")]
        nb = max((p.n for p in blocks), default=0)
        per_b = max((p.per for p in blocks), default=0)
        views = sum(p.n for p in root) * (4 + 2 + 2 + 4) + \
            _ReshardStore.P_SLOTS * nb * (4 + 2 + 2) + _ReshardStore.G_SLOTS * nb * 4
        # the block gather and reduce-scatter rings, the root's own gather and reduce-scatter buffers, and each block's
        # reduced bf16 shard (the bf16 shard itself is in the sharded state)
        staging = 2 * FullyShardedDataParallel.STAGE_SLOTS * per_b * world * 2 + \
            sum(p.per * world for p in root) * (2 + 2) + sum(p.per for p in blocks) * 2
    return {"sharded_state_bytes": sharded, "compute_view_bytes": views, "staging_bytes": staging,
            "total": sharded + views + staging}


class _ReshardStore:
    """FullyShardedDataParallel(reshard_after_forward=True): where the engine's parameter, shadow and gradient views
    live (Engine.store). The root unit (embed + head: wte, wpe, ln_f; used at both ends of the step, and kept gathered
    as torch FSDP keeps its root) has compact resident storage. Every GPT2Block unit borrows one of P_SLOTS parameter
    slots (fp32 parameters, bf16 shadow, bf16 W^T) while it is gathered — the forward of the next units and the
    backward evict it, so the backward gathers it again — and one of G_SLOTS gradient slots from the start of its
    backward until its reduce-scatter has packed the gradient. The compute views are then root + 2 blocks of
    parameters + 3 blocks of gradients per rank instead of the whole model, and the per-rank total shrinks with the
    world size (memory_report). Slot reuse is safe in stream order: a slot is refilled only after every kernel that
    reads its previous unit has been enqueued on the compute stream."""

    P_SLOTS = 2
    G_SLOTS = 3

    def __init__(self, fsdp):
        from . import _lib as K
        eng, lay, plan = fsdp.engine, fsdp.module.layout, fsdp.plan
        dev = fsdp.flat_param.device
        self.K, self.eng, self.plan = K, eng, plan
        e, h = plan["embed"], plan["head"]
        self.root_base = {"embed": e.lo, "head": h.lo - e.n}  # head stored right after embed
        nr = e.n + h.n
        kinds = (("p", torch.float32), ("w16", torch.bfloat16), ("wT", torch.bfloat16), ("g", torch.float32))
        self.root = {k: torch.zeros(nr, dtype=dt, device=dev) for k, dt in kinds}
        self.blocks = [u for u in fsdp.order if u not in self.root_base]
        self.nb = max(plan[u].n for u in self.blocks) if self.blocks else 0
        self.pslots = [{k: torch.zeros(self.nb, dtype=dt, device=dev) for k, dt in kinds[:3]}
                       for _ in range(self.P_SLOTS)]
        self.gslots = [torch.zeros(self.nb, dtype=torch.float32, device=dev) for _ in range(self.G_SLOTS)]
        self.p_of: Dict[str, int] = {}
        self.p_owner: List[Optional[str]] = [None] * self.P_SLOTS
        self.p_next = 0
        self.g_of: Dict[str, int] = {}
        self.g_owner: List[Optional[str]] = [None] * self.G_SLOTS
        self.unit_of = {}
        for name, sl in lay.slots.items():
            self.unit_of[name] = next(u for u in fsdp.order if plan[u].lo <= sl.offset < plan[u].hi)
        dt = torch.int64
        self.acc_root = torch.tensor(eng.acc_ranges(e.lo, e.hi, 0) + eng.acc_ranges(h.lo, h.hi, e.n), dtype=dt).to(dev)
        self.acc_block = {u: torch.tensor(eng.acc_ranges(plan[u].lo, plan[u].hi), dtype=dt).to(dev)
                          for u in self.blocks}
        self.fresh = False
        self.evicted = None  # callback(unit): a block unit lost its parameter slot

    # -- the engine's views --
    def loc(self, kind, name):
        u = self.unit_of[name]
        if u in self.root_base:
            return self.root[kind], self.root_base[u]
        if kind == "g":
            i = self.g_of.get(u)
            if i is None:
                raise RuntimeError(f"reshard_after_forward: {u} has no gradient slot (its backward has not started)")
            return self.gslots[i], self.plan[u].lo
        i = self.p_of.get(u)
        if i is None:
            raise RuntimeError(f"reshard_after_forward: {u} is not gathered")
        return self.pslots[i][kind], self.plan[u].lo

    # -- parameter slots --
    def take_pslot(self, u) -> dict:
        """The parameter slot of block unit u (its own if it still has one, else the next one round-robin, evicting
        its previous unit)."""
        i = self.p_of.get(u)
        if i is None:
            i = self.p_next
            self.p_next = (i + 1) % self.P_SLOTS
            old = self.p_owner[i]
            if old is not None:
                del self.p_of[old]
                if self.evicted is not None:
                    self.evicted(old)
            self.p_owner[i] = u
            self.p_of[u] = i
        return self.pslots[i]

    def unit_params(self, u):
        """(fp32, bf16, W^T storage, arena element of storage element 0) for unpacking gathered unit u."""
        p = self.plan[u]
        if u in self.root_base:
            o = p.lo - self.root_base[u]
            return self.root["p"][o:o + p.n], self.root["w16"][o:o + p.n], self.root["w16"], self.root["wT"], \
                self.root_base[u]
        sl = self.take_pslot(u)
        return sl["p"][:p.n], sl["w16"][:p.n], sl["w16"], sl["wT"], p.lo

    # -- gradient slots --
    def begin_grads(self, fresh: bool):
        """A backward starts: its gradients start from zero (the weight-gradient GEMMs write their slots when fresh,
        every other range is zeroed)."""
        self.fresh = fresh
        self.g_of.clear()
        self.g_owner = [None] * self.G_SLOTS
        if fresh:
            self.K.zero_ranges(self.root["g"], self.acc_root)
        else:
            self.K.zero_(self.root["g"])

    def take_gslot(self, u):
        if u in self.root_base or u in self.g_of:
            return
        i = next((k for k, o in enumerate(self.g_owner) if o is None), None)
        if i is None:
            raise RuntimeError("reshard_after_forward: every gradient slot is in use")
        self.g_owner[i] = u
        self.g_of[u] = i
        g = self.gslots[i]
        if self.fresh:
            self.K.zero_ranges(g, self.acc_block[u])
        else:
            self.K.zero_(g)

    def release_gslot(self, u):
        i = self.g_of.pop(u, None)
        if i is not None:
            self.g_owner[i] = None

    def unit_grad(self, u) -> torch.Tensor:
        p = self.plan[u]
        if u in self.root_base:
            o = p.lo - self.root_base[u]
            return self.root["g"][o:o + p.n]
        return self.gslots[self.g_of[u]][:p.n]

    def view_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.root.values()) + \
            sum(t.numel() * t.element_size() for sl in self.pslots for t in sl.values()) + \
            sum(t.numel() * t.element_size() for t in self.gslots)


class FullyShardedDataParallel(nn.Module):
    """FULL_SHARD data parallelism over per-GPT2Block units (see the module docstring)."""

    # gathered bytes (the all-gathers' outputs, every rank's chunk) in flight ahead of the unit being computed: a GPT-2
    # 124M block is 14 MB in bf16, 350M 25 MB, 1.5B 61 MB, so 512 MiB keeps the whole 124M model, 20 350M blocks or 8
    # 1.5B blocks ahead (at 8 ranks a 1.5B block takes ~0.4 ms of ring all-gather over xGMI against ~1.4 ms of forward
    # compute per block at B = 32), and bounds what a rank receives before it computes
    PREFETCH_BYTES = 512 << 20

    def __init__(self, module, device_ids=None, bucket_mb: float = 64.0, prefetch: bool = True,
                 prefetch_depth: Optional[int] = None, overlap_optimizer: bool = False,
                 prefetch_bytes: Optional[int] = None, reshard_after_forward: bool = True):
        super().__init__()
        self.module = module
        # reshard_after_forward: FULL_SHARD's memory behaviour (torch FSDP's default for FULL_SHARD, which the
        # reference runs, train_gpt2_distributed.py:146-161; the default here too): a GPT2Block unit's gathered
        # parameters are released after its forward and gathered again for its backward, its gradient lives only until
        # its reduce-scatter, and the full-model compute views are freed (_ReshardStore). Off: every gathered unit stays
        # resident until the next optimizer step (no re-gather: 288 GB holds every BASELINE model's views).
        self.reshard_after_forward = bool(reshard_after_forward)
        self.store: Optional[_ReshardStore] = None
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
        # the all-gathers kept in flight ahead of the unit being computed: as many following units as fit
        # prefetch_bytes of gathered output (None: PREFETCH_BYTES), at most prefetch_depth units (None: no unit cap);
        # each unit's forward first retires the gathers that have completed (an event query), and waits only for its
        # own, so the GEMMs run the static persistent schedule exactly while no gather is in flight (GradHooks.inflight)
        self.prefetch_depth = prefetch_depth
        self.prefetch_bytes = self.PREFETCH_BYTES if prefetch_bytes is None else int(prefetch_bytes)
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
        # pending all-gathers the compute stream already waits for (retired once their event reads complete): no
        # kernel enqueued after that wait can overlap them, so they do not count as in flight for the GEMM schedule
        self._fenced = set()
        self._rs_works: List[tuple] = []            # (unit, work, out) of in-flight reduce-scatters
        # every unit's bf16_chunk == bf16(its flat_param range) (set by our AdamW, which writes them)
        self._bf16_fresh = False
        self._compute_dtype: Optional[torch.dtype] = None  # of the latest forward (None before the first)
        self._stage_next = {}                      # reshard: next slot of each staging ring
        self._stage_user: Dict[tuple, Optional[str]] = {}  # reshard: (ring, slot) -> unit whose data it holds
        self._rs_slot_work: Dict[int, object] = {}  # reshard: rs ring slot -> the reduce-scatter that reads it
        self._seen_version = None
        self.hooks = _FSDPHooks(self, W)
        # a torch optimizer on flat_param (fused AdamW does not bump its version): every gathered unit goes stale
        from .engine import watch_optimizer_steps
        watch_optimizer_steps(self, [self.flat_param], FullyShardedDataParallel._stale_after_step)
        eng.grad_sync = self.hooks
        eng.param_provider = self.hooks
        eng.zero_grad()
        eng.bind_grads()
        if self.reshard_after_forward:
            self.store = _ReshardStore(self)
            self.store.evicted = self._evicted
            eng.store = self.store
            # the full-model views are freed (as FSDP frees the unsharded FlatParameter): the module's own parameters
            # keep their shapes but no storage; every view the engine forms comes from the store. Their .grad views
            # pointed into the freed grad arena, so they are dropped: the inner module's parameters then read as
            # torch FSDP's do after resharding (no gradient; data without storage), and what a caller uses is the
            # wrapper's flat_param / state_dict()
            for prm in eng.params_by_name.values():
                prm.grad = None
            for t in (module.arena, eng.shadow, eng.shadowT, eng.grad):
                t.untyped_storage().resize_(0)

    # ---- parameters: the flat shard only (torch optimizers / clip_grad_norm_ see what FSDP exposes) ----
    def parameters(self, recurse: bool = True):
        yield self.flat_param

    def named_parameters(self, prefix: str = "", recurse: bool = True, remove_duplicate: bool = True):
        yield (prefix + ("." if prefix else "") + "flat_param", self.flat_param)

    def memory_report(self) -> dict:
        """Bytes per rank: sharded state (fp32 master, grad, AdamW moments, bf16 AG source) vs the compute views (fp32
        params, bf16 shadow + transposed shadow, transient fp32 gradients) and the collective staging, as allocated now;
        ``per_rank_bytes_by_world``: the same model at other world sizes (fsdp_memory_plan). DDP keeps every one of the
        sharded tensors whole. Resident mode: the views cover the whole model on every rank; reshard_after_forward: the
        root unit plus the store's block slots, so the per-rank total falls with the world size."""
        n_full = self.module.layout.total
        rs = self.store is not None
        views = self.store.view_bytes() if rs else n_full * (4 + 2 + 2 + 4)
        # staging: every collective buffer except the bf16 shard, which sharded_state_bytes counts (18 B/element): the
        # resharded mode's "shard16" buffer, or in the resident mode this rank's chunk of each bf16 gather buffer
        staging = 0
        for (kind, unit, dtype), t in self._bufs.items():
            if kind == "shard16":
                continue
            n = t.numel()
            if kind == "ag" and dtype == torch.bfloat16 and not rs:
                n -= self.plan[unit].per
            staging += n * t.element_size()
        return {"params": n_full, "world": self.world, "reshard_after_forward": rs,
                "sharded_state_bytes": self.shard_total * (4 + 4 + 8 + 2),
                "ddp_equivalent_state_bytes": n_full * (4 + 4 + 8),
                "compute_view_bytes": views,
                "staging_bytes": staging,
                "plan": fsdp_memory_plan(self.units, self.world, rs),  # the same rank priced (activations excluded)
                "per_rank_bytes_by_world": {w: fsdp_memory_plan(self.units, w, rs)["total"] for w in (1, 2, 4, 8)}}

    # ---- buffers ------------------------------------------------------------------------------------
    def _buf(self, kind, unit, dtype, n):
        key = (kind, unit, dtype)
        t = self._bufs.get(key)
        if t is None:
            t = torch.empty(n, dtype=dtype, device=self.flat_param.device)
            self._bufs[key] = t
        return t

    def bf16_chunk(self, unit) -> torch.Tensor:
        """This rank's bf16 shard of ``unit``. Resident mode: its chunk of the unit's all-gather buffer, so the bf16
        gather runs in place (RCCL copies nothing locally; at one rank the gathered unit IS the shard).
        reshard_after_forward: its range of one shard-sized bf16 buffer (the gathers go to staging rings). The
        optimizer writes it."""
        p = self.plan[unit]
        if self.store is not None:
            return self._buf("shard16", None, torch.bfloat16, self.shard_total)[p.soff:p.soff + p.per]
        return self._buf("ag", unit, torch.bfloat16, p.per * self.world)[self.rank * p.per:(self.rank + 1) * p.per]

    def wants_bf16(self) -> bool:
        """The optimizer should write the bf16 shards: the latest forward computed in bf16 (autocast), or none ran yet.
        In fp32 mode no bf16 gather buffer is allocated or written (a later bf16 forward re-rounds every shard)."""
        return self._compute_dtype in (None, torch.bfloat16)

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

    # reshard_after_forward: staging rings (block units' gathers and reduce-scatter inputs); a slot is refilled only
    # after its previous unit's consumer (the unpack, or the reduce-scatter) is enqueued / waited for
    STAGE_SLOTS = 3

    def _ring(self, ring, dtype, n):
        """The next slot of staging ring ``ring`` (STAGE_SLOTS buffers of n elements): (index, buffer). A gather
        ring's slot is handed out only when the unit it holds has been unpacked (no longer pending), a reduce-scatter
        ring's only when the reduce-scatter that read it has been waited for: refilling it earlier would overwrite
        bytes a collective or the unpack still reads (the ordering argument is in stream order: ProcessGroupNCCL makes
        the collective's stream wait on the current stream at issue, and the compute stream waits on the collective
        before it reads the slot)."""
        i = self._stage_next.get(ring, 0)
        if self._stage_user.get((ring, i)) in self._pending:
            raise RuntimeError(f"FSDP staging ring {ring}: slot {i} still holds the pending gather of "
                               f"{self._stage_user[(ring, i)]}")
        if (ring, i) in self._rs_slot_work:
            raise RuntimeError(f"FSDP staging ring {ring}: slot {i} is still read by an unwaited reduce-scatter")
        self._stage_next[ring] = (i + 1) % self.STAGE_SLOTS
        return i, self._buf(ring, i, dtype, n)

    def _ring_free(self, ring) -> bool:
        """The next slot of ``ring`` holds no gathered unit still waiting for its unpack."""
        i = self._stage_next.get(ring, 0)
        return self._stage_user.get((ring, i)) not in self._pending

    def _issue_gather(self, unit, dtype):
        from . import _lib as K
        p = self.plan[unit]
        n = p.per * self.world
        if self.store is not None and unit in self.store.blocks:
            ring = "ag16" if dtype == torch.bfloat16 else "ag32"
            i, out = self._ring(ring, dtype, self._block_ag_len())
            out = out[:n]
            self._stage_user[(ring, i)] = unit
        else:
            out = self._buf("ag", unit, dtype, n)
        if dtype == torch.bfloat16:
            if not self._bf16_fresh:  # a step we did not run (torch optimizer, load): re-round every shard
                fp = self.flat_param.detach()
                for q in self.plans:
                    K.cast_f32_bf16(fp[q.soff:q.soff + q.per], self.bf16_chunk(q.name), q.per)
                self._bf16_fresh = True
            src = self.bf16_chunk(unit)  # resident mode: a view of out (in place)
        else:
            src = self.flat_param.detach()[p.soff:p.soff + p.per]
        if not self.coll:
            if src.data_ptr() != out[self.rank * p.per:].data_ptr():
                out[self.rank * p.per:(self.rank + 1) * p.per].copy_(src)
            work = None
        else:
            work = dist.all_gather_into_tensor(out, src, async_op=True)
        self._pending[unit] = (work, dtype, out)
        self._fenced.discard(unit)  # a new gather of the unit: not waited for yet

    def _block_ag_len(self) -> int:
        return max(self.plan[u].per for u in self.store.blocks) * self.world

    def _gather_for(self, unit, backward=False):
        """Make ``unit``'s parameters readable in the compute precision: wait for (or issue) its all-gather and unpack
        it, with the next units' gathers issued under this unit's compute (forward order, or backward order)."""
        from . import _lib as K
        eng = self.engine
        dtype = eng.compute_dtype() if not backward else self._compute_dtype
        self._compute_dtype = dtype
        self._check_version()
        if self._valid.get(unit) != dtype:
            if unit not in self._pending or self._pending[unit][1] != dtype:
                self._issue_gather(unit, dtype)
        if self.prefetch:  # the next units' all-gathers ride under this unit's compute
            self._prefetch_after(unit, dtype, backward)
        if self.coll:
            self._retire_completed()
        if self._valid.get(unit) == dtype:
            return
        work, _, out = self._pending.pop(unit)
        if work is not None and unit not in self._fenced:
            work.wait()
        self._fenced.discard(unit)
        p = self.plan[unit]
        if self.store is not None:
            f32, b16, b16_all, t16_all, base = self.store.unit_params(unit)
            K.fsdp_unpack(out, f32, b16 if dtype == torch.bfloat16 else None, p.n)
            if dtype == torch.bfloat16:
                names = [n for n, s in self.module.layout.slots.items() if p.lo <= s.offset < p.hi]
                eng.refresh_shadowT(names, shadow=b16_all, shadowT=t16_all, base=base)
        else:
            bf = eng.shadow[p.lo:p.hi] if dtype == torch.bfloat16 else None
            K.fsdp_unpack(out, self.module.arena[p.lo:p.hi], bf, p.n)
            if dtype == torch.bfloat16:
                names = [n for n, s in self.module.layout.slots.items() if p.lo <= s.offset < p.hi]
                eng.refresh_shadowT(names)
        self._valid[unit] = dtype

    def _evicted(self, unit):
        """reshard_after_forward: block ``unit`` lost its parameter slot (its next use gathers it again)."""
        self._valid[unit] = None

    def _bwd_unit(self, unit):
        """reshard_after_forward: before ``unit``'s backward: its parameters gathered again (the next unit in backward
        order prefetched), and gradient slots for it and for the block before it, whose fc2 bias gradient this unit's
        first LayerNorm backward forms (the head's: the last block's)."""
        st = self.store
        if unit != "embed":
            self._gather_for(unit, backward=True)
        i = self.order.index(unit)
        if unit in st.blocks:
            st.take_gslot(unit)
        if i > 0 and self.order[i - 1] in st.blocks:
            st.take_gslot(self.order[i - 1])

    def _gather_bytes(self, unit, dtype) -> int:
        p = self.plan[unit]
        return p.per * self.world * dtype.itemsize

    def _prefetch_after(self, unit, dtype, backward=False):
        """Issue the all-gathers of the units after ``unit`` (forward order; backward order for a backward re-gather)
        while the gathered bytes in flight stay within prefetch_bytes (and the units ahead within prefetch_depth); one
        unit ahead is always allowed. reshard_after_forward: at most STAGE_SLOTS - 1 block gathers wait for their
        unpack (the staging ring), and a unit is gathered ahead only if it will need it (not resident)."""
        seq = self.order if not backward else list(reversed(self.order))
        i = seq.index(unit)
        ahead = seq[i + 1:]
        if backward:
            ahead = [u for u in ahead if u != "embed"]  # the root stays gathered
        if self.prefetch_depth is not None:
            ahead = ahead[:self.prefetch_depth]
        if self.store is not None:
            ahead = ahead[:self.STAGE_SLOTS - 1]
        inflight = sum(self._gather_bytes(u, dt) for u, (_, dt, _) in self._pending.items() if u != unit)
        for k, nxt in enumerate(ahead):
            if self._valid.get(nxt) == dtype:
                continue
            if nxt in self._pending:
                continue
            nb = self._gather_bytes(nxt, dtype)
            if k > 0 and inflight + nb > self.prefetch_bytes:
                break
            if self.store is not None and nxt in self.store.blocks and \
                    not self._ring_free("ag16" if dtype == torch.bfloat16 else "ag32"):
                break
            self._issue_gather(nxt, dtype)
            inflight += nb

    def _retire_completed(self):
        """Stream-wait every pending all-gather whose work reads complete (costs nothing: it is done) so that it stops
        counting as in flight; the rest stay pending until they complete or their unit runs."""
        for u, (w, *_) in self._pending.items():
            if w is not None and u not in self._fenced and w.is_completed():
                w.wait()
                self._fenced.add(u)

    # ---- backward: per-unit reduce-scatter as ranges become final ----------------------------------------
    def _reduce_scatter(self, unit):
        from . import _lib as K
        p = self.plan[unit]
        eng = self.engine
        dtype = eng.bwd_act  # reduce_dtype = the compute precision (bf16 under autocast)
        n = p.per * self.world
        slot = None
        if self.store is not None and unit in self.store.blocks:
            # reshard_after_forward: the packed input goes to a staging ring (its slot's previous reduce-scatter waited
            # for first), the reduced shard to a shard-sized buffer of the unit; the gradient slot is free once packed
            ring = "rs16" if dtype == torch.bfloat16 else "rs32"
            prev = self._rs_slot_work.pop((ring, self._stage_next.get(ring, 0)), None)
            if prev is not None:  # the slot's previous reduce-scatter completes before the pack below refills it
                prev.wait()
            i, inp = self._ring(ring, dtype, self._block_ag_len())
            inp = inp[:n]
            slot = (ring, i)
            out = self._buf("rs_out", unit, dtype, p.per)
            K.fsdp_pack(self.store.unit_grad(unit), inp, p.n, n)
            self.store.release_gslot(unit)
        else:
            inp = self._buf("rs_in", unit, dtype, n)
            src = self.store.unit_grad(unit) if self.store is not None else eng.grad[p.lo:p.hi]
            K.fsdp_pack(src, inp, p.n, n)
            # in place: this rank's chunk of the packed input receives the reduced shard (RCCL copies nothing locally)
            out = inp[self.rank * p.per:(self.rank + 1) * p.per]
        if not self.coll:
            if out.data_ptr() != inp[self.rank * p.per:].data_ptr():
                out.copy_(inp[self.rank * p.per:(self.rank + 1) * p.per])
            work = None
        else:
            work = dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, async_op=True)
            if slot is not None:
                self._rs_slot_work[slot] = work
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
        if self.store is not None:
            # unsharded gradients would have to outlive their unit's backward (the reference loop accumulates without
            # no_sync, reduce-scattering every micro-step into the sharded gradient, which this mode does)
            raise NotImplementedError("no_sync() with reshard_after_forward=True: accumulate without no_sync")
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
        arena = torch.zeros(self.module.layout.total, dtype=torch.float32, device=self.flat_param.device)
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
        lay = m.layout
        arena = torch.zeros(lay.total, dtype=torch.float32, device=self.flat_param.device)
        for n in lay.slots:
            lay.view(arena, n).copy_(sd[n])
        if self.store is None:  # the module's own views (resident mode keeps them)
            m.arena.copy_(arena)
        for pl in self.plans:
            a, b = pl.lo + self.rank * pl.per, min(pl.hi, pl.lo + (self.rank + 1) * pl.per)
            chunk = self.flat_param.detach()[pl.soff:pl.soff + pl.per]
            chunk.zero_()
            if b > a:
                chunk[:b - a].copy_(arena[a:b])
        self.mark_params_updated(False)
        self._seen_version = None  # force a refresh at the next forward


ShardedDataParallel = FullyShardedDataParallel
