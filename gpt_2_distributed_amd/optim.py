"""Fused AdamW over a flat fp32 parameter range (one HIP kernel per step).

Semantics of the reference optimizer (train_gpt2_distributed.py:356-362): ``torch.optim.AdamW(
model.parameters(), lr, weight_decay=0.1, betas=(0.9, 0.95), fused=True)`` — one param group, eps
1e-8, decoupled weight decay on every parameter, bias-corrected moments, constant lr. The kernel
also (a) returns the total grad L2 norm that ``clip_grad_norm_(params, inf)`` reports (:419-421;
with max_norm=inf the clip coefficient is exactly 1.0 so no rescale pass is needed), (b) applies an
optional gradient pre-scale and (c) writes the bf16 copy of the updated weights (the GEMM shadow, or
under FSDP the bf16 shard the next forward all-gathers).

* ``FusedAdamW(model)``: the whole arena of a local / DDP model.
* ``ShardedAdamW(fsdp)``: this rank's FSDP shard (flat_param); the reported grad norm is the global
  one (the reference's FSDP run reports a per-shard norm averaged over ranks, SURVEY §5 quirk iv).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib as K


class _FlatAdamW(torch.optim.Optimizer):
    _gpt2mi_fused = True  # refreshes the engine's shadows itself (engine.watch_optimizer_steps skips it)

    def __init__(self, params, p_flat, lr, betas, eps, weight_decay):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        n = p_flat.numel()
        dev = p_flat.device
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.partials = torch.empty(K.norm_partials_size(), dtype=torch.float32, device=dev)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_count = 0
        self.grad_scale = 1.0

    def _run(self, p, g, pb, lo=0, hi=None, partials=None):
        """One fused AdamW launch over p[lo:hi] (step_count advanced by the caller). partials: the grad-norm partial
        sums go there and the norm is left to the caller (gpt2mi_norm_finalize); else self.grad_norm is written."""
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        hi = p.numel() if hi is None else hi
        K.adamw(p[lo:hi], g[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi], pb, hi - lo, float(grp["lr"]),
                float(grp["weight_decay"]), float(b1), float(b2), float(grp["eps"]), self.step_count,
                float(self.grad_scale), self.partials if partials is None else partials,
                self.grad_norm if partials is None else None)

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [dict(g, params=[]) for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            for k, v in s.items():
                if k != "params":
                    g[k] = v


class FusedAdamW(_FlatAdamW):
    def __init__(self, model, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1):
        super().__init__(list(model.parameters()), model.arena, lr, betas, eps, weight_decay)
        self.model = model
        self.engine = model.engine()
        self.tail_source = None

    def attach_tail(self, hooks):
        """DistributedDataParallel(overlap_optimizer=True): ``hooks.take_tail()`` hands over the backward's last bucket
        (work, lo, hi) still in flight; step() updates the arena outside [lo, hi) first, then waits for it."""
        self.tail_source = hooks
        self.partials = torch.empty(3 * K.norm_partials_size(), dtype=torch.float32, device=self.partials.device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        eng = self.engine
        if all(p.grad is None for p in eng.params_by_name.values()):
            if self.tail_source is not None:
                self.tail_source.wait_tail()
            return loss  # no gradients since zero_grad(set_to_none=True): torch's optimizers skip such params
        self.step_count += 1
        tail = self.tail_source.take_tail() if self.tail_source is not None else None
        arena, n = self.model.arena, self.model.arena.numel()
        if tail is not None and (tail[1] % 4 or tail[2] % 4):  # the kernel takes 4-element groups
            tail[0].wait()
            tail = None
        if tail is None:
            self._run(arena, eng.grad, eng.shadow)
        else:
            # the ranges outside the in-flight bucket run under its all-reduce; then the bucket's own range. The
            # grad-norm partial sums of the pieces go to one buffer, finalised once (the same per-element updates and
            # the same norm as one launch: tests/test_kernels_gpu.py::test_adamw_in_pieces_with_one_norm_finalisation)
            work, lo, hi = tail
            P, k = K.norm_partials_size(), 0
            for a, b in ((0, lo), (hi, n)):
                if b > a:
                    self._run(arena, eng.grad, eng.shadow[a:b], a, b, self.partials[k * P:(k + 1) * P])
                    k += 1
            work.wait()
            self._run(arena, eng.grad, eng.shadow[lo:hi], lo, hi, self.partials[k * P:(k + 1) * P])
            K.norm_finalize(self.partials, (k + 1) * P, self.grad_norm)
        eng.mark_shadow_fresh()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        # The grads are views of one arena. set_to_none (torch's default): unbind them; the next backward
        # rebinds, and a whole-model backward then zeroes only the accumulated slots (its weight-gradient
        # GEMMs write theirs). Otherwise zero the arena in one memset and keep the views bound.
        if self.tail_source is not None:
            self.tail_source.wait_tail()  # a deferred bucket still writes its range of the arena
        if set_to_none:
            for p in self.engine.params_by_name.values():
                p.grad = None
        else:
            self.engine.zero_grad()
            self.engine.bind_grads()


class ShardedAdamW(_FlatAdamW):
    """One launch per FSDP unit: each writes its unit's bf16 shard straight into that unit's all-gather buffer
    (FullyShardedDataParallel.bf16_chunk; only while the model computes in bf16), so the next forward gathers in place,
    and its grad-norm partial sums into its slice of one buffer, finalised once into the clip_grad_norm_ value."""

    def __init__(self, fsdp, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1):
        super().__init__([fsdp.flat_param], fsdp.flat_param, lr, betas, eps, weight_decay)
        self.fsdp = fsdp
        self.unit_partials = torch.empty(len(fsdp.plans) * K.norm_partials_size(), dtype=torch.float32,
                                         device=fsdp.flat_param.device)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        f = self.fsdp
        if f.flat_param.grad is None:
            f.wait_tail()
            return loss  # no backward since zero_grad(set_to_none=True): skipped, as torch's optimizers do
        self.step_count += 1
        p = f.flat_param.detach()
        P = K.norm_partials_size()
        # a unit whose reduce-scatter is still in flight (FullyShardedDataParallel(overlap_optimizer=True)) goes last,
        # after every other unit's update has been enqueued under it
        tail = f.tail_unit()
        order = [i for i, q in enumerate(f.plans) if q.name != tail] + \
            [i for i, q in enumerate(f.plans) if q.name == tail]
        for i in order:
            q = f.plans[i]
            if q.name == tail:
                f.wait_tail()
            pb = f.bf16_chunk(q.name) if f.wants_bf16() else None  # (fp32 FSDP gathers fp32: no bf16 shards)
            self._run(p, f.grad_shard, pb, q.soff, q.soff + q.per, self.unit_partials[i * P:(i + 1) * P])
        f.mark_params_updated(bf16_fresh=f.wants_bf16())
        # the clip_grad_norm_(inf) value of the full model: sum of squares over units (one finalisation) and shards
        K.norm_finalize(self.unit_partials, self.unit_partials.numel(), self.grad_norm)
        if f.coll:
            n2 = self.grad_norm.square()
            dist.all_reduce(n2)
            torch.sqrt(n2, out=self.grad_norm)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.fsdp.zero_grad(set_to_none=set_to_none)
