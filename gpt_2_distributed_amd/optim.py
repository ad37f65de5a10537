"""Fused AdamW over the flat parameter arena (one HIP kernel per step).

Semantics of the reference optimizer (train_gpt2_distributed.py:356-362): ``torch.optim.AdamW(
model.parameters(), lr, weight_decay=0.1, betas=(0.9, 0.95), fused=True)`` — one param group, eps
1e-8, decoupled weight decay on every parameter, bias-corrected moments, constant lr. The kernel
also (a) returns the total grad L2 norm that ``clip_grad_norm_(params, inf)`` reports (:419-421;
with max_norm=inf the clip coefficient is exactly 1.0 so no rescale pass is needed), (b) applies a
gradient pre-scale (1/world for SUM-reduced data-parallel grads) and (c) writes the bf16 weight
shadow the GEMMs read.
"""
from __future__ import annotations

import torch

from . import _lib as K


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, model, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, shard=None):
        super().__init__(list(model.parameters()), dict(lr=lr, betas=tuple(betas), eps=eps,
                                                         weight_decay=weight_decay))
        self.model = model
        self.engine = model.engine()
        self.shard = shard  # (lo, hi) element range owned by this rank (ZeRO/FSDP mode), else whole arena
        arena = model.arena
        lo, hi = shard if shard is not None else (0, arena.numel())
        self._lo, self._hi = lo, hi
        self.exp_avg = torch.zeros(hi - lo, dtype=torch.float32, device=arena.device)
        self.exp_avg_sq = torch.zeros(hi - lo, dtype=torch.float32, device=arena.device)
        self.partials = torch.empty(K.norm_partials_size(), dtype=torch.float32, device=arena.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=arena.device)
        self.step_count = 0
        self.grad_scale = 1.0

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        self.step_count += 1
        eng = self.engine
        lo, hi = self._lo, self._hi
        arena = self.model.arena
        K.adamw(arena[lo:hi], eng.grad[lo:hi], self.exp_avg, self.exp_avg_sq, eng.shadow[lo:hi], hi - lo,
                float(g["lr"]), float(g["weight_decay"]), float(b1), float(b2), float(g["eps"]), self.step_count,
                float(self.grad_scale), self.partials, self.grad_norm)
        eng.mark_shadow_fresh()
        return loss

    def zero_grad(self, set_to_none: bool = True):
        # The grads are views of one arena: zero it in one memset and keep the views bound.
        self.engine.zero_grad()
        self.engine.bind_grads()

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "shard": (self._lo, self._hi), "param_groups": [dict(g, params=[]) for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            for k, v in s.items():
                if k != "params":
                    g[k] = v
