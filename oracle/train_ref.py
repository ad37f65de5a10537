"""Restatement of the reference training step loop — TEST ORACLE.

Test infrastructure only. Follows ``train_gpt2_distributed.py:374-425``:
loss/grad_accum (``:409``) -> backward (``:412``) -> every grad_accum micro-steps
``clip_grad_norm_(params, inf)`` (``:419-421``: reports the total L2 norm, the clip coefficient is
clamp(inf/(n+1e-6), max=1) = 1.0 so grads are unchanged) -> AdamW step (``:356-362,424``:
lr, wd=0.1, betas=(0.9,0.95), eps=1e-8, decoupled decay, one param group) -> zero_grad.

The AdamW update restates ``torch/optim/adam.py`` ``_single_tensor_adam`` (decoupled weight decay):
  p <- p * (1 - lr*wd); m <- lerp(m, g, 1-b1); v <- v*b2 + (1-b2) g^2;
  p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Tuple

import torch

from . import model_ref


def adamw_step(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor], state: dict, step: int,
               lr=1e-4, wd=0.1, b1=0.9, b2=0.95, eps=1e-8):
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    for n, p in params.items():
        g = grads[n]
        if n not in state:
            state[n] = (torch.zeros_like(p), torch.zeros_like(p))
        m, v = state[n]
        p.mul_(1 - lr * wd)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


def total_grad_norm(grads: Iterable[torch.Tensor]) -> float:
    """clip_grad_norm_(..., inf) return value: 2-norm of the per-tensor 2-norms (torch/nn/utils/clip_grad.py)."""
    norms = torch.stack([g.detach().float().norm(2) for g in grads])
    return float(norms.norm(2))


def run(cfg, batches: Iterable[Tuple[torch.Tensor, torch.Tensor]], steps: int, grad_accum: int = 1,
        lr=1e-4, mode="fp32", params=None) -> Tuple[List[float], List[float]]:
    """Run ``steps`` optimizer steps; returns (last-micro-batch loss per step, grad norm per step),
    the two values the reference logs (train_gpt2_distributed.py:432-440)."""
    params = model_ref.init_params(cfg) if params is None else params
    for p in params.values():
        p.requires_grad_(True)
    state: dict = {}
    losses, norms = [], []
    it = iter(batches)
    for step in range(1, steps + 1):
        grads = {n: torch.zeros_like(p) for n, p in params.items()}
        for _ in range(grad_accum):
            x, y = next(it)
            _, loss = model_ref.forward(params, cfg, x, y, mode)
            gl = torch.autograd.grad(loss / grad_accum, list(params.values()))
            for (n, _), g in zip(params.items(), gl):
                grads[n] += g
        norms.append(total_grad_norm(grads.values()))
        losses.append(float(loss.detach()))
        with torch.no_grad():
            adamw_step(params, grads, state, step, lr=lr)
    return losses, norms
