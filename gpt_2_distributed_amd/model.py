"""GPT-2 with the reference's module surface, running on hand-written MI355X kernels.

Drop-in for `/root/reference/model.py`: same ``GPT2Config`` (frozen dataclass, same fields and
defaults, model.py:26-57), same module tree and parameter names (``transformer.wte/wpe/h[i].{ln1,
attn.{qkv,proj},ln2,mlp.{fc1,fc2}}/ln_f``, tied ``lm_head``; 148 parameters, 149 state_dict keys),
the same seed-42 private-generator init (model.py:249-268), and
``GPT2.forward(idx, labels=None) -> (logits, loss)`` (model.py:335-361). nanoGPT-style aliases the
north star names are exported too: ``GPT = GPT2``, ``forward(idx, targets=...)`` and
``configure_optimizers``.

What differs underneath (MI355X-first):
* all parameters live in one flat fp32 arena (``arena.py``) so AdamW / grad-norm / collectives are
  single passes; ``wte`` is padded to a multiple of 256 rows for the lm_head tiling;
* ``GPT2.forward`` is ONE autograd node: forward and backward of the whole network are explicit
  sequences of HIP kernels (``engine.py``) with bf16 MFMA GEMMs, fused epilogues, flash attention;
  under ``torch.autocast("cuda", torch.bfloat16)`` (the reference trainer,
  train_gpt2_distributed.py:404) it computes with CUDA-autocast-bf16 numerics (bf16 MFMA operands,
  fp32 LayerNorm/softmax/loss/residual); without autocast it computes in fp32 like the plain
  reference module (fp32 MFMA GEMMs, fp32 attention). ``model.precision = "bf16" | "fp32"``
  overrides the autocast-following default ``"auto"``;
* no [T,T] ``mask`` buffer (model.py:105-108): causality comes from tile indices (the buffer was
  non-persistent, so state_dicts are unchanged);
* the sub-modules of a GPT2 are callable on their own (``GPT2Backbone.forward(idx)`` -> ln_f output,
  ``GPT2Block.forward(x)``, ``MLP.forward(x)``, ``CausalMultiHeadSelfAttention.forward(x)``) and
  differentiable, through the same kernels; they read the parameters from the owning GPT2's arena, so a
  block constructed outside a GPT2 has no MI355X path (it raises).
The GPU path has no CPU fallback: a CPU ``forward`` raises.
"""
from __future__ import annotations

import math
import weakref
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .arena import ArenaLayout, round_up


@dataclass(frozen=True)
class GPT2Config:
    """Configuration for the GPT-2 model (model.py:26-57)."""
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    resid_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02


# Model sizes of BASELINE.json configs (the reference hard-codes 124M).
MODEL_SIZES = {
    "124M": dict(n_layer=12, n_head=12, n_embd=768),
    "350M": dict(n_layer=24, n_head=16, n_embd=1024),
    "1.5B": dict(n_layer=48, n_head=25, n_embd=1600),
}


class NewGELU(nn.Module):
    """tanh GELU (model.py:63-77). In the training step it is fused into the fc1 GEMM epilogue."""

    def forward(self, input):
        return 0.5 * input * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (input + 0.044715 * torch.pow(input, 3.0))))


class _OwnedByGPT2:
    """Sub-modules of a GPT2 run through the owner's engine (parameters live in its flat arena)."""

    def _bind_owner(self, owner: "GPT2", layer: Optional[int]):
        self._owner_ref = weakref.ref(owner)
        self._layer = layer

    def _owner_engine(self):
        ref = getattr(self, "_owner_ref", None)
        owner = ref() if ref is not None else None
        if owner is None:
            raise RuntimeError(f"{type(self).__name__} runs on the MI355X engine only as a sub-module of a GPT2 "
                               "model (its parameters live in the GPT2's flat arena)")
        if not owner.arena.is_cuda:
            raise RuntimeError("gpt_2_distributed_amd runs only on the MI355X HIP path: move the model to a cuda "
                               "device (there is no CPU fallback)")
        return owner.engine()


class CausalMultiHeadSelfAttention(_OwnedByGPT2, nn.Module):
    """Causal multi-head self-attention (model.py:80-159): qkv, proj, attn/resid dropout. ``forward(x)``
    takes the ln1 output [B,T,C] and returns drop(proj(attention)) (bf16 under autocast)."""

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        assert cfg.n_embd % cfg.n_head == 0
        self.n_head = cfg.n_head
        self.head_dim = cfg.n_embd // cfg.n_head
        self.qkv = nn.Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.proj = nn.Linear(cfg.n_embd, cfg.n_embd)
        self.attn_drop = nn.Dropout(cfg.attn_pdrop)
        self.resid_drop = nn.Dropout(cfg.resid_pdrop)

    def forward(self, x):
        return self._owner_engine().sub_forward("attn", self._layer, x)


class MLP(_OwnedByGPT2, nn.Module):
    """MLP (model.py:162-192): fc1 -> NewGELU -> drop1 -> fc2 -> drop2. ``forward(x)`` takes the ln2
    output [B,T,C] (bf16 under autocast)."""

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        hidden = 4 * cfg.n_embd
        self.fc1 = nn.Linear(cfg.n_embd, hidden)
        self.fc2 = nn.Linear(hidden, cfg.n_embd)
        self.act = NewGELU()
        self.drop1 = nn.Dropout(cfg.resid_pdrop)
        self.drop2 = nn.Dropout(cfg.resid_pdrop)

    def forward(self, x):
        return self._owner_engine().sub_forward("mlp", self._layer, x)


class GPT2Block(_OwnedByGPT2, nn.Module):
    """One transformer block (model.py:195-219); the unit the FSDP mode shards by. ``forward(x)``:
    x + attn(ln1(x)), then x + mlp(ln2(x)) on the fp32 residual stream [B,T,C]."""

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln1 = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.attn = CausalMultiHeadSelfAttention(cfg)
        self.ln2 = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.mlp = MLP(cfg)

    def forward(self, x):
        return self._owner_engine().sub_forward("block", self._layer, x)


class GPT2Backbone(_OwnedByGPT2, nn.Module):
    """Embeddings + blocks + ln_f (model.py:225-313), same init (model.py:249-268)."""

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.drop = nn.Dropout(cfg.resid_pdrop)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = nn.LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.init_rng = torch.Generator()
        self.init_rng.manual_seed(42)
        self.apply(self._init_weights)

    def _init_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            nn.init.normal_(module.weight, mean=0.0, std=self.cfg.initializer_range, generator=self.init_rng)
        if isinstance(module, nn.Linear) and module.bias is not None:
            nn.init.zeros_(module.bias)

    @property
    def max_seq_len(self):
        return self.cfg.n_positions

    def forward(self, idx: torch.Tensor) -> torch.Tensor:
        """Embeddings -> blocks -> ln_f (model.py:275-313); returns the fp32 ln_f output [B,T,C]."""
        B, T = idx.size()
        if T > self.cfg.n_positions:
            raise ValueError(f"Sequence length {T} > model max {self.cfg.n_positions}")
        eng = self._owner_engine()
        if not idx.is_cuda:
            raise RuntimeError("gpt_2_distributed_amd runs only on the MI355X HIP path: move the inputs to a cuda "
                               "device (there is no CPU fallback)")
        return eng.backbone_forward(idx)


class GPT2(nn.Module):
    """GPT-2 backbone + tied language-model head (model.py:316-361)."""

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.transformer = GPT2Backbone(cfg)
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self.lm_head.weight = self.transformer.wte.weight
        self._pack_arena()
        self._engine = None
        self.precision = "auto"
        self._bind_submodules()

    def _bind_submodules(self):
        self.transformer._bind_owner(self, None)
        for i, blk in enumerate(self.transformer.h):
            blk._bind_owner(self, i)
            blk.attn._bind_owner(self, i)
            blk.mlp._bind_owner(self, i)

    # copies (copy.deepcopy / pickling) get their own engine and re-point their sub-modules at themselves
    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        return st

    def __setstate__(self, st):
        super().__setstate__(st)
        self._rebind(self._arena)  # a copied Parameter is a clone, no longer a view of the copied arena
        self._bind_submodules()  # "auto": follow torch.autocast("cuda"); or force "bf16" / "fp32"

    # ---- flat arena ------------------------------------------------------------------------------
    def _pack_arena(self):
        cfg = self.config
        self.vpad = round_up(cfg.vocab_size, 256)
        names = [n for n, _ in self.named_parameters()]
        shapes = {n: tuple(p.shape) for n, p in self.named_parameters()}
        from collections import OrderedDict
        self.layout = ArenaLayout(OrderedDict((n, shapes[n]) for n in names), self.vpad)
        arena = torch.zeros(self.layout.total, dtype=torch.float32)
        for n, p in self.named_parameters():
            self.layout.view(arena, n).copy_(p.detach())
        self._arena = arena
        self._rebind(arena)

    def _rebind(self, arena: torch.Tensor):
        self._arena = arena
        for name in self.layout.slots:
            mod_path, attr = name.rsplit(".", 1)
            mod = self.get_submodule(mod_path)
            old = getattr(mod, attr)
            newp = nn.Parameter(self.layout.view(arena, name), requires_grad=old.requires_grad)
            setattr(mod, attr, newp)
        self.lm_head.weight = self.transformer.wte.weight

    def _apply(self, fn, recurse=True):
        # Move the arena as a whole so parameters stay views of one buffer.
        new = fn(self._arena)
        if new.dtype != torch.float32:
            raise TypeError("GPT2 keeps fp32 master weights in one arena; only device moves are supported "
                            "(the bf16 compute copy is managed by the engine)")
        if new.data_ptr() != self._arena.data_ptr():
            self._rebind(new)
            self._engine = None
        for m in self.children():
            for sub in m.modules():
                for k, b in list(sub._buffers.items()):
                    if b is not None:
                        sub._buffers[k] = fn(b)
        return self

    @property
    def arena(self) -> torch.Tensor:
        return self._arena

    def engine(self):
        if self._engine is None:
            from .engine import Engine
            self._engine = Engine(self)
        return self._engine

    # ---- forward -----------------------------------------------------------------------------------
    def forward(self, idx: torch.Tensor, labels: Optional[torch.Tensor] = None,
                targets: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        if targets is not None:
            if labels is not None:
                raise ValueError("pass labels or targets, not both")
            labels = targets
        B, T = idx.size()
        if T > self.config.n_positions:
            raise ValueError(f"Sequence length {T} > model max {self.config.n_positions}")
        if not idx.is_cuda or not self._arena.is_cuda:
            raise RuntimeError("gpt_2_distributed_amd.GPT2 runs only on the MI355X HIP path: move the model and "
                               "inputs to a cuda device (there is no CPU fallback)")
        return self.engine().forward(idx, labels)

    # ---- optimizer (nanoGPT-style name the north star uses) -----------------------------------------
    def configure_optimizers(self, weight_decay: float = 0.1, learning_rate: float = 1e-4,
                             betas=(0.9, 0.95), device_type: Optional[str] = None, eps: float = 1e-8):
        """The reference builds ``torch.optim.AdamW(model.parameters(), lr, weight_decay=0.1,
        betas=(0.9, 0.95), fused=True)`` inline (train_gpt2_distributed.py:356-362): ONE param group,
        so decay also hits biases/LayerNorm/embeddings. This returns the same optimizer as one fused
        HIP kernel over the flat arena."""
        from .optim import FusedAdamW
        return FusedAdamW(self, lr=learning_rate, betas=betas, eps=eps, weight_decay=weight_decay)


GPT = GPT2  # nanoGPT alias used by the north star
