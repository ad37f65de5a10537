"""The GPT-2 training-step engine: forward -> loss -> backward as explicit HIP kernel sequences.

One ``torch.autograd.Function`` wraps the whole network, so ``loss.backward()`` (the reference's
``train_gpt2_distributed.py:412``) runs ``Engine._backward``: every gradient is produced by the
kernels of libgpt2mi straight into the flat fp32 grad arena (``p.grad`` are views of it). The returned
logits are differentiable too (``model.py:351`` hands them to the caller): a gradient that reaches
them is added to the lm_head's dlogits before the lm_head backward.

The sub-modules are callable on their own with the same kernels (``model.py:110-159,186-192,213-219,
275-313``): ``GPT2Backbone.forward(idx)`` (embedding -> blocks -> ln_f), ``GPT2Block.forward(x)``,
``MLP.forward(x)`` and ``CausalMultiHeadSelfAttention.forward(x)``, each its own autograd node whose
backward accumulates into the same grad arena.

Numerics = the reference under ``torch.autocast("cuda", bfloat16)`` (train_gpt2_distributed.py:404):
bf16 GEMM operands with fp32 accumulation, fp32 residual stream / LayerNorm / softmax / loss,
fp32 master weights and grads. Without autocast everything runs in fp32 (the plain model.py module).
Dropout uses the config's p (model.py:47-51) in train mode with a counter-based mask that backward
regenerates; eval mode / p = 0 disables it.

Sequence lengths that are not a multiple of the 64-token attention tile are padded inside the engine
(tokens 0, labels ignore_index, zero embedding rows): causality keeps the padding invisible to every
real position, the loss counts real labels only, and padded rows carry exactly zero gradient.

HBM layout per (B, T) workspace (M = B*T tokens, C = n_embd, Vp = vocab padded to 256):
  residual stream x[l]          fp32 [L+1][M, C]
  per block: ln1, ln2 bf16 [M,C]; mean/rstd fp32 [M]; qkv bf16 [M,3C]; attn out bf16 [M,C];
             lse fp32 [B*H,T]; x_mid fp32 [M,C]; gelu output h and dgelu = keep/(1-p)*gelu'(u) bf16 [M,4C]
  head:      ln_f bf16 [M,C]; dlogits bf16 [M,Vp]; logits bf16 [M,Vp] are a FRESH tensor per forward
             (returned as a [B,T,V] view that stays valid as long as the caller holds it)
  backward scratch: dres fp32 [M,C], dres_bf bf16 [M,C], dln bf16 [M,C], dU bf16 [M,4C],
             dqkv bf16 [M,3C], delta fp32 [B*H,T], dqkv_cs fp32 [M/32,3C]
"""
from __future__ import annotations

import os
import weakref
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from . import _lib as K
from ._lib import wgrad_group_splits as K_wgrad_group_splits
from ._lib import wgrad_splits as K_wgrad_splits
from .dropout_keys import MULTIPLIERS

BF16 = torch.bfloat16
F32 = torch.float32
ATTN_TILE = 64  # the attention kernels tile T by 64 queries / keys


def _mix(*xs: int) -> int:
    """64-bit seed mixing for per-site dropout streams."""
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h ^= (x + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2)) & 0xFFFFFFFFFFFFFFFF
        h = (h * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    return h


def site_seeds(base_seed: int, step_seed: int, n_layer: int) -> dict:
    """The 64-bit dropout seed of every site of one step ("embd", ("attn"|"proj"|"fc1"|"fc2", l)): the low word a
    mixed counter offset, the high word the site's vetted second-round multiplier (dropout_keys.py; site i takes
    entry i, so no two sites of a step share one: their masks are distinct functions, csrc/common.h)."""
    def seed(i, *key):
        return (MULTIPLIERS[i % len(MULTIPLIERS)] << 32) | (_mix(base_seed, step_seed, *key) & 0xFFFFFFFF)
    s = {"embd": seed(0, 0xE)}
    for l in range(n_layer):
        for k, site in enumerate(("attn", "proj", "fc1", "fc2")):
            s[(site, l)] = seed(1 + 4 * l + k, l, k + 1)
    return s


# Slack elements past the end of every activation buffer. None is needed since ABI v11: the weight-gradient GEMM of a
# width that is not a multiple of 256 (GPT-2 1.5B: 1600, 4800) bounds its partial last tile's reads at the operand's
# last element (gpt2mi.h gpt2mi_gemm_wgrad; v10 read up to 192 elements past it).
ACT_TAIL = 0


def act_empty(*shape, dtype, device):
    n = 1
    for d in shape:
        n *= d
    return torch.empty(n + ACT_TAIL, dtype=dtype, device=device)[:n].view(*shape)


def watch_optimizer_steps(owner, params, on_step) -> None:
    """Call on_step(owner) after any torch optimizer step that updates one of `params` (a global post-step hook).
    In-place updates normally bump a tensor's version counter, which is how the engine notices that its bf16
    shadow (or an FSDP wrapper that its gathered units) went stale, but torch's fused AdamW kernel
    (torch.optim.AdamW(fused=True), the reference trainer's optimizer, train_gpt2_distributed.py:356-362) does not
    bump it. The repo's own optimizers (``_gpt2mi_fused``) refresh the copies themselves and are skipped."""
    ids = {id(p) for p in params}
    ref = weakref.ref(owner)

    def hook(opt, args, kwargs):
        o = ref()
        if o is None or getattr(opt, "_gpt2mi_fused", False):
            return
        if any(id(p) in ids for g in opt.param_groups for p in g["params"]):
            on_step(o)

    from torch.optim.optimizer import register_optimizer_step_post_hook
    handle = register_optimizer_step_post_hook(hook)
    weakref.finalize(owner, handle.remove)


def padded_len(T: int) -> int:
    return (T + ATTN_TILE - 1) // ATTN_TILE * ATTN_TILE


@dataclass
class BlockActs:
    ln1: torch.Tensor
    m1: torch.Tensor
    r1: torch.Tensor
    qkv: torch.Tensor
    ao: torch.Tensor
    lse: torch.Tensor
    xmid: torch.Tensor
    ln2: torch.Tensor
    m2: torch.Tensor
    r2: torch.Tensor
    dgelu: torch.Tensor  # keep/(1-p) * gelu'(u) of the fc1 pre-activation u (from the fc1 epilogue)
    h: torch.Tensor

    @staticmethod
    def alloc(cfg, B, T, device, act, xmid=True):
        M, C, H = B * T, cfg.n_embd, cfg.n_head
        e = lambda *s, dt=act: act_empty(*s, dtype=dt, device=device)  # noqa: E731
        return BlockActs(ln1=e(M, C), m1=e(M, dt=F32), r1=e(M, dt=F32), qkv=e(M, 3 * C), ao=e(M, C),
                         lse=e(B * H, T, dt=F32), xmid=e(M, C, dt=F32) if xmid else None, ln2=e(M, C),
                         m2=e(M, dt=F32), r2=e(M, dt=F32), dgelu=e(M, 4 * C), h=e(M, 4 * C))


class Scratch:
    """Backward scratch of one (B, T) shape (also used by the stand-alone sub-module backwards)."""

    def __init__(self, cfg, B, T, vpad, device, act, head=True):
        C, H = cfg.n_embd, cfg.n_head
        M = B * T
        e = lambda *s, dt=act: act_empty(*s, dtype=dt, device=device)  # noqa: E731
        self.dres = e(M, C, dt=F32)
        self.dres_bf = e(M, C)
        self.dln = e(M, C)
        self.dU = e(M, 4 * C)
        self.dqkv = e(M, 3 * C)
        self.delta = e(B * H, T, dt=F32)
        # bf16 path: the attention backward writes 32-token partial column sums of dqkv (qkv bias grad)
        self.dqkv_cs = e(M // 32, 3 * C, dt=F32) if act == BF16 else None
        # split-K slabs of the 256x256 wgrad GEMMs
        wshapes = [(3 * C, C), (C, C), (4 * C, C), (C, 4 * C)] + ([(vpad, C)] if head else [])
        need = max((K_wgrad_splits(m, n, M) * m * n if K_wgrad_splits(m, n, M) > 1 else 0)
                   for m, n in wshapes) if C % 64 == 0 and act == BF16 else 0
        if C % 256 == 0 and act == BF16 and M % 128 == 0:  # a block's grouped weight gradients (Engine._wgrad_group)
            for gsh in (wshapes[2:4], wshapes[:2]):  # fc1 + fc2, qkv + proj
                need = max(need, K_wgrad_group_splits(gsh, M) * sum(m * n for m, n in gsh))
        if head and C % 64 == 0 and act == BF16 and M % 128 == 0 and vpad % 256 == 0:
            # the lm_head's transposed-X wgrad (taken under exactly these conditions, Engine._backward) always goes
            # through its slabs
            need = max(need, K_wgrad_splits(vpad, C, M) * vpad * C)
        self.wgrad_ws = e(max(need, 4), dt=F32)


class Workspace(Scratch):
    def __init__(self, cfg, B: int, T: int, vpad: int, device, act=BF16):
        super().__init__(cfg, B, T, vpad, device, act, head=True)
        L, C = cfg.n_layer, cfg.n_embd
        M = B * T
        e = lambda *s, dt=act: act_empty(*s, dtype=dt, device=device)  # noqa: E731
        self.act = act
        self.B, self.T, self.M = B, T, M
        self.x = e(L + 1, M, C, dt=F32)
        self.blocks: List[BlockActs] = [BlockActs.alloc(cfg, B, T, device, act) for _ in range(L)]
        self.lnf = e(M, C)
        self.lnf_t = None  # lnf transposed [C][M], formed by the backward for the lm_head wgrad (bf16 only)
        self.mf = e(M, dt=F32)
        self.rf = e(M, dt=F32)
        self.dlogits = e(M, vpad)
        self.loss_rows = e(M, dt=F32)
        self.lse_ce = e(M, dt=F32)
        self.inv_count = e(1, dt=F32)
        self.dscale = e(1, dt=F32)


class _NullCtxT:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NullCtx = _NullCtxT()


class _EventCtx:
    def __init__(self, lst):
        self.lst = lst

    def __enter__(self):
        self.s = torch.cuda.Event(enable_timing=True)
        self.e = torch.cuda.Event(enable_timing=True)
        self.s.record(torch.cuda.current_stream())
        return self

    def __exit__(self, *a):
        self.e.record(torch.cuda.current_stream())
        self.lst.append((self.s, self.e))
        return False


@dataclass
class _Saved:
    idx: torch.Tensor          # [B, Tp] (padded)
    labels: Optional[torch.Tensor]
    T: int                     # caller's sequence length (<= Tp)
    pr: float
    pa: float
    seeds: dict
    act: torch.dtype


class _GPT2Step(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, idx, labels, *params):
        ctx.set_materialize_grads(False)
        logits, loss = engine._forward(idx, labels, True)
        ctx.engine = engine
        ctx.token = engine._fwd_token
        ctx.n_params = len(params)
        return logits, loss

    @staticmethod
    def backward(ctx, grad_logits, grad_loss):
        eng = ctx.engine
        if ctx.token != eng._fwd_token:
            raise RuntimeError("GPT2 activations were overwritten by a later forward before this backward "
                               "(one forward/backward in flight per model)")
        eng._backward(grad_logits, grad_loss)
        return (None, None, None) + (None,) * ctx.n_params


class _TrunkFn(torch.autograd.Function):
    """GPT2Backbone.forward(idx) (model.py:275-313): embedding -> blocks -> ln_f, fp32 output."""

    @staticmethod
    def forward(ctx, engine, idx, *params):
        ctx.set_materialize_grads(False)
        out = engine._trunk_forward_module(idx, True)
        ctx.engine = engine
        ctx.token = engine._fwd_token
        ctx.n_params = len(params)
        return out

    @staticmethod
    def backward(ctx, dy):
        eng = ctx.engine
        if ctx.token != eng._fwd_token:
            raise RuntimeError("GPT2 activations were overwritten by a later forward before this backward")
        eng._trunk_backward_module(dy)
        return (None, None) + (None,) * ctx.n_params


class _SubFn(torch.autograd.Function):
    """A stand-alone block / MLP / attention call (its own activations; grads into the arena)."""

    @staticmethod
    def forward(ctx, engine, kind, layer, x, *params):
        ctx.set_materialize_grads(False)
        y, state = engine._sub_forward(kind, layer, x, True)
        ctx.engine, ctx.kind, ctx.layer, ctx.state, ctx.n_params = engine, kind, layer, state, len(params)
        ctx.x_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = None
        if dy is not None:
            dx = ctx.engine._sub_backward(ctx.kind, ctx.layer, ctx.state, dy).to(ctx.x_dtype)
        ctx.state = None
        return (None, None, None, dx) + (None,) * ctx.n_params


class GradHooks:
    """What a data-parallel wrapper plugs into the engine (parallel.py). All no-ops here."""

    def begin_backward(self) -> float:
        """Called before any gradient is written; returns the factor every gradient of this backward is
        scaled by (1/world for a SUM-reduced data-parallel backward)."""
        return 1.0

    def ready(self, name: str) -> None:
        """Arena range ``name`` (parallel.ready_ranges) holds its final gradient of this backward."""

    def end_backward(self) -> None:
        """The backward's last kernel is enqueued: finish the collective before backward returns."""

    def inflight(self) -> bool:
        """A collective of this wrapper may be running on its own stream concurrently with the kernels enqueued now.
        The engine then launches its GEMMs with GPT2MI_SCHED_SHARED_CUS: the persistent (one block per CU) schedule
        takes its tiles from per-XCD work queues, so a block that lands on a CU held by an RCCL kernel takes fewer
        tiles instead of the whole grid ending on its latest block. Every other launch keeps the static walk."""
        return False

    def fwd_unit(self, unit: str) -> None:
        """FSDP: the parameters of ``unit`` ("embed", "h.<l>", "head") are about to be read."""

    def bwd_unit(self, unit: str) -> None:
        """FSDP (reshard_after_forward): the backward of ``unit`` is about to run: its parameters are read again and its
        gradients (and the fc2 bias gradient of the unit before it, which this unit's LayerNorm backward forms) written."""


class Engine:
    """Owns the workspaces, the bf16 weight shadow and the grad arena of one GPT2 model."""

    WGRAD_SPLITS = 4
    # Weight-gradient split-K partial sums in bf16 slabs (gpt2mi.h GPT2MI_SCHED_BF16_SLABS: half the slab traffic,
    # ~0.5 ms per cfg-2 step) or fp32 slabs (fp32-exact sums of the bf16 products). Off by default since round 4: the
    # reference's autocast wgrad rounds its whole sum once to bf16 (at most 2^-8 relative on every element), while one
    # bf16 rounding per split leaves elements whose partial sums cancel with far larger relative errors
    # (tests/test_kernels_gpu.py::test_wgrad_slab_precision_per_element_at_the_proj_shape, 28 splits).
    WGRAD_BF16_SLABS = False
    # Schedule flag added while a data-parallel wrapper's collective may run (GradHooks.inflight): since ABI v11
    # GPT2MI_SCHED_SHARED_CUS (the persistent GEMM takes its tiles from per-XCD work queues, gemm_pp.hip g_pp_queue);
    # v8-v10 passed GPT2MI_SCHED_NO_PERSISTENT (one tile per block) instead.
    SCHED_UNDER_COLLECTIVES = K.SCHED_SHARED_CUS

    def __init__(self, model):
        self.model = model
        self.cfg = model.config
        self.layout = model.layout
        self.vpad = model.vpad
        self.device = model.arena.device
        arena = model.arena
        self.grad = torch.zeros_like(arena)
        self.shadow = torch.empty(arena.numel(), dtype=BF16, device=self.device)
        # W^T of every 2-D weight (same slot offsets, [in][out] row-major): the backward dgrad
        # dX = dY.W then runs as the forward-layout GEMM with both operands k-contiguous
        self.shadowT = torch.empty(arena.numel(), dtype=BF16, device=self.device)
        self._t_weights = [n for n, sl in self.layout.slots.items()
                           if len(sl.shape) == 2 and n != "lm_head.weight" and "wpe" not in n]
        self._shadowT_stale = True
        self._shadow_versions = None
        self._tdesc_cache: Dict[tuple, tuple] = {}
        self._ws: Dict[tuple, Workspace] = {}
        self._fwd_token = 0
        self._step_seed = 0
        self.base_seed = 1234
        self.grad_sync: Optional[GradHooks] = None  # set by data-parallel wrappers (parallel.py)
        self.param_provider = None  # FSDP: owns the full parameter views (gathers them per unit)
        # FullyShardedDataParallel(reshard_after_forward=True): the storage of every parameter / shadow / gradient view
        # (the resident units' slots instead of the full arenas, which are then freed); None: the full arenas
        self.store = None
        self.grad_dirty = False     # the grad arena holds gradients of an earlier backward (accumulation)
        # the weight-gradient GEMMs of the running backward write their slots outright: set by a full backward
        # that starts from zero_grad(set_to_none=True), which then zeroes only the accumulated slots
        self._grad_fresh = False
        self._acc_ranges = None     # cuda int64 [n, 2]: the arena ranges outside the GEMM-written weight slots
        self._grad_dead = False     # discard_grads(): the arena restarts from zero at the next backward
        self.bwd_act = F32
        self._params = list(model.parameters())
        self.params_by_name = dict(model.named_parameters())
        self.probes: Dict[str, list] = {}  # name -> [(start_event, end_event)] recorded when armed
        # GEMM schedule flags passed with every launch (gpt2mi.h GPT2MI_SCHED_*): base_sched for this engine, gemm_sched
        # for the running pass; a data-parallel wrapper adds SHARED_CUS while its collectives are in flight (_sched)
        self.base_sched = K.SCHED_AUTO
        self.gemm_sched = K.SCHED_AUTO
        # bf16 weight gradients (autocast): split-K partial sums in bf16 (True) or fp32 (False) slabs, see
        # WGRAD_BF16_SLABS
        self.wgrad_bf16_slabs = self.WGRAD_BF16_SLABS
        if not hasattr(K, "load") or self.device.type != "cuda":
            raise RuntimeError("the engine needs the model on a cuda (MI355X) device")
        K.load()
        self.refresh_shadow()
        watch_optimizer_steps(self, self._params, Engine.mark_shadow_stale)

    # ---- live per-kernel timing (bench.py): HIP events on the launch stream around named launches ----
    def _probe(self, name):
        lst = self.probes.get(name)
        if lst is None:
            return _NullCtx
        return _EventCtx(lst)

    def _sched(self):
        """The GEMM schedule flags of a launch enqueued now: the engine's own, plus SCHED_UNDER_COLLECTIVES while a
        data-parallel wrapper's collective may run concurrently (GradHooks.inflight)."""
        s = self.gemm_sched
        if self.grad_sync is not None and self.grad_sync.inflight():
            s |= self.SCHED_UNDER_COLLECTIVES
        return s

    def _gemm(self, *a, **kw):
        K.gemm(*a, sched=self._sched(), **kw)

    def _wgrad_sched(self):
        return self._sched() | (K.SCHED_BF16_SLABS if self.wgrad_bf16_slabs else 0)

    def _gemm_wgrad(self, *a, **kw):  # (bf16 operands only: the fp32 mode's wgrads run gemm layout 2)
        K.gemm_wgrad(*a, sched=self._wgrad_sched(), **kw)

    def _gemm_wgrad_kt(self, *a, **kw):
        K.gemm_wgrad_kt(*a, sched=self._wgrad_sched(), **kw)

    # ---- parameter views ------------------------------------------------------------------------------
    def _loc(self, kind, name):
        """(storage, element offset) of ``name``'s slot in the fp32 parameters ("p"), the bf16 shadow ("w16"), the W^T
        shadow ("wT") or the fp32 gradients ("g"): the full arenas, or the storage of the unit that holds it now
        (FullyShardedDataParallel(reshard_after_forward=True), engine.store)."""
        off = self.layout.slots[name].offset
        if self.store is not None:
            buf, base = self.store.loc(kind, name)
            return buf, off - base
        return {"p": self.model.arena, "g": self.grad, "w16": self.shadow, "wT": self.shadowT}[kind], off

    def _flat(self, kind, name):
        buf, o = self._loc(kind, name)
        return buf[o:o + self.layout.slots[name].reserved]

    def p(self, name):  # fp32 master view
        buf, o = self._loc("p", name)
        s = self.layout.slots[name]
        return buf[o:o + s.numel].view(s.shape)

    def g(self, name):  # fp32 grad view
        buf, o = self._loc("g", name)
        s = self.layout.slots[name]
        return buf[o:o + s.numel].view(s.shape)

    def gpad(self, name, rows):  # fp32 grad view of the whole (padded) slot, [rows, cols]
        return self._flat("g", name).view(rows, -1)

    def w16(self, name):  # bf16 shadow view (flat)
        return self._flat("w16", name)

    def refresh_shadow(self):
        """bf16 copy of the fp32 master weights the GEMMs read. The fused optimizer rewrites it in its
        own pass; after any other in-place update (torch optimizers, load_state_dict) it is re-cast."""
        K.cast_f32_bf16(self.model.arena, self.shadow, self.model.arena.numel())
        self._shadow_versions = self._versions()
        self._shadowT_stale = True

    def _versions(self):
        return tuple(p._version for p in self._params)

    def mark_shadow_stale(self):
        """A foreign in-place update of the master weights: re-cast the shadows before the next forward."""
        self._shadow_versions = None
        self._shadowT_stale = True

    def mark_shadow_fresh(self):
        self._shadow_versions = self._versions()
        self._shadowT_stale = True

    def _rows(self, name):
        sl = self.layout.slots[name]
        return sl.reserved // sl.shape[1]  # wte: the vocab-padded row count

    def wT_ok(self, name) -> bool:
        sl = self.layout.slots[name]
        return self._rows(name) % 64 == 0 and sl.shape[1] % 64 == 0

    def refresh_shadowT(self, names=None, shadow=None, shadowT=None, base=0):
        """Transpose every (or the listed) 2-D weight of the bf16 shadow into shadowT in one launch
        (49 separate 64x64-tile launches cost 0.28 ms per step). shadow / shadowT / base: the bf16 storage of one
        unit whose first element is arena element ``base`` (FSDP's reshard slots) instead of the full shadows."""
        key = (tuple(names) if names is not None else None, base)
        if key not in self._tdesc_cache:
            rows, tiles = [], 0
            for n in (self._t_weights if names is None else [m for m in names if m in self._t_weights]):
                if self.wT_ok(n):
                    sl = self.layout.slots[n]
                    R, Cc = self._rows(n), sl.shape[1]
                    rows.append((sl.offset - base, R, Cc, tiles))
                    tiles += (R // 64) * (Cc // 64)
            self._tdesc_cache[key] = (torch.tensor(rows, dtype=torch.int64, device=self.device) if rows else None,
                                      len(rows), tiles)
        desc, n, tiles = self._tdesc_cache[key]
        if n:
            K.transpose_bf16_batched(self.shadow if shadow is None else shadow,
                                     self.shadowT if shadowT is None else shadowT, desc, n, tiles)
        if names is None:
            self._shadowT_stale = False

    def wT16(self, name):  # bf16 W^T view (flat, [in][out_padded])
        return self._flat("wT", name)

    def _sync_shadows(self, act, need_grad):
        if self.param_provider is not None:
            return  # FSDP: the provider unpacks each gathered unit into the arena / shadow / shadowT
        if act == BF16:
            if self._versions() != self._shadow_versions:
                self.refresh_shadow()
            if self._shadowT_stale and need_grad:
                self.refresh_shadowT()

    def _unit(self, unit):
        if self.param_provider is not None:
            self.param_provider.fwd_unit(unit)

    def _unit_bwd(self, unit):
        if self.param_provider is not None:
            self.param_provider.bwd_unit(unit)

    # ---- grads ---------------------------------------------------------------------------------------
    def bind_grads(self):
        if self.store is not None:
            return  # reshard_after_forward: the module's parameters have no storage; gradients live in the store
        for name, p in self.params_by_name.items():
            if name == "lm_head.weight":
                continue
            p.grad = self.layout.view(self.grad, name)

    def zero_grad(self):
        if self.store is not None:  # reshard_after_forward: the next backward starts from zero (Engine._prepare_grads)
            self._grad_dead = True
            self.grad_dirty = False
            return
        K.zero_(self.grad)
        self.grad_dirty = False
        self._grad_dead = False

    def discard_grads(self):
        """The arena's gradients are consumed (FSDP reduced them into its shard): the next backward starts from zero,
        zeroed lazily as after zero_grad(set_to_none=True) (a whole-model backward's weight-gradient GEMMs write their
        slots and only the rest is zeroed)."""
        self._grad_dead = True
        self.grad_dirty = False

    def _lazy_zero_ok(self, act):
        # every weight-gradient GEMM of the full backward takes a path with a write-or-accumulate choice
        # (gemm_wgrad / EPI_F32; not the EPI_ATOMIC fallback of widths that are not multiples of 64)
        return act == BF16 and self.cfg.n_embd % 64 == 0

    def acc_ranges(self, lo, hi, shift=0):
        """(offset - lo + shift, count) of the arena ranges in [lo, hi) outside the GEMM-written weight slots (wte with
        its pad rows, the four matrices of every block): the LayerNorm params, biases, wpe, ln_f and the alignment gaps,
        which the backward accumulates into and so starts from zero."""
        gemm = sorted((max(sl.offset, lo), min(sl.offset + sl.reserved, hi)) for n, sl in self.layout.slots.items()
                      if n in self._t_weights and sl.offset < hi and sl.offset + sl.reserved > lo)
        rng, pos = [], lo
        for a, b in gemm:
            if a > pos:
                rng.append((pos - lo + shift, a - pos))
            pos = max(pos, b)
        if pos < hi:
            rng.append((pos - lo + shift, hi - pos))
        return rng

    def _zero_accumulated(self):
        """Zero the arena outside the GEMM-written weight slots in one launch."""
        if self._acc_ranges is None:
            self._acc_ranges = torch.tensor(self.acc_ranges(0, self.grad.numel()), dtype=torch.int64).to(self.device)
        K.zero_ranges(self.grad, self._acc_ranges)

    def _prepare_grads(self, full_backward_act=None):
        """Accumulate into the arena when p.grad are its views; start from zero after a
        zero_grad(set_to_none=True) (every p.grad None). full_backward_act: the precision of a backward that
        forms EVERY weight gradient (the whole-model loss backward): its GEMMs then write the weight slots
        and only the rest of the arena is zeroed."""
        self._grad_fresh = False
        if self.store is not None:
            # reshard_after_forward: every backward starts from zero (the previous one's gradients were reduce-scattered
            # into the shard); the store zeroes the root unit's gradients now and each block's as its slot is assigned
            self._grad_fresh = full_backward_act is not None and self._lazy_zero_ok(full_backward_act)
            self.store.begin_grads(self._grad_fresh)
            self._grad_dead = False
            self.grad_dirty = False
            return
        if self._grad_dead or all(p.grad is None for p in self.params_by_name.values()):
            self._grad_dead = False
            if full_backward_act is not None and self._lazy_zero_ok(full_backward_act):
                self._zero_accumulated()
                self._grad_fresh = True
                self.grad_dirty = False
            else:
                self.zero_grad()
            self.bind_grads()
            return
        for n, p in self.params_by_name.items():
            if p.grad is None or p.grad.data_ptr() != self.layout.view(self.grad, n).data_ptr():
                raise RuntimeError(f"{n}.grad is not a view of the engine's grad arena; zero grads with "
                                   "set_to_none=True or the model's optimizer before backward")

    def _begin_grads(self, act, full=False) -> float:
        if act == BF16 and self.param_provider is None and self._shadowT_stale:
            self.refresh_shadowT()  # the dgrads read W^T (a forward run without grad did not build it)
        self._prepare_grads(act if full else None)
        self.bwd_act = act  # the precision of this backward's gradients (FSDP reduces in it)
        scale = self.grad_sync.begin_backward() if self.grad_sync is not None else 1.0
        self.gemm_sched = self.base_sched
        self.grad_dirty = True
        return scale

    def _ready(self, name):
        if self.grad_sync is not None:
            self.grad_sync.ready(name)

    def _end_grads(self):
        self._grad_fresh = False
        self.gemm_sched = self.base_sched
        if self.grad_sync is not None:
            self.grad_sync.end_backward()

    def workspace(self, B, T, act=BF16) -> Workspace:
        key = (B, T, act)
        if key not in self._ws:
            self._ws.clear()  # one live shape at a time keeps HBM use bounded
            torch.cuda.empty_cache()
            self._ws[key] = Workspace(self.cfg, B, T, self.vpad, self.device, act)
        return self._ws[key]

    # ---- precision ----------------------------------------------------------------------------------
    def compute_dtype(self) -> torch.dtype:
        """bf16 under ``torch.autocast("cuda", torch.bfloat16)`` (the reference trainer,
        train_gpt2_distributed.py:404), fp32 without autocast (the reference model.py run plain), unless
        ``model.precision`` forces "bf16" / "fp32"."""
        p = getattr(self.model, "precision", "auto")
        if p == "bf16":
            return BF16
        if p == "fp32":
            return F32
        if p != "auto":
            raise ValueError(f"GPT2.precision must be 'auto', 'bf16' or 'fp32' (got {p!r})")
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            if dt != BF16:
                raise NotImplementedError(f"autocast dtype {dt}: the MI355X kernels implement bf16 autocast only")
            return BF16
        return F32

    def w(self, name, act):
        """GEMM operand of a weight: the bf16 shadow under autocast, the fp32 master weight otherwise
        (wte as its zero-padded [Vp, C] slot for the tied lm_head)."""
        if act == BF16:
            return self.w16(name)
        return self._flat("p", name)

    def _grad_enabled(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in self._params)

    # ---- public entry -------------------------------------------------------------------------------
    def forward(self, idx: torch.Tensor, labels: Optional[torch.Tensor]):
        if self._grad_enabled():
            return _GPT2Step.apply(self, idx, labels, *self._params)
        with torch.no_grad():
            return self._forward(idx, labels, False)

    # (autograd.Function.forward runs with grad mode off: whether a backward will follow is decided here)
    def backbone_forward(self, idx: torch.Tensor) -> torch.Tensor:
        if self._grad_enabled():
            return _TrunkFn.apply(self, idx, *self._params)
        with torch.no_grad():
            return self._trunk_forward_module(idx, False)

    def sub_forward(self, kind: str, layer: int, x: torch.Tensor) -> torch.Tensor:
        if self._grad_enabled() or x.requires_grad:
            return _SubFn.apply(self, kind, layer, x, *self._params)
        with torch.no_grad():
            return self._sub_forward(kind, layer, x, False)[0]

    # ---- shared kernel sequences --------------------------------------------------------------------
    def _dropout(self):
        if not self.model.training:
            return 0.0, 0.0
        return float(self.cfg.resid_pdrop), float(self.cfg.attn_pdrop)

    def _seeds(self, step_seed):
        return site_seeds(self.base_seed, step_seed, self.cfg.n_layer)

    def _next_seeds(self):
        self._step_seed += 1
        return self._seeds(self._step_seed)

    def _ln_fwd(self, x, pre, out, mean, rstd, M, out_f32=None):
        cfg = self.cfg
        K.layernorm_fwd(x, self.p(pre + ".weight"), self.p(pre + ".bias"), out, None, mean, rstd, M, cfg.n_embd,
                        cfg.layer_norm_eps)
        if out_f32 is not None:  # the fp32 copy a stand-alone Backbone returns (autocast LN output is fp32)
            K.layernorm_fwd(x, self.p(pre + ".weight"), self.p(pre + ".bias"), None, out_f32, mean, rstd, M,
                            cfg.n_embd, cfg.layer_norm_eps)

    def _attn_fwd(self, l, A, resid, out, B, T, act, pr, pa, seeds):
        """A.ln1 -> qkv GEMM -> flash attention -> proj GEMM: out = resid + drop(proj(attn))."""
        C, H = self.cfg.n_embd, self.cfg.n_head
        M = B * T
        pre = f"transformer.h.{l}."
        self._gemm(K.FWD, K.EPI_BF16, M, 3 * C, C, A.ln1, C, self.w(pre + "attn.qkv.weight", act), C, A.qkv, 3 * C,
               bias=self.p(pre + "attn.qkv.bias"))
        with self._probe("attn_fwd"):
            K.attn_fwd(A.qkv, A.ao, A.lse, B, T, H, C // H, pa, seeds[("attn", l)])
        self._gemm(K.FWD, K.EPI_RESID, M, C, C, A.ao, C, self.w(pre + "attn.proj.weight", act), C, out, C,
               bias=self.p(pre + "attn.proj.bias"), resid=resid, p_drop=pr, seed=seeds[("proj", l)])

    def _mlp_fwd(self, l, A, resid, out, M, act, pr, seeds):
        """A.ln2 -> fc1 GEMM + GELU + drop1 (also the masked GELU derivative) -> fc2 GEMM: out = resid + drop2(.)."""
        C = self.cfg.n_embd
        pre = f"transformer.h.{l}."
        with self._probe("fc1_fwd"):
            self._gemm(K.FWD, K.EPI_GELU, M, 4 * C, C, A.ln2, C, self.w(pre + "mlp.fc1.weight", act), C, A.h, 4 * C,
                   bias=self.p(pre + "mlp.fc1.bias"), aux=A.dgelu, ldaux=4 * C, p_drop=pr, seed=seeds[("fc1", l)])
        self._gemm(K.FWD, K.EPI_RESID, M, C, 4 * C, A.h, 4 * C, self.w(pre + "mlp.fc2.weight", act), 4 * C, out, C,
               bias=self.p(pre + "mlp.fc2.bias"), resid=resid, p_drop=pr, seed=seeds[("fc2", l)])

    def _block_fwd(self, l, A, x_in, x_out, B, T, act, pr, pa, seeds):
        M = B * T
        pre = f"transformer.h.{l}."
        self._ln_fwd(x_in, pre + "ln1", A.ln1, A.m1, A.r1, M)
        self._attn_fwd(l, A, x_in, A.xmid, B, T, act, pr, pa, seeds)
        self._ln_fwd(A.xmid, pre + "ln2", A.ln2, A.m2, A.r2, M)
        self._mlp_fwd(l, A, A.xmid, x_out, M, act, pr, seeds)

    def _trunk_fwd(self, ws, idx, B, T, T_valid, act, pr, pa, seeds, lnf_f32=None):
        C, L = self.cfg.n_embd, self.cfg.n_layer
        x = ws.x
        self._unit("embed")
        K.embed_fwd(idx, self.p("transformer.wte.weight"), self.p("transformer.wpe.weight"), x[0], B, T, C, pr,
                    seeds["embd"], T_valid=T_valid)
        for l in range(L):
            self._unit(f"h.{l}")
            self._block_fwd(l, ws.blocks[l], x[l], x[l + 1], B, T, act, pr, pa, seeds)
        self._unit("head")
        self._ln_fwd(x[L], "transformer.ln_f", ws.lnf, ws.mf, ws.rf, B * T, out_f32=lnf_f32)

    # -- backward pieces. The data-parallel 1/world factor (GradHooks.begin_backward) enters once, with the
    # gradient that starts the backward (the lm_head dgrad/wgrad alpha, or the incoming dy): every op
    # below is linear in it, so no GEMM here needs a scale. --
    def _wgrad(self, S, act, m, n, M, a, lda, b, ldb, out):
        # dW[m][n] += dY[:, :m]^T X[:, :n] over the M tokens
        with self._probe("wgrad"):
            self._wgrad_launch(S, act, m, n, M, a, lda, b, ldb, out)

    def _wgrad_launch(self, S, act, m, n, M, a, lda, b, ldb, out):
        if act == F32:
            self._gemm(K.WGRAD, K.EPI_F32, m, n, M, a, lda, b, ldb, out, n, accumulate=not self._grad_fresh)
        elif m % 64 == 0 and n % 64 == 0:  # (1.5B: a partial 64-multiple last tile, 1600 / 4800)
            self._gemm_wgrad(m, n, M, a, lda, b, ldb, out, n, accumulate=not self._grad_fresh, workspace=S.wgrad_ws,
                         splits=K_wgrad_splits(m, n, M))
        else:
            assert not self._grad_fresh, "atomic weight gradients need a zeroed arena"
            s = self.WGRAD_SPLITS
            while s > 1 and M % (64 * s) != 0:
                s //= 2
            self._gemm(K.WGRAD, K.EPI_ATOMIC, m, n, M, a, lda, b, ldb, out, n, splits=s)

    def _dgrad(self, act, M, out, dy, wname, n_in, n_out, epi=K.EPI_BF16, **kw):
        # dX[M][n_in] = dY[M][n_out] . W[n_out][n_in]: the forward layout against W^T when it exists
        if act == BF16 and self.wT_ok(wname):
            self._gemm(K.FWD, epi, M, n_in, n_out, dy, n_out, self.wT16(wname), n_out, out, n_in, **kw)
        else:
            self._gemm(K.DGRAD, epi, M, n_in, n_out, dy, n_out, self.w(wname, act), n_in, out, n_in, **kw)

    # A GPT2Block's four weight gradients as two grouped launches (gpt2mi_gemm_wgrad_grouped: one split-K launch + one
    # reduction each), each issued right after the dgrad that finishes its operands: fc2 + fc1 after the fc1 dgrad
    # (72 tiles x 7 splits at GPT-2 124M: 1.97 rounds of 256 CUs), proj + qkv after the qkv dgrad (36 x 7: one round),
    # instead of four launches at 9 / 28 / 7 / 7 splits with four reductions. Same operands, fewer slab bytes to reduce
    # (proj at 7 splits instead of 28): block weight gradients + reductions 9.43 -> 9.27 ms a step (profiles/r6d/).
    # One group of all four at the end of the block (round 6's first build, which needs a second buffer for the proj
    # branch's gradient) measured the same (profiles/r6c/). bf16 autocast with fp32 slabs, widths multiples of 256.
    # GPT2MI_GROUP_WGRADS=0: the four launches (same-box A/B runs of the step).
    GROUP_WGRADS = os.environ.get("GPT2MI_GROUP_WGRADS", "1") != "0"

    def _group_ok(self, act, M) -> bool:
        return self.GROUP_WGRADS and act == BF16 and self.cfg.n_embd % 256 == 0 and M % 128 == 0 and \
            not self.wgrad_bf16_slabs

    def _wgrad_or_defer(self, S, act, m, n, M, a, lda, b, ldb, out, defer):
        if defer is None:
            self._wgrad(S, act, m, n, M, a, lda, b, ldb, out)
        else:
            defer.append((m, n, a, lda, b, ldb, out))

    def _wgrad_group(self, S, M, probs):
        with self._probe("wgrad"):
            K.gemm_wgrad_grouped(probs, M, accumulate=not self._grad_fresh, workspace=S.wgrad_ws,
                                 splits=K_wgrad_group_splits([(q[0], q[1]) for q in probs], M), sched=self._sched())

    def _mlp_bwd(self, l, A, S, dY, dx_out, M, act, defer=None):
        """dY = grad of the fc2 output with drop2 applied (its bias grad already taken) -> dx_out = grad of
        the MLP input (bf16), weight grads of fc1/fc2 (or their problems appended to ``defer``) and the fc1 bias grad."""
        C = self.cfg.n_embd
        pre = f"transformer.h.{l}."
        self._dgrad(act, M, S.dU, dY, pre + "mlp.fc2.weight", 4 * C, C, K.EPI_GELU_BWD, aux=A.dgelu, ldaux=4 * C,
                    dbias=self.g(pre + "mlp.fc1.bias"))
        self._wgrad_or_defer(S, act, C, 4 * C, M, dY, C, A.h, 4 * C, self.g(pre + "mlp.fc2.weight"), defer)
        self._dgrad(act, M, dx_out, S.dU, pre + "mlp.fc1.weight", C, 4 * C)
        self._wgrad_or_defer(S, act, 4 * C, C, M, S.dU, 4 * C, A.ln2, C, self.g(pre + "mlp.fc1.weight"), defer)
        if defer:  # fc2 + fc1, while their operands are the latest written
            self._wgrad_group(S, M, defer)
            defer.clear()

    def _attn_bwd(self, l, A, S, dY, dx_out, B, T, act, pa, seeds, defer=None):
        """dY = grad of the proj output with resid_drop applied -> dx_out = grad of the attention input."""
        C, H = self.cfg.n_embd, self.cfg.n_head
        M = B * T
        pre = f"transformer.h.{l}."
        self._dgrad(act, M, dx_out, dY, pre + "attn.proj.weight", C, C)
        self._wgrad_or_defer(S, act, C, C, M, dY, C, A.ao, C, self.g(pre + "attn.proj.weight"), defer)
        K.attn_bwd(A.qkv, A.ao, dx_out, A.lse, S.delta, S.dqkv, B, T, H, C // H, pa, seeds[("attn", l)],
                   colsum=S.dqkv_cs)
        self._dgrad(act, M, dx_out, S.dqkv, pre + "attn.qkv.weight", C, 3 * C)
        self._wgrad_or_defer(S, act, 3 * C, C, M, S.dqkv, 3 * C, A.ln1, C, self.g(pre + "attn.qkv.weight"), defer)
        if S.dqkv_cs is not None:  # qkv bias grad: sum the attention backward's 32-token partials
            K.colsum_bf16(S.dqkv_cs, self.g(pre + "attn.qkv.bias"), M // 32, 3 * C, 3 * C)
        else:
            K.colsum_bf16(S.dqkv, self.g(pre + "attn.qkv.bias"), M, 3 * C, 3 * C)

    def _block_bwd(self, l, A, S, x_in, B, T, act, pr, pa, seeds, last):
        """S.dres = grad of the block output; S.dres_bf = its fc2 branch grad (drop2 applied) ->
        S.dres = grad of the block input; unless `last`, S.dres_bf = the fc2 branch grad of block l-1."""
        C = self.cfg.n_embd
        M = B * T
        pre = f"transformer.h.{l}."
        grp = [] if self._group_ok(act, M) else None
        self._mlp_bwd(l, A, S, S.dres_bf, S.dln, M, act, grp)
        K.layernorm_bwd(A.xmid, self.p(pre + "ln2.weight"), A.m2, A.r2, S.dln, S.dres, self.g(pre + "ln2.weight"),
                        self.g(pre + "ln2.bias"), S.dres_bf, self.g(pre + "attn.proj.bias"), M, C, pr,
                        seeds[("proj", l)])
        self._attn_bwd(l, A, S, S.dres_bf, S.dln, B, T, act, pa, seeds, grp)
        if grp:  # proj + qkv, before LN1's backward overwrites dres_bf (the proj weight gradient's operand)
            self._wgrad_group(S, M, grp)
        if not last:
            K.layernorm_bwd(x_in, self.p(pre + "ln1.weight"), A.m1, A.r1, S.dln, S.dres,
                            self.g(pre + "ln1.weight"), self.g(pre + "ln1.bias"), S.dres_bf,
                            self.g(f"transformer.h.{l-1}.mlp.fc2.bias"), M, C, pr, seeds[("fc2", l - 1)])
        else:
            K.layernorm_bwd(x_in, self.p(pre + "ln1.weight"), A.m1, A.r1, S.dln, S.dres,
                            self.g(pre + "ln1.weight"), self.g(pre + "ln1.bias"), None, None, M, C)

    def _trunk_bwd(self, ws, sv: _Saved):
        """ws.dln = grad of the ln_f output -> every trunk gradient (ln_f, blocks, embeddings)."""
        C, L = self.cfg.n_embd, self.cfg.n_layer
        idx, pr, pa, seeds, act = sv.idx, sv.pr, sv.pa, sv.seeds, sv.act
        B, T = idx.shape
        M = B * T
        x = ws.x
        # ln_f backward starts the residual gradient; emits the fc2 branch grad of the last block
        self._unit_bwd("head")
        K.layernorm_bwd(x[L], self.p("transformer.ln_f.weight"), ws.mf, ws.rf, ws.dln, ws.dres,
                        self.g("transformer.ln_f.weight"), self.g("transformer.ln_f.bias"), ws.dres_bf,
                        self.g(f"transformer.h.{L-1}.mlp.fc2.bias"), M, C, pr, seeds[("fc2", L - 1)], dres_init=True)
        self._ready("head")
        for l in reversed(range(L)):
            self._unit_bwd(f"h.{l}")
            self._block_bwd(l, ws.blocks[l], ws, x[l], B, T, act, pr, pa, seeds, last=(l == 0))
            self._ready(f"h.{l}")
        # embedding backward: atomics into the tied wte grad (the lm_head wgrad already wrote it)
        self._unit_bwd("embed")
        K.embed_bwd(idx, ws.dres, self.g("transformer.wte.weight"), self.g("transformer.wpe.weight"), B, T, C, pr,
                    seeds["embd"], T_valid=sv.T)
        self._ready("embed")

    # ---- the whole step ------------------------------------------------------------------------------
    def _pad(self, idx, labels):
        B, T = idx.shape
        if idx.dtype != torch.int64:
            idx = idx.long()
        idx = idx.contiguous()
        if labels is not None:
            if labels.shape != idx.shape:
                raise ValueError(f"labels shape {tuple(labels.shape)} != idx shape {tuple(idx.shape)}")
            labels = labels.contiguous().long()
        Tp = padded_len(T)
        if Tp != T:  # pad to the attention tile: token 0, label ignore_index, zero embedding rows
            idx = F.pad(idx, (0, Tp - T))
            if labels is not None:
                labels = F.pad(labels, (0, Tp - T), value=-100)
        return idx, labels, T

    def _forward(self, idx, labels, need_grad):
        cfg = self.cfg
        self.gemm_sched = self.base_sched  # (a backward that raised midway left its flags)
        V, Vp, C = cfg.vocab_size, self.vpad, cfg.n_embd
        idx, labels, T = self._pad(idx, labels)
        B, Tp = idx.shape
        M = B * Tp
        act = self.compute_dtype()
        self._sync_shadows(act, need_grad)
        ws = self.workspace(B, Tp, act)
        pr, pa = self._dropout()
        seeds = self._next_seeds()
        self._fwd_token += 1
        self._saved = _Saved(idx, labels, T, pr, pa, seeds, act)
        self._trunk_fwd(ws, idx, B, Tp, T, act, pr, pa, seeds)
        logits = torch.empty(M, Vp, dtype=act, device=self.device)  # fresh: the caller may keep it
        with self._probe("lm_head_fwd"):
            self._gemm(K.FWD, K.EPI_BF16, M, Vp, C, ws.lnf, C, self.w("transformer.wte.weight", act), C, logits, Vp)
        loss = None
        if labels is not None:
            loss = torch.empty((), dtype=F32, device=self.device)  # fresh: callers may keep it across steps
            K.xent_fwd(logits, Vp, labels, ws.loss_rows, ws.lse_ce, ws.dlogits if need_grad else None, Vp, M, V,
                       loss, ws.inv_count)
        out = logits.view(B, Tp, Vp)
        if Tp != T:  # compact rows, so the reference's own logits.view(-1, V) (model.py:357-358) merges B and T
            out = out[:, :T].contiguous()
        return out[..., :V], loss

    def _backward(self, grad_logits, grad_loss):
        cfg = self.cfg
        sv = self._saved
        B, Tp = sv.idx.shape
        C, V, Vp = cfg.n_embd, cfg.vocab_size, self.vpad
        M = B * Tp
        act = sv.act
        ws = self.workspace(B, Tp, act)
        use_loss = grad_loss is not None and sv.labels is not None
        if not use_loss and grad_logits is None:
            self._prepare_grads()
            return
        gs = self._begin_grads(act, full=True)
        alpha_dev = None
        if use_loss:  # d(loss)/d(logit) = grad_loss / #valid labels times the unscaled dlogits
            K.scale_mul(grad_loss.reshape(1).to(F32), ws.inv_count, ws.dscale)
            alpha_dev = ws.dscale
        if grad_logits is not None:  # a loss on the returned logits: dlogits = alpha*dlogits + g
            g = grad_logits.to(act).contiguous()
            K.dlogits_accum(ws.dlogits, Vp, g, V, B, Tp, sv.T, V, alpha_dev=alpha_dev, init=not use_loss)
            alpha_dev = None
        # lm_head (tied): dlnf = gs * dlogits @ wte ; dwte (+)= gs * dlogits^T @ lnf
        with self._probe("lm_head_dgrad"):
            self._dgrad(act, M, ws.dln, ws.dlogits, "transformer.wte.weight", C, Vp, K.EPI_BF16, alpha_dev=alpha_dev,
                        alpha=gs)
        wte_g = self.gpad("transformer.wte.weight", Vp)
        with self._probe("lm_head_wgrad"), self._probe("wgrad"):
            if C % 64 == 0 and act == BF16 and M % 128 == 0 and Vp % 256 == 0:
                # dwte^T = lnf^T . dlogits with lnf transposed once (0.1 GB at cfg 2): one transposed GEMM operand
                # instead of two (gpt2mi_gemm_wgrad_kt; lm_head wgrad ~18 % faster, the same bits)
                if ws.lnf_t is None:
                    ws.lnf_t = torch.empty(C, M, dtype=act, device=ws.lnf.device)
                K.transpose_bf16(ws.lnf, ws.lnf_t, M, C, C, M)
                self._gemm_wgrad_kt(Vp, C, M, ws.dlogits, Vp, ws.lnf_t, M, wte_g, C, accumulate=not self._grad_fresh,
                                    alpha_dev=alpha_dev, alpha=gs, workspace=ws.wgrad_ws,
                                    splits=K_wgrad_splits(Vp, C, M))
            elif C % 64 == 0 and act == BF16:
                self._gemm_wgrad(Vp, C, M, ws.dlogits, Vp, ws.lnf, C, wte_g, C, accumulate=not self._grad_fresh,
                             alpha_dev=alpha_dev, alpha=gs, workspace=ws.wgrad_ws, splits=K_wgrad_splits(Vp, C, M))
            else:
                self._gemm(K.WGRAD, K.EPI_F32, Vp, C, M, ws.dlogits, Vp, ws.lnf, C, wte_g, C, alpha_dev=alpha_dev,
                       alpha=gs, accumulate=not self._grad_fresh)
        self._trunk_bwd(ws, sv)
        self._end_grads()

    # ---- GPT2Backbone.forward on its own -------------------------------------------------------------
    def _trunk_forward_module(self, idx, need_grad):
        self.gemm_sched = self.base_sched  # (a backward that raised midway left its flags)
        idx, _, T = self._pad(idx, None)
        B, Tp = idx.shape
        act = self.compute_dtype()
        self._sync_shadows(act, need_grad)
        ws = self.workspace(B, Tp, act)
        pr, pa = self._dropout()
        seeds = self._next_seeds()
        self._fwd_token += 1
        self._saved = _Saved(idx, None, T, pr, pa, seeds, act)
        out = torch.empty(B * Tp, self.cfg.n_embd, dtype=F32, device=self.device)
        self._trunk_fwd(ws, idx, B, Tp, T, act, pr, pa, seeds, lnf_f32=out)
        return out.view(B, Tp, -1)[:, :T]

    def _trunk_backward_module(self, dy):
        sv = self._saved
        B, Tp = sv.idx.shape
        C = self.cfg.n_embd
        ws = self.workspace(B, Tp, sv.act)
        gs = self._begin_grads(sv.act)
        dy = dy.to(F32)
        if Tp != sv.T:
            dy = F.pad(dy, (0, 0, 0, Tp - sv.T))
        dy = (dy * gs if gs != 1.0 else dy).contiguous()
        if sv.act == BF16:
            K.cast_f32_bf16(dy, ws.dln, B * Tp * C)
        else:
            ws.dln.copy_(dy.view(B * Tp, C))
        self._trunk_bwd(ws, sv)
        self._end_grads()

    # ---- GPT2Block / MLP / CausalMultiHeadSelfAttention forward on their own --------------------------
    def _sub_forward(self, kind, l, x, need_grad):
        """kind: "block" (x = residual stream, model.py:213-219), "mlp" (x = ln2 output, model.py:186-192),
        "attn" (x = ln1 output, model.py:110-159). Returns (y, saved state)."""
        self.gemm_sched = self.base_sched  # (a backward that raised midway left its flags)
        if self.store is not None:
            raise NotImplementedError("sub-module calls under FullyShardedDataParallel(reshard_after_forward=True): "
                                      "call the wrapped model")
        cfg = self.cfg
        C = cfg.n_embd
        if x.dim() != 3 or x.shape[-1] != C:
            raise ValueError(f"expected x of shape [B, T, {C}], got {tuple(x.shape)}")
        if not x.is_cuda:
            raise RuntimeError("the MI355X sub-module kernels take cuda tensors (there is no CPU fallback)")
        B, T, _ = x.shape
        if kind == "attn" and T > cfg.n_positions:
            raise ValueError(f"Sequence length {T} > model max {cfg.n_positions}")
        Tp = padded_len(T)
        M = B * Tp
        act = self.compute_dtype()
        self._sync_shadows(act, need_grad)
        xf = x.to(F32)
        if Tp != T:
            xf = F.pad(xf, (0, 0, 0, Tp - T))
        xf = xf.contiguous().view(M, C)
        pr, pa = self._dropout()
        seeds = self._next_seeds()
        self.last_seeds = seeds
        A = BlockActs.alloc(cfg, B, Tp, self.device, act, xmid=(kind == "block"))
        y = torch.empty(M, C, dtype=F32, device=self.device)
        self._unit(f"h.{l}")
        if kind == "block":
            self._block_fwd(l, A, xf, y, B, Tp, act, pr, pa, seeds)
        else:
            zero = torch.zeros(M, C, dtype=F32, device=self.device)
            if kind == "mlp":
                A.ln2 = self._to_act(xf, act)
                self._mlp_fwd(l, A, zero, y, M, act, pr, seeds)
            elif kind == "attn":
                A.ln1 = self._to_act(xf, act)
                self._attn_fwd(l, A, zero, y, B, Tp, act, pr, pa, seeds)
            else:
                raise ValueError(kind)
        state = (A, xf, B, Tp, T, act, pr, pa, seeds)
        out = y.view(B, Tp, C)[:, :T]
        if kind != "block":  # the branch output is a linear's output: bf16 under autocast (model.py:158,191)
            out = out.to(act)
        return out, state

    @staticmethod
    def _to_act(xf, act):
        if act == F32:
            return xf
        out = act_empty(*xf.shape, dtype=BF16, device=xf.device)
        K.cast_f32_bf16(xf, out, xf.numel())
        return out

    def _sub_backward(self, kind, l, state, dy):
        A, xf, B, Tp, T, act, pr, pa, seeds = state
        C = self.cfg.n_embd
        M = B * Tp
        S = Scratch(self.cfg, B, Tp, self.vpad, self.device, act, head=False)
        gs = self._begin_grads(act)
        d = dy.to(F32)
        if Tp != T:
            d = F.pad(d, (0, 0, 0, Tp - T))
        S.dres.copy_(d.reshape(M, C))
        if gs != 1.0:
            K.scale_(S.dres, gs)
        pre = f"transformer.h.{l}."
        if kind == "block":
            K.branch_bwd(S.dres, S.dres_bf, self.g(pre + "mlp.fc2.bias"), M, C, pr, seeds[("fc2", l)])
            self._block_bwd(l, A, S, xf, B, Tp, act, pr, pa, seeds, last=True)
            dx = S.dres
        else:
            site, bias = ("fc2", "mlp.fc2.bias") if kind == "mlp" else ("proj", "attn.proj.bias")
            K.branch_bwd(S.dres, S.dres_bf, self.g(pre + bias), M, C, pr, seeds[(site, l)])
            if kind == "mlp":
                self._mlp_bwd(l, A, S, S.dres_bf, S.dln, M, act)
            else:
                self._attn_bwd(l, A, S, S.dres_bf, S.dln, B, Tp, act, pa, seeds)
            if act == BF16:
                dx = torch.empty(M, C, dtype=F32, device=self.device)
                K.cast_bf16_f32(S.dln, dx, M * C)
            else:
                dx = S.dln
        if gs != 1.0:  # the grads were formed from gs*dy; the input grad leaves the node unscaled
            dx = dx / gs
        self._end_grads()
        return dx.view(B, Tp, C)[:, :T]
