"""The GPT-2 training-step engine: forward -> loss -> backward as explicit HIP kernel sequences.

One ``torch.autograd.Function`` wraps the whole network, so ``loss.backward()`` (the reference's
``train_gpt2_distributed.py:412``) runs ``Engine.backward``: every gradient is produced by the
kernels of libgpt2mi straight into the flat fp32 grad arena (``p.grad`` are views of it).

Numerics = the reference under ``torch.autocast("cuda", bfloat16)`` (train_gpt2_distributed.py:404):
bf16 GEMM operands with fp32 accumulation, fp32 residual stream / LayerNorm / softmax / loss,
fp32 master weights and grads. Dropout uses the config's p (model.py:47-51) in train mode with a
counter-based mask that backward regenerates; eval mode / p = 0 disables it.

HBM layout per (B, T) workspace (M = B*T tokens, C = n_embd, Vp = vocab padded to 128):
  residual stream x[l]          fp32 [L+1][M, C]
  per block: ln1, ln2 bf16 [M,C]; mean/rstd fp32 [M]; qkv bf16 [M,3C]; attn out bf16 [M,C];
             lse fp32 [B*H,T]; x_mid fp32 [M,C]; gelu output h and dgelu = keep/(1-p)*gelu'(u) bf16 [M,4C]
  head:      ln_f bf16 [M,C]; logits bf16 [M,Vp] (returned as a [B,T,V] view); dlogits bf16 [M,Vp]
  backward scratch: dres fp32 [M,C], dres_bf bf16 [M,C], dln bf16 [M,C], dU bf16 [M,4C],
             dqkv bf16 [M,3C], delta fp32 [B*H,T], dqkv_cs fp32 [M/32,3C]
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import _lib as K
from ._lib import wgrad_splits as K_wgrad_splits

BF16 = torch.bfloat16
F32 = torch.float32


def _mix(*xs: int) -> int:
    """64-bit seed mixing for per-site dropout streams."""
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h ^= (x + 0x9E3779B97F4A7C15 + ((h << 6) & 0xFFFFFFFFFFFFFFFF) + (h >> 2)) & 0xFFFFFFFFFFFFFFFF
        h = (h * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    return h


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


class Workspace:
    def __init__(self, cfg, B: int, T: int, vpad: int, device, act=BF16):
        L, C, H = cfg.n_layer, cfg.n_embd, cfg.n_head
        M = B * T
        e = lambda *s, dt=act: torch.empty(*s, dtype=dt, device=device)  # noqa: E731
        self.act = act
        self.B, self.T, self.M = B, T, M
        self.x = e(L + 1, M, C, dt=F32)
        self.blocks: List[BlockActs] = []
        for _ in range(L):
            self.blocks.append(BlockActs(
                ln1=e(M, C), m1=e(M, dt=F32), r1=e(M, dt=F32), qkv=e(M, 3 * C), ao=e(M, C),
                lse=e(B * H, T, dt=F32), xmid=e(M, C, dt=F32), ln2=e(M, C), m2=e(M, dt=F32), r2=e(M, dt=F32),
                dgelu=e(M, 4 * C), h=e(M, 4 * C)))
        self.lnf = e(M, C)
        self.mf = e(M, dt=F32)
        self.rf = e(M, dt=F32)
        self.logits = e(M, vpad)
        self.dlogits = e(M, vpad)
        self.loss_rows = e(M, dt=F32)
        self.lse_ce = e(M, dt=F32)
        self.inv_count = e(1, dt=F32)
        self.dscale = e(1, dt=F32)
        # backward scratch
        self.dres = e(M, C, dt=F32)
        self.dres_bf = e(M, C)
        self.dln = e(M, C)
        self.dU = e(M, 4 * C)
        self.dqkv = e(M, 3 * C)
        self.delta = e(B * H, T, dt=F32)
        # bf16 path: the attention backward writes 32-token partial column sums of dqkv (qkv bias grad)
        self.dqkv_cs = e(M // 32, 3 * C, dt=F32) if act == BF16 else None
        # split-K slabs of the 256x256 wgrad GEMMs
        wshapes = [(3 * C, C), (C, C), (4 * C, C), (C, 4 * C), (vpad, C)]
        need = max((K_wgrad_splits(m, n, M) * m * n if K_wgrad_splits(m, n, M) > 1 else 0)
                   for m, n in wshapes) if C % 256 == 0 and act == BF16 else 0
        self.wgrad_ws = e(max(need, 4), dt=F32)


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


class _GPT2Step(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, idx, labels, need_grad, *params):
        ctx.set_materialize_grads(False)
        logits, loss = engine._forward(idx, labels, need_grad)
        ctx.engine = engine
        ctx.token = engine._fwd_token
        ctx.n_params = len(params)
        ctx.mark_non_differentiable(logits)
        return logits, loss

    @staticmethod
    def backward(ctx, grad_logits, grad_loss):
        eng = ctx.engine
        if grad_logits is not None:
            raise NotImplementedError("gradients through the returned logits are not supported; "
                                      "backpropagate the returned loss")
        if ctx.token != eng._fwd_token:
            raise RuntimeError("GPT2 activations were overwritten by a later forward before this backward "
                               "(one forward/backward in flight per model)")
        eng._backward(grad_loss)
        return (None, None, None, None) + (None,) * ctx.n_params


class Engine:
    """Owns the workspaces, the bf16 weight shadow and the grad arena of one GPT2 model."""

    WGRAD_SPLITS = 4

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
        self._ws: Dict[tuple, Workspace] = {}
        self._fwd_token = 0
        self._step_seed = 0
        self.base_seed = 1234
        self.grad_sync = None  # set by DDP wrappers: called as grad_sync(event, **kw)
        self._params = list(model.parameters())
        self._grads_bound = False
        self.params_by_name = dict(model.named_parameters())
        self.probes: Dict[str, list] = {}  # name -> [(start_event, end_event)] recorded when armed
        if not hasattr(K, "load") or self.device.type != "cuda":
            raise RuntimeError("the engine needs the model on a cuda (MI355X) device")
        K.load()
        self.refresh_shadow()

    # ---- live per-kernel timing (bench.py): HIP events on the launch stream around named launches ----
    def _probe(self, name):
        lst = self.probes.get(name)
        if lst is None:
            return _NullCtx
        return _EventCtx(lst)

    # ---- parameter views ------------------------------------------------------------------------------
    def _off(self, name: str) -> int:
        return self.layout.slots[name].offset

    def p(self, name):  # fp32 master view
        return self.layout.view(self.model.arena, name)

    def g(self, name):  # fp32 grad view
        return self.layout.view(self.grad, name)

    def w16(self, name):  # bf16 shadow view (flat)
        s = self.layout.slots[name]
        return self.shadow[s.offset:s.offset + s.reserved]

    def refresh_shadow(self):
        """bf16 copy of the fp32 master weights the GEMMs read. The fused optimizer rewrites it in its
        own pass; after any other in-place update (torch optimizers, load_state_dict) it is re-cast."""
        K.cast_f32_bf16(self.model.arena, self.shadow, self.model.arena.numel())
        self._shadow_versions = self._versions()
        self._shadowT_stale = True

    def _versions(self):
        return tuple(p._version for p in self._params)

    def mark_shadow_fresh(self):
        self._shadow_versions = self._versions()
        self._shadowT_stale = True

    def _rows(self, name):
        sl = self.layout.slots[name]
        return sl.reserved // sl.shape[1]  # wte: the vocab-padded row count

    def wT_ok(self, name) -> bool:
        sl = self.layout.slots[name]
        return self._rows(name) % 64 == 0 and sl.shape[1] % 64 == 0

    def _refresh_shadowT(self):
        # every transposable weight in one launch (49 separate 64x64-tile launches cost 0.28 ms per step)
        if getattr(self, "_tdesc", None) is None:
            rows, tiles = [], 0
            for n in self._t_weights:
                if self.wT_ok(n):
                    sl = self.layout.slots[n]
                    R, Cc = self._rows(n), sl.shape[1]
                    rows.append((sl.offset, R, Cc, tiles))
                    tiles += (R // 64) * (Cc // 64)
            self._tdesc = (torch.tensor(rows, dtype=torch.int64, device=self.device) if rows else None, len(rows),
                           tiles)
        desc, n, tiles = self._tdesc
        if n:
            K.transpose_bf16_batched(self.shadow, self.shadowT, desc, n, tiles)
        self._shadowT_stale = False

    def wT16(self, name):  # bf16 W^T view (flat, [in][out_padded])
        s = self.layout.slots[name]
        return self.shadowT[s.offset:s.offset + s.reserved]

    def _maybe_refresh_shadow(self):
        if self._versions() != self._shadow_versions:
            self.refresh_shadow()

    # ---- grads ---------------------------------------------------------------------------------------
    def bind_grads(self):
        for name, p in self.params_by_name.items():
            if name == "lm_head.weight":
                continue
            p.grad = self.layout.view(self.grad, name)
        self._grads_bound = True

    def zero_grad(self):
        K.zero_(self.grad)

    def _prepare_grads(self):
        """Accumulate into the arena when p.grad are its views; start from zero after a
        zero_grad(set_to_none=True) (every p.grad None)."""
        ps = [p for n, p in self.params_by_name.items()]
        if all(p.grad is None for p in ps):
            self.zero_grad()
            self.bind_grads()
            return
        for n, p in self.params_by_name.items():
            if p.grad is None or p.grad.data_ptr() != self.layout.view(self.grad, n).data_ptr():
                raise RuntimeError(f"{n}.grad is not a view of the engine's grad arena; zero grads with "
                                   "set_to_none=True or the model's optimizer before backward")

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
        s = self.layout.slots[name]
        return self.model.arena[s.offset:s.offset + s.reserved]

    # ---- public entry -------------------------------------------------------------------------------
    def forward(self, idx: torch.Tensor, labels: Optional[torch.Tensor]):
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self._params)
        if need_grad and labels is None:
            need_grad = False
        if need_grad:
            return _GPT2Step.apply(self, idx, labels, True, *self._params)
        with torch.no_grad():
            return self._forward(idx, labels, False)

    # ---- forward ------------------------------------------------------------------------------------
    def _dropout(self):
        if not self.model.training:
            return 0.0, 0.0
        return float(self.cfg.resid_pdrop), float(self.cfg.attn_pdrop)

    def _seeds(self, step_seed):
        L = self.cfg.n_layer
        s = {"embd": _mix(self.base_seed, step_seed, 0xE)}
        for l in range(L):
            for k, site in enumerate(("attn", "proj", "fc1", "fc2")):
                s[(site, l)] = _mix(self.base_seed, step_seed, l, k + 1)
        return s

    def _forward(self, idx, labels, need_grad):
        cfg = self.cfg
        B, T = idx.shape
        C, H, L, V = cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.vocab_size
        Vp = self.vpad
        M = B * T
        if idx.dtype != torch.int64:
            idx = idx.long()
        idx = idx.contiguous()
        if labels is not None:
            labels = labels.contiguous().long()
        act = self.compute_dtype()
        if act == BF16:
            self._maybe_refresh_shadow()
            if self._shadowT_stale and need_grad:
                self._refresh_shadowT()
        ws = self.workspace(B, T, act)
        W = lambda n: self.w(n, act)  # noqa: E731
        pr, pa = self._dropout()
        self._step_seed += 1
        seeds = self._seeds(self._step_seed)
        self._fwd_token += 1
        self._saved = (idx, labels, pr, pa, seeds, act)

        x = ws.x
        K.embed_fwd(idx, self.p("transformer.wte.weight"), self.p("transformer.wpe.weight"), x[0], B, T, C, pr,
                    seeds["embd"])
        for l in range(L):
            A = ws.blocks[l]
            pre = f"transformer.h.{l}."
            K.layernorm_fwd(x[l], self.p(pre + "ln1.weight"), self.p(pre + "ln1.bias"), A.ln1, None, A.m1, A.r1,
                            M, C, cfg.layer_norm_eps)
            K.gemm(K.FWD, K.EPI_BF16, M, 3 * C, C, A.ln1, C, W(pre + "attn.qkv.weight"), C, A.qkv, 3 * C,
                   bias=self.p(pre + "attn.qkv.bias"))
            with self._probe("attn_fwd"):
                K.attn_fwd(A.qkv, A.ao, A.lse, B, T, H, C // H, pa, seeds[("attn", l)])
            K.gemm(K.FWD, K.EPI_RESID, M, C, C, A.ao, C, W(pre + "attn.proj.weight"), C, A.xmid, C,
                   bias=self.p(pre + "attn.proj.bias"), resid=x[l], p_drop=pr, seed=seeds[("proj", l)])
            K.layernorm_fwd(A.xmid, self.p(pre + "ln2.weight"), self.p(pre + "ln2.bias"), A.ln2, None, A.m2, A.r2,
                            M, C, cfg.layer_norm_eps)
            with self._probe("fc1_fwd"):
                K.gemm(K.FWD, K.EPI_GELU, M, 4 * C, C, A.ln2, C, W(pre + "mlp.fc1.weight"), C, A.h, 4 * C,
                       bias=self.p(pre + "mlp.fc1.bias"), aux=A.dgelu, ldaux=4 * C, p_drop=pr, seed=seeds[("fc1", l)])
            K.gemm(K.FWD, K.EPI_RESID, M, C, 4 * C, A.h, 4 * C, W(pre + "mlp.fc2.weight"), 4 * C, x[l + 1], C,
                   bias=self.p(pre + "mlp.fc2.bias"), resid=A.xmid, p_drop=pr, seed=seeds[("fc2", l)])
        K.layernorm_fwd(x[L], self.p("transformer.ln_f.weight"), self.p("transformer.ln_f.bias"), ws.lnf, None,
                        ws.mf, ws.rf, M, C, cfg.layer_norm_eps)
        with self._probe("lm_head_fwd"):
            K.gemm(K.FWD, K.EPI_BF16, M, Vp, C, ws.lnf, C, W("transformer.wte.weight"), C, ws.logits, Vp)
        loss = None
        if labels is not None:
            loss = torch.empty((), dtype=F32, device=self.device)  # fresh: callers may keep it across steps
            K.xent_fwd(ws.logits, Vp, labels, ws.loss_rows, ws.lse_ce, ws.dlogits if need_grad else None, Vp, M, V,
                       loss, ws.inv_count)
        logits = ws.logits.view(B, T, Vp)[:, :, :V]
        return logits, loss

    # ---- backward -----------------------------------------------------------------------------------
    def _backward(self, grad_loss: torch.Tensor):
        cfg = self.cfg
        idx, labels, pr, pa, seeds, act = self._saved
        B, T = idx.shape
        C, H, L = cfg.n_embd, cfg.n_head, cfg.n_layer
        Vp = self.vpad
        M = B * T
        ws = self.workspace(B, T, act)
        W = lambda n: self.w(n, act)  # noqa: E731
        self._prepare_grads()
        if grad_loss is None:
            return
        grad_loss = grad_loss.reshape(1).to(F32)
        K.scale_mul(grad_loss, ws.inv_count, ws.dscale)  # d(loss)/d(logit) scale = grad / #valid
        sync = self.grad_sync
        S = self.WGRAD_SPLITS
        while S > 1 and M % (64 * S) != 0:
            S //= 2

        def wgrad(m, n, a, lda, b, ldb, out):
            # dW[m][n] += dY[:, :m]^T X[:, :n] over the M tokens
            if act == F32:
                K.gemm(K.WGRAD, K.EPI_F32, m, n, M, a, lda, b, ldb, out, n, accumulate=True)
            elif m % 256 == 0 and n % 256 == 0:
                K.gemm_wgrad(m, n, M, a, lda, b, ldb, out, n, accumulate=True, workspace=ws.wgrad_ws,
                             splits=K_wgrad_splits(m, n, M))
            else:
                K.gemm(K.WGRAD, K.EPI_ATOMIC, m, n, M, a, lda, b, ldb, out, n, splits=S)
        x = ws.x

        def dgrad(out, dy, wname, n_in, n_out, epi=K.EPI_BF16, **kw):
            # dX[M][n_in] = dY[M][n_out] . W[n_out][n_in]: the forward layout against W^T when it exists
            if act == BF16 and self.wT_ok(wname):
                K.gemm(K.FWD, epi, M, n_in, n_out, dy, n_out, self.wT16(wname), n_out, out, n_in, **kw)
            else:
                K.gemm(K.DGRAD, epi, M, n_in, n_out, dy, n_out, W(wname), n_in, out, n_in, **kw)

        # lm_head (tied): dlnf = dlogits @ wte ; dwte (+)= dlogits^T @ lnf
        with self._probe("lm_head_dgrad"):
            dgrad(ws.dln, ws.dlogits, "transformer.wte.weight", C, Vp, K.EPI_BF16, alpha_dev=ws.dscale)
        wte_g = self.layout.padded_view(self.grad, "transformer.wte.weight", Vp)
        with self._probe("lm_head_wgrad"):
            if C % 256 == 0 and act == BF16:
                K.gemm_wgrad(Vp, C, M, ws.dlogits, Vp, ws.lnf, C, wte_g, C, accumulate=True, alpha_dev=ws.dscale,
                             workspace=ws.wgrad_ws, splits=K_wgrad_splits(Vp, C, M))
            else:
                K.gemm(K.WGRAD, K.EPI_F32, Vp, C, M, ws.dlogits, Vp, ws.lnf, C, wte_g, C, alpha_dev=ws.dscale,
                       accumulate=True)
        # ln_f backward starts the residual gradient; emits the fc2 branch grad of the last block
        K.layernorm_bwd(x[L], self.p("transformer.ln_f.weight"), ws.mf, ws.rf, ws.dln, ws.dres,
                        self.g("transformer.ln_f.weight"), self.g("transformer.ln_f.bias"), ws.dres_bf,
                        self.g(f"transformer.h.{L-1}.mlp.fc2.bias"), M, C, pr, seeds[("fc2", L - 1)], dres_init=True)
        if sync:
            sync("ready", name="transformer.ln_f.bias")
        for l in reversed(range(L)):
            A = ws.blocks[l]
            pre = f"transformer.h.{l}."
            # ---- MLP: dY2 = dres_bf (fc2 dropout applied), db2 done by the LN bwd above
            dgrad(ws.dU, ws.dres_bf, pre + "mlp.fc2.weight", 4 * C, C, K.EPI_GELU_BWD, aux=A.dgelu, ldaux=4 * C,
                  dbias=self.g(pre + "mlp.fc1.bias"))
            wgrad(C, 4 * C, ws.dres_bf, C, A.h, 4 * C, self.g(pre + "mlp.fc2.weight"))
            dgrad(ws.dln, ws.dU, pre + "mlp.fc1.weight", C, 4 * C)
            wgrad(4 * C, C, ws.dU, 4 * C, A.ln2, C, self.g(pre + "mlp.fc1.weight"))
            K.layernorm_bwd(A.xmid, self.p(pre + "ln2.weight"), A.m2, A.r2, ws.dln, ws.dres, self.g(pre + "ln2.weight"),
                            self.g(pre + "ln2.bias"), ws.dres_bf, self.g(pre + "attn.proj.bias"), M, C, pr,
                            seeds[("proj", l)])
            # ---- attention
            dgrad(ws.dln, ws.dres_bf, pre + "attn.proj.weight", C, C)
            wgrad(C, C, ws.dres_bf, C, A.ao, C, self.g(pre + "attn.proj.weight"))
            K.attn_bwd(A.qkv, A.ao, ws.dln, A.lse, ws.delta, ws.dqkv, B, T, H, C // H, pa, seeds[("attn", l)],
                       colsum=ws.dqkv_cs)
            dgrad(ws.dln, ws.dqkv, pre + "attn.qkv.weight", C, 3 * C)
            wgrad(3 * C, C, ws.dqkv, 3 * C, A.ln1, C, self.g(pre + "attn.qkv.weight"))
            if ws.dqkv_cs is not None:  # qkv bias grad: sum the attention backward's 32-token partials
                K.colsum_bf16(ws.dqkv_cs, self.g(pre + "attn.qkv.bias"), M // 32, 3 * C, 3 * C)
            else:
                K.colsum_bf16(ws.dqkv, self.g(pre + "attn.qkv.bias"), M, 3 * C, 3 * C)
            if l > 0:
                K.layernorm_bwd(x[l], self.p(pre + "ln1.weight"), A.m1, A.r1, ws.dln, ws.dres,
                                self.g(pre + "ln1.weight"), self.g(pre + "ln1.bias"), ws.dres_bf,
                                self.g(f"transformer.h.{l-1}.mlp.fc2.bias"), M, C, pr, seeds[("fc2", l - 1)])
            else:
                K.layernorm_bwd(x[l], self.p(pre + "ln1.weight"), A.m1, A.r1, ws.dln, ws.dres,
                                self.g(pre + "ln1.weight"), self.g(pre + "ln1.bias"), None, None, M, C)
            if sync:
                sync("ready", name=pre + "ln1.weight")
        K.embed_bwd(idx, ws.dres, self.g("transformer.wte.weight"), self.g("transformer.wpe.weight"), B, T, C, pr,
                    seeds["embd"])
        if sync:
            sync("ready", name="transformer.wte.weight")
