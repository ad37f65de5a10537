"""Functional CPU restatement of the reference GPT-2 (`/root/reference/model.py`) — TEST ORACLE.

Test infrastructure only (see ``oracle/__init__.py``). Two numeric modes:

* ``"fp32"``: the reference run on the CPU in fp32 (what ``model.py`` computes with no autocast).
* ``"bf16"``: an explicit-cast restatement of the CUDA ``torch.autocast("cuda", bfloat16)`` policy
  the reference trainer wraps the forward in (``train_gpt2_distributed.py:404``): linear/bmm in bf16
  with fp32 accumulation and bf16 outputs; layer_norm, softmax, pow and cross_entropy upcast to fp32;
  embedding and the residual adds follow type promotion (fp32). CPU autocast uses a different policy
  (softmax/LN stay bf16), so it cannot serve as this oracle.

Everything is differentiable with torch autograd, which gives the backward oracle.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass(frozen=True)
class Cfg:
    """Mirror of ``GPT2Config`` (model.py:26-57)."""
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    resid_pdrop: float = 0.1
    attn_pdrop: float = 0.1
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02


BLOCK_KEYS = (
    "ln1.weight", "ln1.bias",
    "attn.qkv.weight", "attn.qkv.bias", "attn.proj.weight", "attn.proj.bias",
    "ln2.weight", "ln2.bias",
    "mlp.fc1.weight", "mlp.fc1.bias", "mlp.fc2.weight", "mlp.fc2.bias",
)


def param_shapes(cfg) -> "OrderedDict[str, tuple]":
    """Parameter names/shapes in ``GPT2.parameters()`` order (model.py:235-247, 95-96, 174-177, 204-210)."""
    C, V, T = cfg.n_embd, cfg.vocab_size, cfg.n_positions
    shapes = OrderedDict()
    shapes["transformer.wte.weight"] = (V, C)
    shapes["transformer.wpe.weight"] = (T, C)
    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}."
        shapes[p + "ln1.weight"] = (C,)
        shapes[p + "ln1.bias"] = (C,)
        shapes[p + "attn.qkv.weight"] = (3 * C, C)
        shapes[p + "attn.qkv.bias"] = (3 * C,)
        shapes[p + "attn.proj.weight"] = (C, C)
        shapes[p + "attn.proj.bias"] = (C,)
        shapes[p + "ln2.weight"] = (C,)
        shapes[p + "ln2.bias"] = (C,)
        shapes[p + "mlp.fc1.weight"] = (4 * C, C)
        shapes[p + "mlp.fc1.bias"] = (4 * C,)
        shapes[p + "mlp.fc2.weight"] = (C, 4 * C)
        shapes[p + "mlp.fc2.bias"] = (C,)
    shapes["transformer.ln_f.weight"] = (C,)
    shapes["transformer.ln_f.bias"] = (C,)
    return shapes


def init_params(cfg) -> "OrderedDict[str, torch.Tensor]":
    """Seed-42 init (model.py:249-268).

    ``self.apply(self._init_weights)`` is a post-order walk, so the private generator draws
    N(0, 0.02) in the order wte, wpe, then per block qkv, proj, fc1, fc2 (Linear/Embedding only);
    biases are zero and LayerNorms are (1, 0) (nn.LayerNorm defaults). lm_head is tied to wte
    (model.py:333) and draws nothing from this generator.
    """
    g = torch.Generator()
    g.manual_seed(42)
    std = cfg.initializer_range
    params = OrderedDict()
    for name, shape in param_shapes(cfg).items():
        params[name] = torch.zeros(shape, dtype=torch.float32)
    ln_names = [n for n in params if ".ln" in n and n.endswith(".weight")]
    for n in ln_names:
        params[n].fill_(1.0)
    draw = ["transformer.wte.weight", "transformer.wpe.weight"]
    for i in range(cfg.n_layer):
        p = f"transformer.h.{i}."
        draw += [p + "attn.qkv.weight", p + "attn.proj.weight", p + "mlp.fc1.weight", p + "mlp.fc2.weight"]
    for n in draw:
        params[n].normal_(mean=0.0, std=std, generator=g)
    return params


# ---------------------------------------------------------------------------------------------
# per-op restatements (mode-aware)
# ---------------------------------------------------------------------------------------------
def _bf(x: torch.Tensor) -> torch.Tensor:
    """Round to bf16 and come back to fp32 (autocast's cast; differentiable)."""
    return x.to(torch.bfloat16).to(torch.float32)


def embed(wte, wpe, idx):
    """x = wte[idx] + wpe[0..T) (model.py:295-301); fp32 under autocast (embedding not on the list)."""
    T = idx.shape[1]
    return wte[idx] + wpe[:T].unsqueeze(0)


def layer_norm(x, w, b, eps=1e-5):
    """nn.LayerNorm over the last dim, biased variance (model.py:204,210,247); fp32 under autocast."""
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) * torch.rsqrt(var + eps) * w + b


def linear(x, w, b=None, mode="fp32"):
    """nn.Linear (model.py:95-96,174-177,326). bf16 mode: bf16 operands, fp32 accumulate, bf16 out."""
    if mode == "fp32":
        y = x @ w.t()
        return y + b if b is not None else y
    y = _bf(x) @ _bf(w).t()
    if b is not None:
        y = y + _bf(b)
    return _bf(y)


def gelu_tanh(u, mode="fp32"):
    """NewGELU (model.py:63-77): 0.5u(1+tanh(sqrt(2/pi)(u+0.044715u^3))). Under autocast ``pow``
    upcasts so the chain runs in fp32 (output fp32)."""
    return 0.5 * u * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (u + 0.044715 * torch.pow(u, 3.0))))


def causal_attention(q, k, v, mode="fp32", drop=None):
    """Attention core (model.py:137-151) for q,k,v [B,H,T,D]: (q k^T)/sqrt(D), masked_fill(tril==0,
    -1e4), softmax (fp32 under autocast), then P v. bf16 mode rounds the scores (bmm output) and
    P (cast back to bf16 for the second bmm) the way autocast does."""
    D = q.shape[-1]
    T = q.shape[-2]
    att = q @ k.transpose(-2, -1)
    if mode == "bf16":
        att = _bf(att)
    att = att / math.sqrt(D)
    if mode == "bf16":
        att = _bf(att)
    mask = torch.tril(torch.ones(T, T, dtype=torch.bool))
    att = att.masked_fill(~mask, -1e4)
    att = torch.softmax(att, dim=-1)
    if drop is not None:
        att = att * drop                                                     # attn_drop (model.py:146)
    if mode == "bf16":
        return _bf(_bf(att) @ v)
    return att @ v


def cross_entropy(logits, labels):
    """F.cross_entropy(mean, ignore_index=-100) (model.py:357-359); fp32 under autocast."""
    lg = logits.reshape(-1, logits.shape[-1]).float()
    y = labels.reshape(-1)
    return F.cross_entropy(lg, y, ignore_index=-100)


def attn_forward(x, p, cfg, mode="fp32", drop=None, layer=0):
    """CausalMultiHeadSelfAttention.forward (model.py:110-159) on the ln1 output x [B,T,C]:
    resid_drop(proj(attention(qkv(x)))). ``p`` holds the block's parameters (BLOCK_KEYS names)."""
    dm = (lambda site: drop[(site, layer)]) if drop is not None else (lambda site: None)
    B, T, C = x.shape
    H = cfg.n_head
    D = C // H
    qkv = linear(x, p["attn.qkv.weight"], p["attn.qkv.bias"], mode)          # [B,T,3C]
    qkv = qkv.view(B, T, 3, H, D).transpose(1, 3)                           # model.py:124
    q, k, v = qkv.unbind(dim=2)                                             # [B,H,T,D]
    y = causal_attention(q, k, v, mode, dm("attn"))
    y = y.transpose(1, 2).contiguous().view(B, T, C)                        # model.py:155
    y = linear(y, p["attn.proj.weight"], p["attn.proj.bias"], mode)
    m = dm("proj")
    return y if m is None else y * m                                        # resid_drop (model.py:158)


def mlp_forward(x, p, cfg, mode="fp32", drop=None, layer=0):
    """MLP.forward (model.py:186-192) on the ln2 output x: drop2(fc2(drop1(gelu(fc1(x)))))."""
    dm = (lambda site: drop[(site, layer)]) if drop is not None else (lambda site: None)

    def dr(t, site):
        m = dm(site)
        return t if m is None else t * m
    u = linear(x, p["mlp.fc1.weight"], p["mlp.fc1.bias"], mode)
    a = dr(gelu_tanh(u, mode), "fc1")                                       # drop1 (model.py:188)
    return dr(linear(a, p["mlp.fc2.weight"], p["mlp.fc2.bias"], mode), "fc2")  # drop2 (model.py:191)


def block_forward(x, p, cfg, mode="fp32", drop=None, layer=0):
    """GPT2Block.forward (model.py:213-219): x + attn(ln1(x)); x + mlp(ln2(x)). ``drop``: optional
    table of dropout multipliers keep/(1-p) per site (``dropout_ref.step_masks``); None = dropout 0."""
    h = layer_norm(x, p["ln1.weight"], p["ln1.bias"], cfg.layer_norm_eps)
    x = x + attn_forward(h, p, cfg, mode, drop, layer)
    h = layer_norm(x, p["ln2.weight"], p["ln2.bias"], cfg.layer_norm_eps)
    return x + mlp_forward(h, p, cfg, mode, drop, layer)


def backbone_forward(params, cfg, idx, mode="fp32", drop=None):
    """GPT2Backbone.forward (model.py:275-313): embeddings -> blocks -> ln_f (fp32 output)."""
    B, T = idx.shape
    if T > cfg.n_positions:
        raise ValueError(f"Sequence length {T} > model max {cfg.n_positions}")
    x = embed(params["transformer.wte.weight"], params["transformer.wpe.weight"], idx)
    if drop is not None:
        x = x * drop["embd"]                                                 # self.drop (model.py:304)
    for i in range(cfg.n_layer):
        pre = f"transformer.h.{i}."
        p = {k: params[pre + k] for k in BLOCK_KEYS}
        x = block_forward(x, p, cfg, mode, drop, i)
    return layer_norm(x, params["transformer.ln_f.weight"], params["transformer.ln_f.bias"], cfg.layer_norm_eps)


def forward(params, cfg, idx, labels=None, mode="fp32", drop=None):
    """GPT2.forward (model.py:335-361) -> (logits, loss). ``drop``: None = dropout 0 (parity runs), else
    the per-site multipliers of one step (``dropout_ref.step_masks``)."""
    x = backbone_forward(params, cfg, idx, mode, drop)
    logits = linear(x, params["transformer.wte.weight"], None, mode)  # tied lm_head (model.py:333)
    loss = cross_entropy(logits, labels) if labels is not None else None
    return logits, loss


def flops_per_token(cfg, T=None) -> int:
    """6 * matmul params (incl. tied lm_head) + 12 * L * T * C."""
    T = cfg.n_positions if T is None else T
    C, L, V = cfg.n_embd, cfg.n_layer, cfg.vocab_size
    p_mm = L * (3 * C * C + C * C + 4 * C * C + 4 * C * C) + V * C
    return 6 * p_mm + 12 * L * T * C
