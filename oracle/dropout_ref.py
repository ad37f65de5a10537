"""CPU restatement of the framework's dropout masks — TEST ORACLE (test infrastructure only).

The reference draws its masks from torch's Philox stream (``nn.Dropout``, model.py:99-100,183-184,241);
no GPU kernel can reproduce that stream, so the MI355X step uses its own counter-based RNG: keep(i) is
a pure function of (site seed, element index) that the backward regenerates (`csrc/common.h`
``drop_hash`` / ``drop_keep16``). This module restates that function in numpy so that the oracle forward
(``model_ref.forward(..., drop=...)``) can be run with exactly the masks the HIP step drew, which makes
the dropout-on step checkable element for element against autograd of the reference's math:
``nn.Dropout`` in train mode is ``x * keep / (1 - p)`` (torch/nn/functional.py dropout).

Element indexing per site (the kernels' own):
  * embedding / attn proj / fc1 / fc2 outputs, logical [M, N] row-major: element e = row * N + col,
    hash(seed, e >> 1), 16-bit half e & 1 (`csrc/norm_embed.hip`, `csrc/gemm_common.h`);
  * attention probabilities [B*H, T(q), T(key)]: hash(seed, (bh * T + (q & ~16)) * T + key), half
    (q >> 4) & 1 (`csrc/attention.hip`, `csrc/fp32.hip`).
keep = int16(uniform16) >= round(p * 2^16) - 2^15, i.e. (uniform16 ^ 0x8000) >= round(p * 2^16): P(keep) = 1 - p
(a signed threshold, so the attention forward decides a pair with one packed int16 subtract).
The 64-bit site seed's low word is the additive offset of the first round, its high word (made odd; 0 means
murmur3's 0x85EBCA6B) the multiplier of the second (`csrc/common.h` seed32 / seed_kx).
"""
from __future__ import annotations

import numpy as np
import torch

M32 = np.uint64(0xFFFFFFFF)


def seed32(seed: int) -> np.uint32:
    return np.uint32(seed & 0xFFFFFFFF)


def seed_kx(seed: int) -> np.uint64:
    """The second-round multiplier of a site (csrc/common.h seed_kx)."""
    hi = (seed >> 32) & 0xFFFFFFFF
    return np.uint64(hi | 1 if hi else 0x85EBCA6B)


def threshold(p: float) -> int:
    """drop_threshold (csrc/common.h)."""
    if p <= 0.0:
        return 0
    return int(min(p * 65536.0 + 0.5, 65536.0))


def drop_hash(seed: int, x: np.ndarray) -> np.ndarray:
    """Two multiply(-xorshift) rounds over uint32 (csrc/common.h drop_hash): ((x + s32) * C1 ^ >> 16) * kx."""
    h = ((x.astype(np.uint64) + np.uint64(seed32(seed))) & M32) * np.uint64(0x9E3779B1) & M32
    h ^= h >> np.uint64(16)
    return h * seed_kx(seed) & M32


def _keep(h: np.ndarray, half: np.ndarray, thr: int) -> np.ndarray:
    """drop_keep16 (csrc/common.h): the 16-bit half as int16 >= thr - 2^15."""
    u = (h >> (np.uint64(16) * half.astype(np.uint64))) & np.uint64(0xFFFF)
    return (u ^ np.uint64(0x8000)) >= np.uint64(thr)


def site_scale(seed: int, rows: int, cols: int, p: float) -> torch.Tensor:
    """keep / (1 - p) multipliers of an [rows, cols] site (embedding, proj, fc1, fc2)."""
    e = np.arange(rows * cols, dtype=np.uint64)
    keep = _keep(drop_hash(seed, (e >> np.uint64(1)) & M32), e & np.uint64(1), threshold(p))
    return torch.from_numpy(keep.reshape(rows, cols).astype(np.float32) / np.float32(1.0 - p))


def attn_scale(seed: int, BH: int, T: int, p: float) -> torch.Tensor:
    """keep / (1 - p) multipliers of the attention probabilities, [BH, T(q), T(key)]."""
    bh = np.arange(BH, dtype=np.uint64)[:, None, None]
    q = np.arange(T, dtype=np.uint64)[None, :, None]
    k = np.arange(T, dtype=np.uint64)[None, None, :]
    x = ((bh * np.uint64(T) + (q & ~np.uint64(16))) * np.uint64(T) + k) & M32
    keep = _keep(drop_hash(seed, x), (q >> np.uint64(4)) & np.uint64(1), threshold(p))
    return torch.from_numpy(keep.astype(np.float32) / np.float32(1.0 - p))


def step_masks(seeds: dict, B: int, T: int, C: int, H: int, L: int, p_resid: float, p_attn: float) -> dict:
    """All masks of one step, keyed like the engine's seed table: "embd", ("attn"|"proj"|"fc1"|"fc2", l)."""
    M = B * T
    out = {"embd": site_scale(seeds["embd"], M, C, p_resid).view(B, T, C)}
    for l in range(L):
        out[("attn", l)] = attn_scale(seeds[("attn", l)], B * H, T, p_attn).view(B, H, T, T)
        out[("proj", l)] = site_scale(seeds[("proj", l)], M, C, p_resid).view(B, T, C)
        out[("fc1", l)] = site_scale(seeds[("fc1", l)], M, 4 * C, p_resid).view(B, T, 4 * C)
        out[("fc2", l)] = site_scale(seeds[("fc2", l)], M, C, p_resid).view(B, T, C)
    return out
