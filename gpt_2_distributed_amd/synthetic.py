"""Synthetic token shards in the reference's on-disk format.

The reference's shards are raw little-endian uint16 token files with no header
(data/fineweb_10BT_hugging_face.ipynb ``write_token_shard_uint16_to_bin``; read back by
dataloader.py:85-102). There is no network here, so every run uses synthetic shards written by
:func:`write_shards` (SURVEY.md §6/§8d recipe: ``np.random.default_rng(1234)``; Zipf(1.2) clipped
to the vocabulary, or uniform).
"""
from __future__ import annotations

import os
from typing import List

import numpy as np

VOCAB = 50257


def make_tokens(rng: np.random.Generator, n: int, dist: str = "zipf", vocab: int = VOCAB) -> np.ndarray:
    if dist == "zipf":
        return (np.minimum(rng.zipf(1.2, size=n), vocab) - 1).astype("<u2")
    if dist == "uniform":
        return rng.integers(0, vocab, size=n).astype("<u2")
    raise ValueError(dist)


def write_shards(out_dir, n_shards: int, tokens_per_shard: int, dist: str = "zipf", seed: int = 1234,
                 split: str = "train", vocab: int = VOCAB) -> List[str]:
    """Write ``n_shards`` files ``{split}_{i:06d}.bin`` of ``tokens_per_shard`` uint16 tokens each."""
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    paths = []
    for i in range(n_shards):
        p = os.path.join(str(out_dir), f"{split}_{i:06d}.bin")
        make_tokens(rng, tokens_per_shard, dist, vocab).tofile(p)
        paths.append(p)
    return paths
