"""Product loader (gpt_2_distributed_amd.dataloader) bit-exact against the reference's batch stream
(tests/golden/loader.json, captured from /root/reference/dataloader.py) — CPU only."""
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest
import torch

from gpt_2_distributed_amd import dataloader as dl_mod
from tests.conftest import GOLDEN


def _ragged_shards(d):
    rng = np.random.default_rng(5)
    lens = [1, 10, 17, 33, 50, 64, 65, 81, 97, 130, 160]
    for i, n in enumerate(lens):
        rng.integers(0, 50257, size=n).astype("<u2").tofile(os.path.join(d, f"train_{i:03d}.bin"))
    rng.integers(0, 50257, size=100).astype("<u2").tofile(os.path.join(d, "val_000.bin"))


def _h(x, y):
    return hashlib.sha256(x.numpy().tobytes() + y.numpy().tobytes()).hexdigest()[:16]


@pytest.fixture(scope="module")
def shards():
    with tempfile.TemporaryDirectory() as d:
        _ragged_shards(d)
        yield d


def test_shard_paths(shards):
    ref = json.load(open(os.path.join(GOLDEN, "loader.json")))
    assert [p.name for p in dl_mod.get_shard_paths(shards, "train")] == ref["names"]
    assert [p.name for p in dl_mod.get_shard_paths(shards, "val")] == ["val_000.bin"]


def test_iter_batches_bit_exact_over_grid(shards):
    ref = json.load(open(os.path.join(GOLDEN, "loader.json")))
    paths = dl_mod.get_shard_paths(shards, "train")
    for c in ref["cases"]:
        hs = [_h(x, y) for x, y in dl_mod.iter_batches(paths, c["seq_len"], c["batch"], c["workers"], c["epoch"],
                                                       c["rank"], c["world"])]
        assert hs == c["hashes"], c


@pytest.mark.parametrize("case_idx", [0, 9, 30, 61, 83])
def test_dataloader_bit_exact(shards, case_idx):
    """The torch-DataLoader path (worker processes) yields the same stream."""
    ref = json.load(open(os.path.join(GOLDEN, "loader.json")))
    c = ref["cases"][case_idx]
    paths = dl_mod.get_shard_paths(shards, "train")
    ds = dl_mod.TokenShardDataset(paths, seq_len=c["seq_len"], shuffle=True)
    ds.rank, ds.world = c["rank"], c["world"]
    ds.set_epoch(c["epoch"])
    dl = dl_mod.create_dataloader(ds, batch_size=c["batch"], num_workers=c["workers"])
    hs = []
    for x, y in dl:
        assert x.dtype == torch.int64 and x.shape == (c["batch"], c["seq_len"])
        hs.append(_h(x, y))
    assert hs == c["hashes"]


def test_empty_shard_raises_like_reference():
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "train_0.bin"), "wb").close()
        paths = dl_mod.get_shard_paths(d, "train")
        with pytest.raises(ValueError):
            list(dl_mod.iter_batches(paths, 8, 2, 1))
