"""Token-shard loader with the reference's exact batch order (`/root/reference/dataloader.py`).

Surface (dataloader.py:15-219): ``DEFAULT_*`` constants, ``get_shard_paths(dir, split, file_type)``,
``TokenShardDataset(shard_paths, seq_len=1024, shuffle=True)`` with ``set_epoch``, and
``create_dataloader(ds, batch_size, num_workers, pin_memory, prefetch_factor, persistent_workers,
drop_last)`` returning a torch DataLoader that yields int64 ``(x, y)`` of shape [B, T].

Order (bit-exact with the reference, tests/test_loader.py against tests/golden/loader.json):
  shards: sorted names containing ``split`` and ending in ``.{file_type}``; per (rank, worker) the
  list is shuffled with ``random.Random(epoch)`` and strided ``[rank*nw + wid :: world*nw]``;
  per shard: offsets ``range(0, n-(T+1), T)`` shuffled by ``random.Random`` seeded
  ``(epoch*17) ^ (rank*971) ^ (wid*31)``; each sample is tokens[o : o+T+1] -> (x, y) = (s[:-1], s[1:]).
Shards are raw little-endian uint16 files (memory-mapped, never loaded whole).

Beyond the reference: ``iter_batches`` is an in-process, vectorised iterator over the same order
(one fancy-indexed gather per batch instead of B per-sample copies + collate), used by the trainer
when ``--workers 0`` (the reference crashes there: prefetch_factor with 0 workers).
"""
from __future__ import annotations

import os
import pathlib
import random
from typing import Iterator, List, Tuple

import numpy as np
import torch
from torch.utils import data as torch_data
import torch.distributed as dist

DEFAULT_BATCH_SIZE = 4
DEFAULT_CONTEXT_LENGTH = 1024
DEFAULT_N_PROCS = 2
DEFAULT_PREFETCH_FACTOR = 2


def get_shard_paths(data_cache_dir: pathlib.Path, split: str = "train", file_type: str = "bin") -> List[pathlib.Path]:
    d = pathlib.Path(data_cache_dir)
    return sorted(d / f for f in os.listdir(d) if f.endswith(f".{file_type}") and split in f)


def _open(path) -> Tuple[np.ndarray, int]:
    n = os.path.getsize(path) // 2
    # np.memmap raises ValueError on an empty file, as the reference does
    return np.memmap(path, dtype="<u2", mode="r", shape=(n,)), n


def _stream_plan(paths, seq_len, rank, world, wid, nw, epoch, shuffle):
    """(path, offsets) for one (rank, worker) stream in reference order."""
    shards = list(paths)
    if shuffle:
        random.Random(epoch).shuffle(shards)
    for path in shards[rank * nw + wid:: world * nw]:
        mm, n = _open(path)
        max_offset = n - (seq_len + 1)
        if max_offset <= 0:
            continue
        offs = list(range(0, max_offset, seq_len))
        if shuffle:
            g = random.Random()
            g.seed((epoch * 17) ^ (rank * 971) ^ (wid * 31))
            g.shuffle(offs)
        yield mm, offs


class TokenShardDataset(torch_data.IterableDataset):
    """Streams (T+1)-token windows from uint16 shards (dataloader.py:54-171)."""

    def __init__(self, shard_paths: List[pathlib.Path], seq_len: int = 1024, shuffle: bool = True):
        super().__init__()
        self.shard_paths = list(shard_paths)
        self.seq_len = seq_len
        self.shuffle = shuffle
        self.rank, self.world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        info = torch_data.get_worker_info()
        self.worker_id, self.num_workers = (info.id, info.num_workers) if info is not None else (0, 1)
        self.epoch = getattr(self, "_epoch", 0)
        T = self.seq_len
        for mm, offs in _stream_plan(self.shard_paths, T, self.rank, self.world, self.worker_id,
                                     self.num_workers, self.epoch, self.shuffle):
            for o in offs:
                s = np.array(mm[o:o + T + 1], dtype=np.int64)
                yield torch.from_numpy(s[:-1]), torch.from_numpy(s[1:])

    def set_epoch(self, epoch: int):
        self._epoch = epoch


def _collate(batch):
    return tuple(torch.stack(x) for x in zip(*batch))


def create_dataloader(ds: TokenShardDataset, batch_size: int = DEFAULT_BATCH_SIZE, num_workers: int = DEFAULT_N_PROCS,
                      pin_memory: bool = True, prefetch_factor: int = DEFAULT_PREFETCH_FACTOR,
                      persistent_workers: bool = True, drop_last: bool = True):
    return torch_data.DataLoader(ds, batch_size=batch_size, num_workers=num_workers,
                                 pin_memory=pin_memory and torch.cuda.is_available(),
                                 prefetch_factor=prefetch_factor, persistent_workers=persistent_workers,
                                 drop_last=drop_last, collate_fn=_collate)


def iter_batches(shard_paths, seq_len: int, batch_size: int, num_workers: int = 2, epoch: int = 0, rank: int = None,
                 world: int = None, shuffle: bool = True) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
    """The exact batch sequence ``create_dataloader(TokenShardDataset(...), batch_size, num_workers)``
    yields (workers' batches interleaved round-robin, exhausted workers skipped, per-worker drop_last),
    produced in-process with one vectorised gather per batch."""
    if rank is None or world is None:
        rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    nw = max(1, num_workers)
    T = seq_len

    def worker(wid):
        pend_mm, pend_off = [], []
        for mm, offs in _stream_plan(shard_paths, T, rank, world, wid, nw, epoch, shuffle):
            for o in offs:
                pend_mm.append(mm)
                pend_off.append(o)
                if len(pend_off) == batch_size:
                    out = np.empty((batch_size, T + 1), dtype=np.int64)
                    ar = np.arange(T + 1)
                    # group rows by shard: one fancy-indexed gather per shard present in the batch
                    for key in {id(m) for m in pend_mm}:
                        rows = [i for i, m in enumerate(pend_mm) if id(m) == key]
                        m = pend_mm[rows[0]]
                        out[rows] = m[np.asarray([pend_off[i] for i in rows])[:, None] + ar[None, :]]
                    t = torch.from_numpy(out)
                    yield t[:, :-1].contiguous(), t[:, 1:].contiguous()
                    pend_mm, pend_off = [], []

    gens = [worker(w) for w in range(nw)]
    alive = list(range(nw))
    while alive:
        nxt = []
        for w in alive:
            try:
                yield next(gens[w])
                nxt.append(w)
            except StopIteration:
                pass
        alive = nxt
