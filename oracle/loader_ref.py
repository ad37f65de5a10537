"""Pure-python restatement of the reference loader's order (`/root/reference/dataloader.py`) — TEST ORACLE.

Test infrastructure only. Restates, with no torch DataLoader and no worker processes, the exact
sequence of (x, y) batches that ``create_dataloader(TokenShardDataset(...))`` yields on one rank:

* ``get_shard_paths`` (dataloader.py:31-51): sorted names ending in ``.{file_type}`` containing ``split``.
* per worker ``wid`` of ``nw`` on rank ``r`` of ``world`` (dataloader.py:136-160): the shard list is
  shuffled with ``random.Random(epoch)`` and strided ``[r*nw+wid :: world*nw]``.
* per shard (dataloader.py:104-133): ``max_offset = n - (T+1)``, skip if ``<= 0``; offsets
  ``range(0, max_offset, T)`` shuffled by ``random.Random`` seeded ``(epoch*17)^(r*971)^(wid*31)``;
  sample = ``mm[o:o+T+1]`` -> (x = s[:-1], y = s[1:]) as int64.
* batching (dataloader.py:208-217 + torch DataLoader semantics): each worker groups its own samples
  into consecutive batches of B (remainder dropped, ``drop_last=True``); the main process takes
  batches round-robin over workers, skipping exhausted ones. With ``num_workers=0`` there is one
  in-process stream with ``worker_id=0, num_workers=1``.
* persistent workers freeze the epoch at the value the dataset had when the workers started
  (SURVEY.md §5 "Epoch freeze"); pass that value as ``epoch``.
"""
from __future__ import annotations

import os
import random
from typing import Iterator, List, Tuple

import numpy as np


def get_shard_paths(data_dir, split="train", file_type="bin") -> List[str]:
    return sorted(os.path.join(str(data_dir), f) for f in os.listdir(data_dir)
                  if f.endswith(f".{file_type}") and split in f)


def worker_samples(paths, seq_len, rank, world, wid, nw, epoch, shuffle=True) -> Iterator[np.ndarray]:
    shards = list(paths)
    if shuffle:
        random.Random(epoch).shuffle(shards)
    mine = shards[rank * nw + wid:: world * nw]
    for path in mine:
        n = os.path.getsize(path) // 2
        mm = np.memmap(path, dtype="<u2", mode="r", shape=(n,))
        max_offset = n - (seq_len + 1)
        if max_offset <= 0:
            continue
        g = random.Random()
        g.seed((epoch * 17) ^ (rank * 971) ^ (wid * 31))
        offs = list(range(0, max_offset, seq_len))
        if shuffle:
            g.shuffle(offs)
        for o in offs:
            yield np.array(mm[o:o + seq_len + 1], dtype=np.int64)


def batches(paths, seq_len, batch_size, rank=0, world=1, num_workers=2, epoch=0,
            shuffle=True) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    nw = max(num_workers, 1)
    streams = [worker_samples(paths, seq_len, rank, world, w, nw, epoch, shuffle) for w in range(nw)]

    def worker_batches(s):
        buf = []
        for smp in s:
            buf.append(smp)
            if len(buf) == batch_size:
                arr = np.stack(buf)
                yield arr[:, :-1].copy(), arr[:, 1:].copy()
                buf = []

    gens = [worker_batches(s) for s in streams]
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
