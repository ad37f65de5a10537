#!/usr/bin/env python
"""Loader throughput at BASELINE cfg 2's shape (B = 64, T = 1024): the reference-compatible
``create_dataloader(TokenShardDataset(...), 64, num_workers)`` (torch DataLoader, worker processes,
pinned memory; the reference's own path, dataloader.py:104-160,208-217) against the in-process
vectorised ``iter_batches`` (one fancy-indexed gather per batch, same order). One MI355X consumes
~14 batches/s at the measured 912k tok/s (18/s at the 40 % MFU target): SURVEY A20.

    python tools/loader_bench.py [--tokens 25000000] [--shards 4] [--batches 60]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=25_000_000, help="tokens per shard")
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq_len", type=int, default=1024)
    args = ap.parse_args()
    from gpt_2_distributed_amd import dataloader as D
    B, T = args.batch, args.seq_len
    out = {"batch": B, "seq_len": T, "shards": args.shards, "tokens_per_shard": args.tokens,
           "host_cpus": os.cpu_count()}
    with tempfile.TemporaryDirectory() as d:
        rng = np.random.default_rng(0)
        for i in range(args.shards):
            rng.integers(0, 50257, size=args.tokens, dtype=np.uint16).astype("<u2").tofile(
                os.path.join(d, f"train_{i:03d}.bin"))
        paths = D.get_shard_paths(d, "train")

        def rate(it, n, warm=5):
            for _ in range(warm):
                next(it)
            t0 = time.perf_counter()
            for _ in range(n):
                x, y = next(it)
                assert x.shape == (B, T)
            dt = time.perf_counter() - t0
            return round(n / dt, 2)

        for nw in (2, 4, 8):
            ds = D.TokenShardDataset(paths, seq_len=T, shuffle=True)
            dl = D.create_dataloader(ds, batch_size=B, num_workers=nw)
            out[f"dataloader_w{nw}_batches_per_s"] = rate(iter(dl), args.batches)
            del dl
        out["iter_batches_batches_per_s"] = rate(D.iter_batches(paths, T, B, num_workers=2), args.batches)
    out["needed_batches_per_s_at_912k_tok_s"] = round(912_000 / (B * T), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
