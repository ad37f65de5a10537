"""Generate golden fixtures by running the REFERENCE (`/root/reference/model.py`, `dataloader.py`).

Run in the build container only (the reference is not present on the GPU box):
    python tests/golden/make_golden.py [--skip-traj]

Outputs (all small data files, no reference source):
  tiny_fwd_bwd.npz  tiny config (L=2, C=128, H=2, V=509, T=64, B=2, dropout 0): idx, labels,
                    logits, loss and every parameter gradient, fp32, from model.GPT2 + autograd.
  tiny_traj.json    tiny config 20-step fp32 loss / grad-norm trajectory (torch AdamW fused=True
                    as train_gpt2_distributed.py:356-362, clip_grad_norm_(inf) :419).
  init_124m.json    124M seed-42 init checksums per tensor (sum, sum of squares, first values).
  traj_124m.json    124M fp32 CPU trajectory: B=4, T=1024, grad_accum=1, 20 steps, Zipf(1.2)
                    synthetic shards (2 x 200k tokens, rng 1234), 2 loader workers.
  loader.json       sha256 of every batch the reference DataLoader yields over a grid of
                    (world, rank, workers, epoch, T, B) on synthetic ragged shards.
  tiny_accum.json   tiny config, grad_accum=4 (loss/grad_accum, backward per micro-batch, one clip+step per 4,
                    train_gpt2_distributed.py:404-425), 6 optimizer steps: losses, grad norms, final-param checks.
  ddp_golden.json   the DDP identity: the reference run single-process on the concatenation of two
                    ranks' micro-batches (L=2, C=256, H=4, V=509, T=64; 2 ranks x B=2, grad_accum=2, 3 steps,
                    lr 1e-3): per-step loss and grad norm, and final-parameter checks, for the 2-rank tests.
  cfg5_golden.json  the same identity at BASELINE cfg 5's widths (GPT-2 1.5B: C=1600, H=25, V=50257) on 2 layers,
                    T=256, 2 ranks x B=1, grad_accum=2, 2 steps, lr 1e-4, Zipf tokens stored in the file: the FSDP +
                    gradient-accumulation test of the 1.5B configuration.
  ddp124_golden.json the same identity at cfg 3's widths (GPT-2 124M: C=768, H=12, V=50257, T=1024) on 2 layers,
                    2 ranks x B=2, grad_accum=1, 3 steps, lr 1e-3, Zipf tokens stored in the file: the DDP test (the
                    wrapper runs it with its default 25 MiB buckets, torch DDP's bucket_cap_mb).
  cfg4_golden.json  the same identity at BASELINE cfg 4's widths (GPT-2 350M: C=1024, H=16, V=50257, T=1024) on 2
                    layers, 2 ranks x B=1, grad_accum=2, 3 steps, lr 1e-3, Zipf tokens stored in the file: the FSDP
                    (FULL_SHARD) test of the 350M configuration (train_gpt2_distributed.py:146-161).
  ddp8_golden.json  ddp_golden.json's configuration over 8 rows per micro-batch (8 ranks x B=1; round 6): the
                    eight-rank test on gloo ranks sharing one GPU.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

import model as ref_model          # noqa: E402  (reference)
import dataloader as ref_loader    # noqa: E402  (reference)

from gpt_2_distributed_amd import synthetic  # noqa: E402

TINY = dict(n_layer=2, n_head=2, n_embd=128, vocab_size=509, n_positions=64,
            resid_pdrop=0.0, attn_pdrop=0.0)


def tiny_fwd_bwd():
    cfg = ref_model.GPT2Config(**TINY)
    m = ref_model.GPT2(cfg)
    g = torch.Generator().manual_seed(7)
    idx = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    labels = torch.randint(0, cfg.vocab_size, (2, 64), generator=g)
    logits, loss = m(idx, labels=labels)
    loss.backward()
    out = {"idx": idx.numpy(), "labels": labels.numpy(), "logits": logits.detach().numpy(),
           "loss": np.array(loss.item(), dtype=np.float64)}
    for n, p in m.named_parameters():
        out["grad:" + n] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "tiny_fwd_bwd.npz"), **out)
    print("tiny loss", loss.item())


def _param_checks(m):
    """Final-parameter fingerprint: per-tensor sum / sum of squares, and a few tensors' leading values."""
    out = {}
    for n, p in m.named_parameters():
        d = p.detach().double()
        out[n] = {"sum": float(d.sum()), "sumsq": float((d * d).sum()),
                  "head": [float(v) for v in p.detach().reshape(-1)[:16]]}
    return out


def _ref_traj(cfg, batches, steps, grad_accum=1, lr=1e-4, model_out=None):
    torch.manual_seed(42)
    m = ref_model.GPT2(cfg)
    if model_out is not None:
        model_out.append(m)
    opt = torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=0.1, betas=(0.9, 0.95), fused=True)
    opt.zero_grad()
    losses, norms = [], []
    it = iter(batches)
    for _ in range(steps):
        for _a in range(grad_accum):
            x, y = next(it)
            _, loss = m(x, labels=y)
            loss = loss / grad_accum
            loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(m.parameters(), float("inf"))
        opt.step()
        opt.zero_grad()
        losses.append(loss.item() * grad_accum)
        norms.append(float(gn))
    return losses, norms


def tiny_traj():
    cfg = ref_model.GPT2Config(**TINY)
    rng = np.random.default_rng(99)
    toks = (np.minimum(rng.zipf(1.2, size=(20, 4, 65)), cfg.vocab_size) - 1).astype(np.int64)
    batches = [(torch.from_numpy(t[:, :-1].copy()), torch.from_numpy(t[:, 1:].copy())) for t in toks]
    losses, norms = _ref_traj(cfg, batches, 20)
    with open(os.path.join(HERE, "tiny_traj.json"), "w") as f:
        json.dump({"config": TINY, "data": "np.random.default_rng(99).zipf(1.2, (20,4,65)) clipped",
                   "batch": 4, "seq_len": 64, "lr": 1e-4, "losses": losses, "grad_norms": norms}, f, indent=1)
    print("tiny traj", losses[0], losses[-1])


def tiny_accum(steps=6, grad_accum=4):
    cfg = ref_model.GPT2Config(**TINY)
    rng = np.random.default_rng(17)
    toks = (np.minimum(rng.zipf(1.2, size=(steps * grad_accum, 2, 65)), cfg.vocab_size) - 1).astype(np.int64)
    batches = [(torch.from_numpy(t[:, :-1].copy()), torch.from_numpy(t[:, 1:].copy())) for t in toks]
    ms = []
    losses, norms = _ref_traj(cfg, batches, steps, grad_accum=grad_accum, lr=1e-3, model_out=ms)
    with open(os.path.join(HERE, "tiny_accum.json"), "w") as f:
        json.dump({"config": TINY, "data": "np.random.default_rng(17).zipf(1.2, (24,2,65)) clipped; micro-batch i "
                   "= row i", "batch": 2, "seq_len": 64, "grad_accum": grad_accum, "steps": steps, "lr": 1e-3,
                   "losses": losses, "grad_norms": norms, "params": _param_checks(ms[0])}, f, indent=0)
    print("tiny accum", losses[0], losses[-1])


DDPCFG = dict(n_layer=2, n_head=4, n_embd=256, vocab_size=509, n_positions=64, resid_pdrop=0.0, attn_pdrop=0.0)


def ddp_golden(steps=3, grad_accum=2, world=2, per_rank=2, name="ddp_golden.json"):
    """Single-process reference on the concatenated batch: rank r's micro-batch a of step s is
    toks[s, a, r*per_rank:(r+1)*per_rank] (torch.Generator().manual_seed(5), the tests' generator)."""
    cfg = ref_model.GPT2Config(**DDPCFG)
    g = torch.Generator().manual_seed(5)
    toks = torch.randint(0, 509, (steps, grad_accum, world * per_rank, 65), generator=g)
    batches = [(toks[s, a, :, :-1].contiguous(), toks[s, a, :, 1:].contiguous())
               for s in range(steps) for a in range(grad_accum)]
    ms = []
    losses, norms = _ref_traj(cfg, batches, steps, grad_accum=grad_accum, lr=1e-3, model_out=ms)
    with open(os.path.join(HERE, name), "w") as f:
        json.dump({"config": DDPCFG, "world": world, "per_rank": per_rank, "grad_accum": grad_accum,
                   "steps": steps, "lr": 1e-3,
                   "data": "torch.randint(0,509,(steps,grad_accum,world*per_rank,65), Generator seed 5); rank r "
                           "takes rows r*per_rank..", "losses": losses, "grad_norms": norms,
                   "params": _param_checks(ms[0])}, f, indent=0)
    print(name, losses, norms)


def ddp8_golden():
    """The DDP golden over 8 rows of each micro-batch (round 6): eight ranks of one row each, the rank count of the
    BASELINE node, rehearsed on gloo ranks sharing one GPU (tests/test_ddp_gpu.py EIGHT_RUNS)."""
    ddp_golden(world=8, per_rank=1, name="ddp8_golden.json")


def _wide_golden(name, cfg_kw, seq_len, steps, grad_accum, world, per_rank, lr, seed):
    """Reference run on the concatenated batch at a production width; the Zipf(1.2) tokens are stored in the file
    (tokens[s][a][row] = the T+1 tokens of row `row` of micro-batch a of step s; rank r takes rows r*per_rank..)."""
    cfg = ref_model.GPT2Config(**cfg_kw)
    rng = np.random.default_rng(seed)
    toks = (np.minimum(rng.zipf(1.2, size=(steps, grad_accum, world * per_rank, seq_len + 1)), cfg.vocab_size)
            - 1).astype(np.int64)
    batches = [(torch.from_numpy(toks[s_, a, :, :-1].copy()), torch.from_numpy(toks[s_, a, :, 1:].copy()))
               for s_ in range(steps) for a in range(grad_accum)]
    torch.set_num_threads(8)
    ms = []
    t0 = time.time()
    losses, norms = _ref_traj(cfg, batches, steps, grad_accum=grad_accum, lr=lr, model_out=ms)
    with open(os.path.join(HERE, name), "w") as f:
        json.dump({"config": cfg_kw, "world": world, "per_rank": per_rank, "grad_accum": grad_accum, "steps": steps,
                   "seq_len": seq_len, "lr": lr,
                   "data": f"np.random.default_rng({seed}).zipf(1.2) clipped to [0, V); stored in 'tokens'",
                   "tokens": toks.tolist(), "losses": losses, "grad_norms": norms,
                   "params": _param_checks(ms[0])}, f, indent=0)
    print(name, losses, norms, f"{time.time() - t0:.1f} s")


def cfg5_golden():
    _wide_golden("cfg5_golden.json", dict(n_layer=2, n_head=25, n_embd=1600, vocab_size=50257, n_positions=256,
                                          resid_pdrop=0.0, attn_pdrop=0.0),
                 seq_len=256, steps=2, grad_accum=2, world=2, per_rank=1, lr=1e-4, seed=31)


def ddp124_golden():
    _wide_golden("ddp124_golden.json", dict(n_layer=2, n_head=12, n_embd=768, vocab_size=50257, n_positions=1024,
                                            resid_pdrop=0.0, attn_pdrop=0.0),
                 seq_len=1024, steps=3, grad_accum=1, world=2, per_rank=2, lr=1e-3, seed=37)


def cfg4_golden():
    _wide_golden("cfg4_golden.json", dict(n_layer=2, n_head=16, n_embd=1024, vocab_size=50257, n_positions=1024,
                                          resid_pdrop=0.0, attn_pdrop=0.0),
                 seq_len=1024, steps=3, grad_accum=2, world=2, per_rank=1, lr=1e-3, seed=41)


def init_124m():
    cfg = ref_model.GPT2Config(n_layer=12, n_head=12, n_embd=768, n_positions=1024, vocab_size=50257)
    m = ref_model.GPT2(cfg)
    rec = {}
    for n, p in m.named_parameters():
        d = p.detach().double()
        rec[n] = {"shape": list(p.shape), "sum": float(d.sum()), "sumsq": float((d * d).sum()),
                  "head": [float(v) for v in p.detach().reshape(-1)[:4]]}
    with open(os.path.join(HERE, "init_124m.json"), "w") as f:
        json.dump({"n_params": sum(p.numel() for p in m.parameters()), "tensors": rec}, f, indent=1)


def traj_124m(steps=20):
    cfg = ref_model.GPT2Config(n_layer=12, n_head=12, n_embd=768, n_positions=1024, vocab_size=50257,
                               resid_pdrop=0.0, attn_pdrop=0.0)
    with tempfile.TemporaryDirectory() as d:
        synthetic.write_shards(d, 2, 200_000, dist="zipf", seed=1234)
        ds = ref_loader.TokenShardDataset(ref_loader.get_shard_paths(__import__("pathlib").Path(d), "train"),
                                          seq_len=1024, shuffle=True)
        dl = ref_loader.create_dataloader(ds, batch_size=4, num_workers=2)
        torch.set_num_threads(8)
        t0 = time.time()
        losses, norms = _ref_traj(cfg, dl, steps)
        dt = time.time() - t0
    with open(os.path.join(HERE, "traj_124m.json"), "w") as f:
        json.dump({"config": "124M (12L/768d/12H, V=50257, T=1024), dropout 0, fp32 CPU",
                   "data": "synthetic.write_shards(d, 2, 200000, 'zipf', seed=1234); 2 loader workers",
                   "batch": 4, "seq_len": 1024, "grad_accum": 1, "lr": 1e-4, "steps": steps,
                   "losses": losses, "grad_norms": norms,
                   "cpu_tok_per_s": steps * 4 * 1024 / dt, "cpu_threads": 8}, f, indent=1)
    print("124m traj", losses[0], losses[-1], f"{steps*4096/dt:.1f} tok/s")


def _write_ragged_shards(d):
    rng = np.random.default_rng(5)
    lens = [1, 10, 17, 33, 50, 64, 65, 81, 97, 130, 160]
    for i, n in enumerate(lens):
        rng.integers(0, 50257, size=n).astype("<u2").tofile(os.path.join(d, f"train_{i:03d}.bin"))
    rng.integers(0, 50257, size=100).astype("<u2").tofile(os.path.join(d, "val_000.bin"))


def loader_grid():
    import pathlib
    cases = []
    with tempfile.TemporaryDirectory() as d:
        _write_ragged_shards(d)
        paths = ref_loader.get_shard_paths(pathlib.Path(d), "train")
        names = [p.name for p in paths]
        for world in (1, 2, 4, 8):
            for rank in sorted({0, world - 1}):
                for nw in (1, 2, 3):
                    for epoch in (0, 1):
                        for (T, B) in ((16, 3), (8, 2)):
                            ds = ref_loader.TokenShardDataset(paths, seq_len=T, shuffle=True)
                            ds.rank, ds.world = rank, world
                            ds.set_epoch(epoch)
                            dl = ref_loader.create_dataloader(ds, batch_size=B, num_workers=nw)
                            hs = []
                            for x, y in dl:
                                assert x.dtype == torch.int64 and x.shape == (B, T)
                                hs.append(hashlib.sha256(x.numpy().tobytes() + y.numpy().tobytes()).hexdigest()[:16])
                            del dl
                            cases.append({"world": world, "rank": rank, "workers": nw, "epoch": epoch,
                                          "seq_len": T, "batch": B, "hashes": hs})
    with open(os.path.join(HERE, "loader.json"), "w") as f:
        json.dump({"shards": "tests/golden/make_golden.py:_write_ragged_shards", "names": names,
                   "cases": cases}, f, indent=0)
    print("loader cases", len(cases))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-traj", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    jobs = {"tiny": tiny_fwd_bwd, "tinytraj": tiny_traj, "init": init_124m, "loader": loader_grid,
            "traj": traj_124m, "accum": tiny_accum, "ddp": ddp_golden, "cfg5": cfg5_golden,
            "ddp124": ddp124_golden, "cfg4": cfg4_golden, "ddp8": ddp8_golden}
    for k, fn in jobs.items():
        if a.only and k not in a.only.split(","):
            continue
        if k == "traj" and a.skip_traj:
            continue
        fn()
