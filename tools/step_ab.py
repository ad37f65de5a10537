"""Whole-step A/B of an engine attribute in one process (bench.py's cfg-2 step: 124M, B=64, T=1024, bf16 autocast,
dropout 0.1, fwd + loss + bwd + AdamW), rounds alternating between the settings, HIP-synchronised wall time.

    python tools/step_ab.py wgrad_bf16_slabs False True [--rounds 4 --steps 10]
"""
import argparse
import ast
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("attr")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    from gpt_2_distributed_amd.model import GPT2, GPT2Config, MODEL_SIZES
    dev = torch.device("cuda", 0)
    cfg = GPT2Config(**MODEL_SIZES["124M"], n_positions=1024, resid_pdrop=0.1, attn_pdrop=0.1)
    model = GPT2(cfg).to(dev)
    model.train()
    opt = model.configure_optimizers(learning_rate=1e-4)
    eng = model.engine()
    g = torch.Generator().manual_seed(1234)
    t = torch.randint(0, cfg.vocab_size, (64, 1025), generator=g)
    x, y = t[:, :-1].contiguous().to(dev), t[:, 1:].contiguous().to(dev)
    vals = [ast.literal_eval(v) for v in args.values]  # literals from the command line (True, 4, ...)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = model(x, labels=y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    for v in vals:  # warm-up of every setting
        setattr(eng, args.attr, v)
        for _ in range(3):
            step()
    torch.cuda.synchronize()
    res = {i: [] for i in range(len(vals))}
    for _ in range(args.rounds):
        for i, v in enumerate(vals):
            setattr(eng, args.attr, v)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                loss = step()
            torch.cuda.synchronize()
            res[i].append((time.perf_counter() - t0) / args.steps * 1e3)
    for i, v in enumerate(vals):
        ms = sorted(res[i])
        print(f"{args.attr}={v!r:8}: ms/step {' '.join(f'{m:.2f}' for m in res[i])}  median {ms[len(ms) // 2]:.2f}  "
              f"({64 * 1024 / ms[len(ms) // 2] * 1e3 / 1e6:.4f} M tok/s)  loss {float(loss.detach()):.4f}", flush=True)


if __name__ == "__main__":
    main()
