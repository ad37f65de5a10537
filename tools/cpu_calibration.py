#!/usr/bin/env python
"""BASELINE.md §4 calibration: the oracle's CPU step (oracle/train_ref.py, what bench.py's cpu_baseline times on the
GPU box) against the REFERENCE itself (/root/reference/model.py under the reference loop,
train_gpt2_distributed.py:396-425: forward, loss, backward, clip_grad_norm_(inf), torch fused AdamW) on the same
cores, same shape (GPT-2 124M, B=4, T=1024, fp32, dropout 0), same token batches. Run in the build container only
(the reference is not on the GPU box); writes profiles/cpu_calibration_r3.json.
    python tools/cpu_calibration.py [threads] [steps]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(threads=8, steps=3, B=4, T=1024):
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    data = [(torch.randint(0, 50257, (B, T), generator=g), torch.randint(0, 50257, (B, T), generator=g))
            for _ in range(steps + 1)]
    out = {"threads": threads, "batch": B, "seq_len": T, "timed_steps": steps, "warmup_steps": 1}
    # the oracle (bench.py cpu_baseline's measured function)
    from oracle import model_ref, train_ref
    cfg = model_ref.Cfg(resid_pdrop=0.0, attn_pdrop=0.0, n_positions=T)
    params = model_ref.init_params(cfg)
    train_ref.run(cfg, data[:1], 1, params=params)
    t0 = time.perf_counter()
    lo, _ = train_ref.run(cfg, data[1:], steps, params=params)
    out["oracle_tok_s"] = steps * B * T / (time.perf_counter() - t0)
    del params
    # the reference model under the reference loop
    sys.path.insert(0, "/root/reference")
    import model as ref_model
    torch.manual_seed(42)
    m = ref_model.GPT2(ref_model.GPT2Config(n_positions=T, resid_pdrop=0.0, attn_pdrop=0.0))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.1, betas=(0.9, 0.95), fused=True)

    def step(x, y):
        _, loss = m(x, labels=y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), float("inf"))
        opt.step()
        opt.zero_grad()
        return loss.item()
    step(*data[0])
    t0 = time.perf_counter()
    lr = [step(*d) for d in data[1:]]
    out["reference_tok_s"] = steps * B * T / (time.perf_counter() - t0)
    out["ratio_oracle_over_reference"] = out["oracle_tok_s"] / out["reference_tok_s"]
    out["losses_oracle"], out["losses_reference"] = lo, lr
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "cpu_calibration_r3.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
