"""Is the step host-bound? bench.py's default step (124M, B=64, T=1024, bf16 autocast, dropout 0.1), timed on the host
without synchronising (how long Python takes to enqueue a step) against the GPU's own time per step.

    python tools/host_probe.py [steps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpt_2_distributed_amd.model import GPT2, GPT2Config, MODEL_SIZES  # noqa: E402


def main(steps=10):
    dev = torch.device("cuda", 0)
    cfg = GPT2Config(**MODEL_SIZES["124M"], n_positions=1024, resid_pdrop=0.1, attn_pdrop=0.1)
    model = GPT2(cfg).to(dev)
    model.train()
    opt = model.configure_optimizers(learning_rate=1e-4)
    g = torch.Generator().manual_seed(0)
    t = torch.randint(0, cfg.vocab_size, (64, 1025), generator=g)
    x, y = t[:, :-1].contiguous().to(dev), t[:, 1:].contiguous().to(dev)
    ph = {"fwd": 0.0, "bwd": 0.0, "opt": 0.0}

    def step(rec):
        t0 = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = model(x, labels=y)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        opt.step()
        opt.zero_grad()
        t3 = time.perf_counter()
        if rec:
            ph["fwd"] += t1 - t0
            ph["bwd"] += t2 - t1
            ph["opt"] += t3 - t2

    for _ in range(3):
        step(False)
    torch.cuda.synchronize()
    # 1) host enqueue time with the GPU queue starting empty
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tt = time.perf_counter() - t0
    print(f"host enqueue {th / steps * 1e3:.2f} ms/step (fwd {ph['fwd'] / steps * 1e3:.2f}, bwd "
          f"{ph['bwd'] / steps * 1e3:.2f}, opt {ph['opt'] / steps * 1e3:.2f}); wall incl. GPU {tt / steps * 1e3:.2f} ms/step",
          flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
