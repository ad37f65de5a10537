"""Multi-rank data parallel on the GPU box: 2 ranks on the one visible MI355X (gloo carries the grad
buckets, GPT2MI_SINGLE_DEVICE=1), exercising the engine's in-backward bucket launches, the DDP
optimizer proxy and the identity that the DDP step equals one process on the concatenated batch."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from gpt_2_distributed_amd.parallel import init_distributed, DistributedDataParallel, ShardedDataParallel
from gpt_2_distributed_amd.model import GPT2, GPT2Config
init_distributed()
r, w = dist.get_rank(), dist.get_world_size()
cfg = GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=509, n_positions=64, resid_pdrop=0.0, attn_pdrop=0.0)
m = GPT2(cfg).to("cuda:0")
Wrap = ShardedDataParallel if os.environ["MODE"] == "fsdp" else DistributedDataParallel
ddp = Wrap(m, bucket_mb=0.25)
opt = ddp.configure_optimizers(learning_rate=1e-3)
g = torch.Generator().manual_seed(5)
toks = torch.randint(0, 509, (3, 4, 65), generator=g)
losses = []
for step in range(3):
    t = toks[step].cuda()
    x, y = t[:, :-1], t[:, 1:]
    xs, ys = x[2 * r:2 * r + 2], y[2 * r:2 * r + 2]   # rank r gets half of the batch
    with torch.autocast("cuda", dtype=torch.bfloat16):
        _, loss = ddp(xs, labels=ys)
    loss.backward()
    opt.step(); opt.zero_grad()
    lt = loss.detach().clone(); dist.all_reduce(lt); losses.append(lt.item() / w)
if r == 0:
    print("RESULT", json.dumps({"losses": losses, "norm": opt.grad_norm.item(),
                                "arena_sum": float(m.arena.double().sum())}), flush=True)
dist.barrier(); dist.destroy_process_group()
"""


@pytest.mark.parametrize("mode", ["ddp", "fsdp"])
def test_ddp_two_ranks_matches_single_process(tmp_path, mode):
    """ddp: bucketed all-reduce in the backward; fsdp: reduce-scatter of the grad arena, AdamW on the
    rank's 1/N slice, all-gather of the updated parameters (parallel.ShardedDataParallel)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, REPO=REPO, MODE=mode, GPT2MI_SINGLE_DEVICE="1", GPT2MI_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29555", str(script)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("RESULT")][0][7:])
    # single process on the full batch of 4
    from gpt_2_distributed_amd.model import GPT2, GPT2Config
    cfg = GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=509, n_positions=64, resid_pdrop=0.0,
                     attn_pdrop=0.0)
    m = GPT2(cfg).to("cuda:0")
    opt = m.configure_optimizers(learning_rate=1e-3)
    g = torch.Generator().manual_seed(5)
    toks = torch.randint(0, 509, (3, 4, 65), generator=g)
    losses = []
    for step in range(3):
        t = toks[step].cuda()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = m(t[:, :-1], labels=t[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    for a, b in zip(res["losses"], losses):
        assert abs(a - b) < 2e-3 * b, (res["losses"], losses)
    assert abs(res["norm"] - opt.grad_norm.item()) < 2e-2 * opt.grad_norm.item()
    assert abs(res["arena_sum"] - float(m.arena.double().sum())) < 1e-3 * abs(float(m.arena.double().sum())) + 1e-3
