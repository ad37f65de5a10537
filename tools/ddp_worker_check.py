"""2-rank DDP rehearsal worker (see tests/test_ddp_gpu.py)."""

import os, sys, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ["REPO"])
from gpt_2_distributed_amd.parallel import init_distributed, DistributedDataParallel
from gpt_2_distributed_amd.model import GPT2, GPT2Config
init_distributed()
r, w = dist.get_rank(), dist.get_world_size()
cfg = GPT2Config(n_layer=2, n_head=4, n_embd=256, vocab_size=509, n_positions=64, resid_pdrop=0.0, attn_pdrop=0.0)
m = GPT2(cfg).to("cuda:0")
ddp = DistributedDataParallel(m, bucket_mb=0.25)
opt = ddp.configure_optimizers(learning_rate=1e-3)
g = torch.Generator().manual_seed(5)
toks = torch.randint(0, 509, (3, 4, 65), generator=g)
losses = []
for step in range(3):
    t = toks[step].cuda()
    x, y = t[:, :-1], t[:, 1:]
    xs, ys = x[2 * r:2 * r + 2], y[2 * r:2 * r + 2]   # rank r gets half of the batch
    _, loss = ddp(xs, labels=ys)
    loss.backward()
    opt.step(); opt.zero_grad()
    lt = loss.detach().clone(); dist.all_reduce(lt); losses.append(lt.item() / w)
if r == 0:
    print("RESULT", json.dumps({"losses": losses, "norm": opt.grad_norm.item(),
                                "arena_sum": float(m.arena.double().sum())}), flush=True)
dist.barrier(); dist.destroy_process_group()
