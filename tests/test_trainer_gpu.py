"""The trainer surface of SURVEY §8(f) items 1-2 on the GPU: the reference CLI run end to end on synthetic
shards, its checkpoint format (step_{:07d}/model.pt with the reference state_dict keys + optim.pt,
train_gpt2_distributed.py:67-101), and resume (the reference's load_checkpoint is a stub, :104-111):
a step taken after reloading a checkpoint matches the same step of the uninterrupted run (to the last bits: the
tied wte gradient sums repeated tokens with float atomics in the embedding backward, as torch's CUDA embedding
backward does, so its summation order is not fixed)."""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests.conftest import REPO

pytestmark = pytest.mark.gpu
dev = "cuda"

TINY = dict(n_layer=2, n_head=2, n_embd=128, vocab_size=509, n_positions=64, resid_pdrop=0.0, attn_pdrop=0.0)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _batches(n, B=2, T=64, V=509):
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n):
        t = torch.randint(0, V, (B, T + 1), generator=g)
        out.append((t[:, :-1].contiguous().to(dev), t[:, 1:].contiguous().to(dev)))
    return out


def _step(model, opt, batch):
    x, y = batch
    with torch.autocast("cuda", dtype=torch.bfloat16):
        _, loss = model(x, labels=y)
    loss.backward()
    opt.step()
    opt.zero_grad()
    return loss.item()


def test_checkpoint_resume_matches_uninterrupted_run(tmp_path):
    from gpt_2_distributed_amd.model import GPT2, GPT2Config
    from gpt_2_distributed_amd.train_gpt2_distributed import load_checkpoint, save_checkpoint

    bs = _batches(4)
    m = GPT2(GPT2Config(**TINY)).to(dev)
    opt = m.configure_optimizers(learning_rate=1e-3)
    for b in bs[:2]:
        _step(m, opt, b)
    ck = save_checkpoint(m, opt, 2, str(tmp_path))
    assert os.path.basename(ck) == "step_0000002"
    sd = torch.load(os.path.join(ck, "model.pt"), map_location="cpu", weights_only=True)
    assert list(sd) == list(m.state_dict())  # the reference's keys and order (149 at 124M, incl. lm_head.weight)
    ref_losses = [_step(m, opt, b) for b in bs[2:]]
    ref_params = {k: v.detach().clone() for k, v in m.named_parameters()}

    m2 = GPT2(GPT2Config(**TINY)).to(dev)  # same seed-42 init; overwritten by the checkpoint
    opt2 = m2.configure_optimizers(learning_rate=1e-3)
    assert load_checkpoint(m2, opt2, ck)["step"] == 2
    losses = [_step(m2, opt2, b) for b in bs[2:]]
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) <= 1e-6 * abs(b)
    for k, v in m2.named_parameters():
        assert (v - ref_params[k]).abs().max().item() <= 1e-6, k


def test_checkpoint_resume_restores_the_dropout_stream(tmp_path):
    """Dropout on (p = 0.1): the resumed run draws the same masks as the uninterrupted one (the engine's
    dropout stream position is saved in trainer.json and restored)."""
    from gpt_2_distributed_amd.model import GPT2, GPT2Config
    from gpt_2_distributed_amd.train_gpt2_distributed import load_checkpoint, save_checkpoint
    cfg = dict(TINY, resid_pdrop=0.1, attn_pdrop=0.1)
    bs = _batches(4)
    m = GPT2(GPT2Config(**cfg)).to(dev)
    opt = m.configure_optimizers(learning_rate=1e-3)
    for b in bs[:2]:
        _step(m, opt, b)
    ck = save_checkpoint(m, opt, 2, str(tmp_path), {"epoch": 0, "micro": 2})
    ref_losses = [_step(m, opt, b) for b in bs[2:]]
    m2 = GPT2(GPT2Config(**cfg)).to(dev)
    opt2 = m2.configure_optimizers(learning_rate=1e-3)
    st = load_checkpoint(m2, opt2, ck)
    assert (st["step"], st["epoch"], st["micro"]) == (2, 0, 2)
    losses = [_step(m2, opt2, b) for b in bs[2:]]
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) <= 1e-6 * abs(b)


def test_trainer_cli_resume_skips_consumed_batches(tmp_path):
    """--resume continues the data stream where the checkpoint left it: 2 steps + resume for 2 more logs
    the same losses as 4 uninterrupted steps (dropout 0.1, 2 micro-batches per step)."""
    data = tmp_path / "data"
    base = [sys.executable, "-m", "gpt_2_distributed_amd.train_gpt2_distributed", "--data_dir", str(data),
            "--synthetic", "2", "--synthetic_tokens", "60000", "--seq_len", "128", "--batch", "4",
            "--grad_accum_steps", "2", "--workers", "1", "--log_every", "1", "--training_mode", "local"]
    r = subprocess.run(base + ["--max_steps", "4", "--save_every", "2", "--save_dir", str(tmp_path / "a")], cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    full = [json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")]
    r = subprocess.run(base + ["--max_steps", "4", "--save_every", "100", "--save_dir", str(tmp_path / "b"),
                               "--resume", str(tmp_path / "a" / "step_0000002")], cwd=REPO, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    resumed = {json.loads(l)["step"]: json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")}
    assert abs(resumed[3] - full[2]) <= 1e-4 * full[2] and abs(resumed[4] - full[3]) <= 1e-4 * full[3]


def test_trainer_cli_resume_in_a_later_epoch(tmp_path):
    """Resume inside epoch 1 with DataLoader workers: the persistent workers replay the order they were
    spawned with (epoch 0), so the resumed run must spawn its workers with that epoch, not the one it
    resumes in. 11 batches per epoch, 2 micro-batches per step: step 7 ends inside epoch 1; steps 8-9 after a resume
    from it log the uninterrupted run's losses."""
    data = tmp_path / "data"
    base = [sys.executable, "-m", "gpt_2_distributed_amd.train_gpt2_distributed", "--data_dir", str(data),
            "--synthetic", "2", "--synthetic_tokens", "3000", "--seq_len", "128", "--batch", "4",
            "--grad_accum_steps", "2", "--workers", "1", "--log_every", "1", "--training_mode", "local",
            "--epochs", "3", "--max_steps", "9"]
    r = subprocess.run(base + ["--save_every", "7", "--save_dir", str(tmp_path / "a")], cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    full = {json.loads(l)["step"]: json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")}
    st = json.load(open(tmp_path / "a" / "step_0000007" / "trainer.json"))
    assert (st["epoch"], st["worker_epoch"]) == (1, 0), st
    r = subprocess.run(base + ["--save_every", "100", "--save_dir", str(tmp_path / "b"),
                               "--resume", str(tmp_path / "a" / "step_0000007")], cwd=REPO, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    resumed = {json.loads(l)["step"]: json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")}
    for s in (8, 9):
        assert abs(resumed[s] - full[s]) <= 1e-4 * full[s], (s, resumed, full)


def test_trainer_cli_end_to_end(tmp_path):
    """python -m gpt_2_distributed_amd.train_gpt2_distributed with the reference's flags on synthetic
    shards: runs, logs JSON steps with a finite loss and the reference's epoch_time / memory metrics
    (stats_tracker.py:265-364), and writes the checkpoint layout."""
    data, ckpt = tmp_path / "data", tmp_path / "ckpt"
    cmd = [sys.executable, "-m", "gpt_2_distributed_amd.train_gpt2_distributed", "--data_dir", str(data),
           "--synthetic", "2", "--synthetic_tokens", "60000", "--seq_len", "128", "--batch", "4",
           "--grad_accum_steps", "2", "--max_steps", "3", "--save_every", "2", "--save_dir", str(ckpt),
           "--workers", "1", "--log_every", "1", "--training_mode", "local"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    steps = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [s["step"] for s in steps] == [1, 2, 3]
    assert all(0.0 < s["loss"] < 20.0 and s["tok_per_s_node"] > 0 for s in steps)
    for s in steps:
        assert 0 < s["gpu_alloc_gb"] <= s["gpu_max_alloc_gb"] and s["gpu_alloc_gb"] <= s["gpu_reserved_gb"]
        assert 0 < s["gpu_utilization_pct"] < 100 and s["cpu_mb"] > 0 and s["epoch_time"] > 0
    for st in ("step_0000002", "step_0000003"):
        assert (ckpt / st / "model.pt").exists() and (ckpt / st / "optim.pt").exists()


@pytest.mark.parametrize("mode", ["ddp", "fsdp", "fsdp_resident"])
def test_trainer_cli_wrapped_one_rank_resume(tmp_path, mode):
    """The trainer under torchrun in the reference's ddp / fsdp modes (one rank, RCCL collectives forced on); fsdp is
    FULL_SHARD's memory behaviour by default, as the reference's (every micro-step reduce-scatters, no no_sync), and
    --fsdp_resident keeps the gathered units; 2 micro-batches per step: 2 steps + a resume for 2 more log the losses
    of 4 uninterrupted steps (the sharded checkpoint: model.pt gathered on rank 0, optim_rank{r}.pt per rank)."""
    data = tmp_path / "data"
    mode_args = ["--training_mode", "fsdp", "--fsdp_resident"] if mode == "fsdp_resident" else ["--training_mode", mode]
    port = {"ddp": 29571, "fsdp": 29572, "fsdp_resident": 29573}[mode]
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
            f"--master-port={port}", "-m", "gpt_2_distributed_amd.train_gpt2_distributed", "--data_dir", str(data),
            "--synthetic", "2", "--synthetic_tokens", "60000", "--seq_len", "128", "--batch", "4", "--model", "124M",
            "--grad_accum_steps", "2", "--workers", "0", "--log_every", "1", *mode_args]
    env = dict(os.environ, GPT2MI_FORCE_COLLECTIVES="1")
    r = subprocess.run(base + ["--max_steps", "4", "--save_every", "2", "--save_dir", str(tmp_path / "a")], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    full = {json.loads(l)["step"]: json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")}
    assert sorted(full) == [1, 2, 3, 4] and all(0.0 < v < 20.0 for v in full.values()), full
    ck = tmp_path / "a" / "step_0000002"
    assert (ck / "model.pt").exists() and ((ck / "optim_rank0.pt").exists() if mode != "ddp" else (ck / "optim.pt").exists())
    r = subprocess.run(base + ["--max_steps", "4", "--save_every", "100", "--save_dir", str(tmp_path / "b"),
                               "--resume", str(ck)], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    resumed = {json.loads(l)["step"]: json.loads(l)["loss"] for l in r.stdout.splitlines() if l.startswith("{")}
    for s in (3, 4):
        assert abs(resumed[s] - full[s]) <= 1e-4 * full[s], (s, resumed, full)
