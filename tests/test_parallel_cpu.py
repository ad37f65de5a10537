"""Multi-process data-parallel logic on CPU with gloo (world sizes 2, 3 and the 8 of the BASELINE node): the bucketed SUM
all-reduce over a flat arena (DDP path), the FSDP shard plan (any world size) and its bf16/fp32
reduce-scatter / all-gather round trip. Gradients reach the collectives pre-divided by world (the
engine's GradHooks.begin_backward), so a SUM is the average on every backend; the identity the DDP
golden rests on is then: the mean of per-rank grads of equal-size batches equals the
single-process grad of the concatenated batch (tests/test_ddp_gpu.py checks it against the reference)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # pragma: no cover - surfaced in the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


def _bucketed(rank, world):
    from gpt_2_distributed_amd.parallel import BucketedReducer
    n = 10_000
    g = torch.Generator().manual_seed(rank)
    flat = torch.randn(n, generator=g) / world  # what a synced backward hands over: grads pre-divided by world
    expect = sum(torch.randn(n, generator=torch.Generator().manual_seed(r)) for r in range(world)) / world
    # ranges become final in descending arena order (like blocks L-1 .. 0, then the embeddings)
    bounds = [0, 1000, 2500, 4000, 7000, 9000, n]
    order = [(f"r{i}", bounds[i], bounds[i + 1]) for i in reversed(range(len(bounds) - 1))]
    red = BucketedReducer(flat, order, bucket_mb=3000 * 4 / 2**20)
    for name, _, _ in order[:3]:
        red.mark_ready(name)
    n_launched = red.launched
    red.finish()
    return (torch.allclose(flat, expect, atol=1e-6), n_launched, red.launched == 0 and red.next == 0)


def _bucketed_deferred(rank, world):
    """finish(defer_last=True) (DistributedDataParallel(overlap_optimizer=True)): every bucket but the last is complete
    when finish returns; the last is handed back as (work, lo, hi) over the range that became final last."""
    from gpt_2_distributed_amd.parallel import BucketedReducer
    n = 10_000
    flat = torch.randn(n, generator=torch.Generator().manual_seed(rank)) / world
    expect = sum(torch.randn(n, generator=torch.Generator().manual_seed(r)) for r in range(world)) / world
    bounds = [0, 1000, 2500, 4000, 7000, 9000, n]
    order = [(f"r{i}", bounds[i], bounds[i + 1]) for i in reversed(range(len(bounds) - 1))]
    red = BucketedReducer(flat, order, bucket_mb=2000 * 4 / 2**20)
    for name, _, _ in order[:-1]:
        red.mark_ready(name)
    work, lo, hi = red.finish(defer_last=True)
    work.wait()
    return (torch.allclose(flat, expect, atol=1e-6), lo, hi, red.launched == 0 and red.next == 0)


def test_bucketed_allreduce_deferred_last_bucket_gloo():
    out = _spawn(_bucketed_deferred)
    for r, v in out.items():
        assert isinstance(v, tuple), v
        ok, lo, hi, was_reset = v
        assert ok and was_reset
        assert (lo, hi) == (0, 1000)  # the embeddings' range (first in the arena, final last)


@pytest.mark.parametrize("world", [2, 8])  # 8: the rank count of the BASELINE node, rehearsed on CPU
def test_bucketed_allreduce_gloo(world):
    out = _spawn(_bucketed, world)
    for r, v in out.items():
        assert isinstance(v, tuple), v
        ok, n_launched, was_reset = v
        assert ok
        assert n_launched >= 1  # buckets issued before finish (they overlap the rest of the backward)
        assert was_reset        # finish() leaves the reducer ready for the next backward


def _ddp_inflight(rank, world):
    """DDP's GEMM-schedule signal (GradHooks.inflight): False in the backward until the first bucket's all-reduce is
    issued (the lm_head backward and the last blocks keep the persistent GEMM schedule), then True while a bucket has
    not completed, False after finish(); never in a no_sync micro-step."""
    from gpt_2_distributed_amd.parallel import BucketedReducer, _DDPHooks

    class _Eng:
        grad_dirty = False
    n = 8000
    flat = torch.ones(n) / world
    order = [(f"r{i}", i * 1000, (i + 1) * 1000) for i in reversed(range(8))]
    red = BucketedReducer(flat, order, bucket_mb=2500 * 4 / 2**20)
    hooks = _DDPHooks(_Eng(), world, red)
    seen = []
    hooks.begin_backward()
    seen.append(hooks.inflight())
    hooks.ready("r7")              # 1000 elements ready: below one bucket, nothing issued
    seen.append(hooks.inflight())
    hooks.ready("r6")
    hooks.ready("r5")              # 3000 >= 2500: the first bucket goes out
    seen.append(hooks.inflight() == any(not w.is_completed() for w in red.works) and len(red.works) == 1)
    hooks.end_backward()
    seen.append(hooks.inflight())
    hooks.sync = False
    hooks.ready("r7")
    seen.append(hooks.inflight())
    return seen, bool(torch.allclose(flat, torch.ones(n)))


def test_ddp_inflight_signal_gloo():
    out = _spawn(_ddp_inflight)
    for r, v in out.items():
        assert isinstance(v, tuple), v
        assert v[0] == [False, False, True, False, False], v  # (3rd: inflight tracks the bucket's completion)
        assert v[1]


def test_backward_ready_order_is_contiguous():
    """The engine's ready events (head, h.L-1 .. h.0, embed) tile the arena contiguously in reverse order."""
    from gpt_2_distributed_amd.model import GPT2, GPT2Config
    from gpt_2_distributed_amd.parallel import backward_order, unit_ranges
    m = GPT2(GPT2Config(n_layer=3, n_head=2, n_embd=128, vocab_size=509, n_positions=64))
    units = unit_ranges(m.layout, 3)
    assert [u[0] for u in units] == ["embed", "h.0", "h.1", "h.2", "head"]
    assert units[0][1] == 0 and units[-1][2] == m.layout.total
    for (_, _, hi), (_, lo, _) in zip(units, units[1:]):
        assert hi == lo
    order = backward_order(units)
    assert [u[0] for u in order] == ["head", "h.2", "h.1", "h.0", "embed"]
    # every parameter lies in exactly one unit, and each block's 12 tensors in its own
    for n, sl in m.layout.slots.items():
        owners = [u for u, lo, hi in units if lo <= sl.offset < hi]
        assert len(owners) == 1
        if n.startswith("transformer.h."):
            assert owners[0] == "h." + n.split(".")[2]


@pytest.mark.parametrize("world", [1, 2, 3, 6, 8, 32])
def test_shard_plan_any_world_size(world):
    """FSDP shard plan: every unit splits into `world` aligned equal chunks covering it (zero padding
    past its end), for world sizes with odd factors too (3, 6, 12 ...)."""
    from gpt_2_distributed_amd.model import GPT2, GPT2Config
    from gpt_2_distributed_amd.parallel import SHARD_ALIGN, plan_shards, unit_ranges
    m = GPT2(GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=509, n_positions=64))
    plans, total = plan_shards(unit_ranges(m.layout, 2), world)
    off = 0
    for p in plans:
        assert p.per % SHARD_ALIGN == 0 and p.per * world >= p.n > p.per * (world - 1) - SHARD_ALIGN * world
        assert p.soff == off
        off += p.per
    assert total == off


def _shard_math(rank, world):
    """The FSDP collective pattern of one unit, in both reduce/param dtypes: a unit of n elements packed
    (zero-padded) to world*per, reduce-scattered (SUM of world-pre-divided grads) into this rank's per
    chunk, and the chunks all-gathered back: the first n elements are the average, in unit order. Both
    collectives run in place as the wrapper issues them (parallel.py _reduce_scatter: the shard is this rank's
    chunk of the packed input; bf16_chunk: the gather source is this rank's chunk of the gather buffer)."""
    from gpt_2_distributed_amd.parallel import plan_shards
    ok = True
    n = 1000
    (p,), _ = plan_shards([("u", 0, n)], world)
    for dt in (torch.float32, torch.bfloat16):
        g = torch.zeros(p.per * world, dtype=dt)
        g[:n] = (torch.arange(n, dtype=torch.float32) % 64 * (rank + 1) / world).to(dt)
        shard = g[rank * p.per:(rank + 1) * p.per]
        dist.reduce_scatter_tensor(shard, g, op=dist.ReduceOp.SUM)
        full = torch.full((p.per * world,), float("nan"), dtype=dt)
        full[rank * p.per:(rank + 1) * p.per] = shard
        dist.all_gather_into_tensor(full, full[rank * p.per:(rank + 1) * p.per])
        exp = (torch.arange(n, dtype=torch.float32) % 64) * sum(range(1, world + 1)) / world
        tol = 1e-6 if dt == torch.float32 else 2e-2
        ok &= bool(torch.allclose(full[:n].float(), exp, rtol=tol, atol=tol)) and bool((full[n:] == 0).all())
    return ok


@pytest.mark.parametrize("world", [2, 3, 8])
def test_reduce_scatter_all_gather_gloo(world):
    out = _spawn(_shard_math, world)
    assert all(v is True for v in out.values()), out


def _loader_partition(rank, world):
    import numpy as np
    from gpt_2_distributed_amd import dataloader as D
    d = tempfile.mkdtemp()
    rng = np.random.default_rng(0)
    for i in range(8):
        rng.integers(0, 50257, size=2000).astype("<u2").tofile(os.path.join(d, f"train_{i:02d}.bin"))
    paths = D.get_shard_paths(d)
    ds = D.TokenShardDataset(paths, seq_len=64)
    return (ds.rank, ds.world, [x[0, :4].tolist() for x, _ in D.iter_batches(paths, 64, 4, num_workers=2)])


def test_loader_partitions_by_rank_gloo():
    out = _spawn(_loader_partition)
    assert out[0][:2] == (0, 2) and out[1][:2] == (1, 2)
    assert out[0][2] and out[1][2] and out[0][2] != out[1][2]


def test_wgrad_split_choice_balances_the_last_round():
    """Host-side split-K choice (gpt_2_distributed_amd/_lib.py): the tied lm_head wgrad (591 tiles =
    2.3 rounds of 256 CUs) is split 3 ways; the block wgrads fill one round; every split keeps >= 4
    K-tiles."""
    from gpt_2_distributed_amd._lib import wgrad_splits
    assert wgrad_splits(50432, 768, 65536) == 3
    assert wgrad_splits(3072, 768, 65536) * 36 <= 256
    assert wgrad_splits(768, 768, 65536) * 9 <= 256
    for m, n, k in [(50432, 768, 4096), (2304, 768, 1024), (768, 768, 512)]:
        s = wgrad_splits(m, n, k)
        assert s >= 1 and k // s >= 256
