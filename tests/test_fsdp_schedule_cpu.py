"""FullyShardedDataParallel's all-gather schedule (CPU: the scheduling logic only, on a stand-in with fake works).

VERDICT r4 item 5: the prefetch is bounded by a byte budget of gathered output instead of issuing every unit's gather at
the first unit, and pending gathers are retired by an event query (work.is_completed()) instead of a fixed fence unit,
so the compute stream never waits for a gather other than the one of the unit about to run."""
import torch
import torch.nn as nn

from gpt_2_distributed_amd.parallel import FullyShardedDataParallel, ShardPlan


class _Work:
    def __init__(self, done=False):
        self.done, self.waited = done, False

    def is_completed(self):
        return self.done

    def wait(self):
        self.waited = True


def _stand_in(n_blocks=12, per=1 << 20, world=4, budget=None, depth=None):
    f = FullyShardedDataParallel.__new__(FullyShardedDataParallel)
    nn.Module.__init__(f)
    f.world, f.store = world, None
    names = ["embed"] + [f"h.{i}" for i in range(n_blocks)] + ["head"]
    f.order = names
    f.plan = {n: ShardPlan(n, 0, per * world, per, 0) for n in names}
    f.prefetch_depth = depth
    f.prefetch_bytes = FullyShardedDataParallel.PREFETCH_BYTES if budget is None else budget
    f._valid = {n: None for n in names}
    f._pending, f._fenced = {}, set()
    issued = []

    def issue(unit, dtype):
        issued.append(unit)
        f._pending[unit] = (_Work(), dtype, None)
    f._issue_gather = issue
    return f, issued


def test_prefetch_stays_within_the_byte_budget():
    bf = torch.bfloat16
    # 8 MiB of gathered bf16 per unit (1 Mi elements x 4 ranks x 2 B): a 20 MiB budget keeps 2 units ahead
    f, issued = _stand_in(budget=20 << 20)
    f._pending["h.0"] = (_Work(), bf, None)
    f._prefetch_after("h.0", bf)
    assert issued == ["h.1", "h.2"]
    # consuming h.1 frees its bytes: one more unit goes out
    f._pending.pop("h.0")
    f._pending.pop("h.1")
    f._prefetch_after("h.1", bf)
    assert issued == ["h.1", "h.2", "h.3"]


def test_prefetch_always_allows_one_unit_ahead_and_respects_depth():
    bf = torch.bfloat16
    f, issued = _stand_in(budget=1)  # smaller than any unit
    f._prefetch_after("h.3", bf)
    assert issued == ["h.4"]
    f, issued = _stand_in(depth=3)
    f._prefetch_after("embed", bf)
    assert issued == ["h.0", "h.1", "h.2"]
    # the default budget (512 MiB) holds the whole stand-in model
    f, issued = _stand_in()
    f._prefetch_after("embed", bf)
    assert issued == f.order[1:]


def test_prefetch_skips_gathered_and_pending_units():
    bf = torch.bfloat16
    f, issued = _stand_in(budget=100 << 20)
    f._valid["h.1"] = bf
    f._pending["h.2"] = (_Work(), bf, None)
    f._prefetch_after("h.0", bf)
    assert "h.1" not in issued and "h.2" not in issued and issued[0] == "h.3"


def test_completed_gathers_are_retired_without_waiting_for_pending_ones():
    bf = torch.bfloat16
    f, _ = _stand_in()
    done, busy = _Work(done=True), _Work(done=False)
    f._pending = {"h.1": (done, bf, None), "h.2": (busy, bf, None)}
    f._retire_completed()
    assert done.waited and "h.1" in f._fenced
    assert not busy.waited and "h.2" not in f._fenced


def _units(cfg):
    """unit_ranges of a model of ``cfg`` without building it: the layout from the parameter shapes (model.py order)."""
    from collections import OrderedDict
    from gpt_2_distributed_amd.arena import ArenaLayout, round_up
    from gpt_2_distributed_amd.parallel import unit_ranges
    C, V, L = cfg["n_embd"], cfg["vocab_size"], cfg["n_layer"]
    shapes = OrderedDict([("transformer.wte.weight", (V, C)), ("transformer.wpe.weight", (1024, C))])
    for l in range(L):
        p = f"transformer.h.{l}."
        for n, sh in (("ln1.weight", (C,)), ("ln1.bias", (C,)), ("attn.qkv.weight", (3 * C, C)),
                      ("attn.qkv.bias", (3 * C,)), ("attn.proj.weight", (C, C)), ("attn.proj.bias", (C,)),
                      ("ln2.weight", (C,)), ("ln2.bias", (C,)), ("mlp.fc1.weight", (4 * C, C)),
                      ("mlp.fc1.bias", (4 * C,)), ("mlp.fc2.weight", (C, 4 * C)), ("mlp.fc2.bias", (C,))):
            shapes[p + n] = sh
    shapes["transformer.ln_f.weight"] = (C,)
    shapes["transformer.ln_f.bias"] = (C,)
    return unit_ranges(ArenaLayout(shapes, round_up(V, 256)), L)


def test_reshard_memory_plan_of_the_baseline_models():
    """with reshard_after_forward the per-rank memory (sharded state + compute views + staging)
    falls with the world size for GPT-2 124M / 350M / 1.5B, and at 8 ranks it is well under the resident mode's, whose
    compute views stay the whole model on every rank."""
    from gpt_2_distributed_amd.parallel import fsdp_memory_plan
    for name, cfg in {"124M": dict(n_embd=768, n_layer=12, vocab_size=50257),
                      "350M": dict(n_embd=1024, n_layer=24, vocab_size=50257),
                      "1.5B": dict(n_embd=1600, n_layer=48, vocab_size=50257)}.items():
        units = _units(cfg)
        rs = [fsdp_memory_plan(units, w, True)["total"] for w in (1, 2, 4, 8)]
        rd = [fsdp_memory_plan(units, w, False)["total"] for w in (1, 2, 4, 8)]
        assert rs[0] > rs[1] > rs[2] > rs[3], (name, rs)
        assert rs[3] < 0.6 * rd[3], (name, rs[3], rd[3])
        v8 = fsdp_memory_plan(units, 8, True)["compute_view_bytes"]
        assert v8 == fsdp_memory_plan(units, 1, True)["compute_view_bytes"]  # independent of the world size
        print(name, "per-rank GB at 1/2/4/8 ranks: reshard", [round(x / 1e9, 2) for x in rs],
              "resident", [round(x / 1e9, 2) for x in rd])


def test_staging_ring_slots_are_not_reissued_while_in_use():
    """reshard_after_forward's 3-slot staging rings. A gather ring's next slot is not handed out while the
    unit it holds is still pending (not unpacked), nor a reduce-scatter ring's while the reduce-scatter that read it
    has not been waited for; the ring otherwise walks its slots round-robin."""
    import pytest
    bf = torch.bfloat16
    f, _ = _stand_in()
    f.flat_param = nn.Parameter(torch.zeros(4))
    f._bufs, f._stage_next, f._stage_user, f._rs_slot_work = {}, {}, {}, {}
    S = FullyShardedDataParallel.STAGE_SLOTS
    for k in range(S):  # three gathers in flight, one per slot
        i, _buf = f._ring("ag16", bf, 8)
        assert i == k
        f._stage_user[("ag16", i)] = f"h.{k}"
        f._pending[f"h.{k}"] = (_Work(), bf, None)
    assert not f._ring_free("ag16")
    with pytest.raises(RuntimeError, match="pending gather of h.0"):
        f._ring("ag16", bf, 8)
    f._pending.pop("h.0")  # h.0 unpacked: its slot may be refilled
    assert f._ring_free("ag16") and f._ring("ag16", bf, 8)[0] == 0
    # reduce-scatter ring: a slot whose reduce-scatter was not waited for is refused
    w = _Work()
    i, _buf = f._ring("rs16", bf, 8)
    f._rs_slot_work[("rs16", i)] = w
    for _ in range(S - 1):
        f._ring("rs16", bf, 8)
    with pytest.raises(RuntimeError, match="unwaited reduce-scatter"):
        f._ring("rs16", bf, 8)
    f._rs_slot_work.pop(("rs16", i)).wait()
    assert f._ring("rs16", bf, 8)[0] == i and w.waited


def test_memory_plan_counts_the_bf16_shard_once():
    """the bf16 shard is part of the sharded state (18 B per sharded element); the staging the plan prices
    leaves it out in both modes (resident: this rank's chunk of every unit's bf16 gather buffer; resharded: the shard
    buffer), so at one rank the resident mode stages only the reduce-scatter inputs."""
    from gpt_2_distributed_amd.parallel import fsdp_memory_plan, plan_shards
    units = _units(dict(n_embd=768, n_layer=12, vocab_size=50257))
    plans, shard_total = plan_shards(units, 1)
    rd = fsdp_memory_plan(units, 1, False)
    assert rd["staging_bytes"] == shard_total * 2  # world 1: gather buffer == shard; one bf16 reduce-scatter input
    plans8, shard8 = plan_shards(units, 8)
    rd8 = fsdp_memory_plan(units, 8, False)
    assert rd8["staging_bytes"] == sum(p.per * 7 * 2 + p.per * 8 * 2 for p in plans8)
    assert rd8["sharded_state_bytes"] == shard8 * 18
