"""Model surface checks that need no GPU: config, module tree, parameter order/names, init parity
with the reference (tests/golden/init_124m.json), the arena layout, and the no-CPU-fallback rule."""
import dataclasses
import json
import os

import pytest
import torch

from gpt_2_distributed_amd import model as M
from oracle import model_ref
from tests.conftest import GOLDEN


def test_config_is_frozen_and_replaceable():
    cfg = M.GPT2Config()
    assert (cfg.vocab_size, cfg.n_positions, cfg.n_embd, cfg.n_layer, cfg.n_head) == (50257, 1024, 768, 12, 12)
    assert cfg.resid_pdrop == cfg.attn_pdrop == 0.1 and cfg.layer_norm_eps == 1e-5
    with pytest.raises(dataclasses.FrozenInstanceError):
        cfg.n_layer = 3
    assert dataclasses.replace(cfg, n_positions=256).n_positions == 256


def test_124m_params_names_order_and_init_match_reference():
    ref = json.load(open(os.path.join(GOLDEN, "init_124m.json")))
    m = M.GPT2(M.GPT2Config())
    named = list(m.named_parameters())
    assert [n for n, _ in named] == list(ref["tensors"])
    assert len(named) == 148 and sum(p.numel() for _, p in named) == 124_439_808
    sd = m.state_dict()
    assert len(sd) == 149 and "lm_head.weight" in sd
    assert m.lm_head.weight is m.transformer.wte.weight
    for n, p in named:
        r = ref["tensors"][n]
        assert list(p.shape) == r["shape"]
        assert [float(v) for v in p.detach().reshape(-1)[:4]] == r["head"], n
        d = p.detach().double()
        assert abs(float(d.sum()) - r["sum"]) <= 1e-9 * max(1.0, abs(r["sum"])), n


def test_params_are_views_of_one_arena_with_zero_vocab_pad():
    cfg = M.GPT2Config(n_layer=2, n_head=2, n_embd=128, vocab_size=509, n_positions=64)
    m = M.GPT2(cfg)
    base = m.arena.data_ptr()
    for n, p in m.named_parameters():
        s = m.layout.slots[n]
        assert p.data_ptr() == base + 4 * s.offset, n
        assert s.offset % 64 == 0
    assert m.vpad == 512
    wte = m.layout.padded_view(m.arena, "transformer.wte.weight", m.vpad)
    assert torch.all(wte[509:] == 0)
    ref = model_ref.init_params(model_ref.Cfg(**dataclasses.asdict(cfg)))
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), ref[n]), n


def test_cpu_forward_raises_no_fallback():
    cfg = M.GPT2Config(n_layer=1, n_head=2, n_embd=128, vocab_size=509, n_positions=64)
    m = M.GPT2(cfg)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(torch.zeros(1, 64, dtype=torch.long))
    with pytest.raises(ValueError, match="Sequence length"):
        m(torch.zeros(1, 65, dtype=torch.long))


def test_aliases():
    assert M.GPT is M.GPT2
    assert set(M.MODEL_SIZES) == {"124M", "350M", "1.5B"}
