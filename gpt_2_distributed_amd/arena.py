"""Flat parameter arena: every GPT-2 parameter is a view into ONE fp32 buffer.

Why (MI355X-first): the fused AdamW, the clip-norm sum of squares and the DDP/ZeRO collectives all
run over a single contiguous fp32 range (one kernel / one bucketed stream of RCCL calls instead of
148 tensors), and the bf16 weight shadow that the MFMA GEMMs read has the same offsets.

Layout: parameters in ``GPT2.parameters()`` order (model.py:235-247 module order), each starting
at a multiple of 64 elements (256 B). ``wte`` is allocated as [Vpad, C] with Vpad = V rounded up to
256 so the tied lm_head GEMM tiles evenly; rows >= V stay zero forever (zero grad, zero moments).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

ALIGN = 64


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class Slot:
    name: str
    shape: Tuple[int, ...]
    offset: int      # element offset in the arena
    numel: int       # elements of the parameter proper
    reserved: int    # elements reserved (>= numel; wte includes the zero pad rows)


class ArenaLayout:
    def __init__(self, shapes: "OrderedDict[str, tuple]", vpad: int):
        self.slots: "OrderedDict[str, Slot]" = OrderedDict()
        off = 0
        for name, shape in shapes.items():
            n = 1
            for s in shape:
                n *= s
            res = n
            if name.endswith("wte.weight"):
                res = vpad * shape[1]
            self.slots[name] = Slot(name, tuple(shape), off, n, res)
            off = round_up(off + res, ALIGN)
        self.total = round_up(off, 1024)

    def view(self, arena: torch.Tensor, name: str) -> torch.Tensor:
        s = self.slots[name]
        return arena[s.offset:s.offset + s.numel].view(s.shape)

    def padded_view(self, arena: torch.Tensor, name: str, rows: int) -> torch.Tensor:
        s = self.slots[name]
        return arena[s.offset:s.offset + s.reserved].view(rows, -1)

    def ranges(self) -> List[Tuple[str, int, int]]:
        return [(s.name, s.offset, s.reserved) for s in self.slots.values()]
