"""MI355X-native GPT-2 training step: a drop-in for dpickem/gpt_2_distributed's model.py /
dataloader.py / train_gpt2_distributed.py surfaces, running on hand-written gfx950 HIP kernels
(libgpt2mi.so, C ABI in include/gpt2mi.h)."""
import os as _os

# Kernel arguments in device memory: each launch's waves then read their arguments from HBM instead of host memory over
# PCIe (a step launches ~300 kernels; bench A/B 58.90 / 59.07 -> 58.59 / 58.63 ms, profiles/r5v/). Read when the HIP
# runtime initialises, so it takes effect when this package is imported before the first GPU call; an explicit
# HIP_FORCE_DEV_KERNARG in the environment wins.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from .model import (GPT, GPT2, GPT2Backbone, GPT2Block, GPT2Config, MLP, MODEL_SIZES,  # noqa: F401
                    CausalMultiHeadSelfAttention, NewGELU)
from .parallel import DistributedDataParallel, ShardedDataParallel, init_distributed  # noqa: F401

DEFAULT_CONFIG = GPT2Config()  # train_gpt2_distributed.py:42-44 (124M; --seq_len replaces n_positions)

__all__ = ["GPT", "GPT2", "GPT2Backbone", "GPT2Block", "GPT2Config", "MLP", "CausalMultiHeadSelfAttention",
           "NewGELU", "MODEL_SIZES", "DEFAULT_CONFIG", "DistributedDataParallel", "ShardedDataParallel",
           "init_distributed"]
