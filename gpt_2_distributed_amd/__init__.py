"""MI355X-native GPT-2 training step: a drop-in for dpickem/gpt_2_distributed's model.py /
dataloader.py / train_gpt2_distributed.py surfaces, running on hand-written gfx950 HIP kernels
(libgpt2mi.so, C ABI in include/gpt2mi.h)."""
# Runtime setting (not set here: importing the package changes no process-wide state): the entry points bench.py and
# train_gpt2_distributed's __main__ set HIP_FORCE_DEV_KERNARG=1 before the HIP runtime starts, so that each launch's
# waves read their kernel arguments from device memory instead of host memory over PCIe (a step launches ~300 kernels;
# bench A/B 58.90 / 59.07 -> 58.59 / 58.63 ms, profiles/r5v/). A program embedding the model can export it itself
# (INTEGRATION.md §4); it affects every kernel of the process, torch's included.

from .model import (GPT, GPT2, GPT2Backbone, GPT2Block, GPT2Config, MLP, MODEL_SIZES,  # noqa: F401
                    CausalMultiHeadSelfAttention, NewGELU)
from .parallel import DistributedDataParallel, ShardedDataParallel, init_distributed  # noqa: F401

DEFAULT_CONFIG = GPT2Config()  # train_gpt2_distributed.py:42-44 (124M; --seq_len replaces n_positions)

__all__ = ["GPT", "GPT2", "GPT2Backbone", "GPT2Block", "GPT2Config", "MLP", "CausalMultiHeadSelfAttention",
           "NewGELU", "MODEL_SIZES", "DEFAULT_CONFIG", "DistributedDataParallel", "ShardedDataParallel",
           "init_distributed"]
