"""C-ABI checks that need no GPU: libgpt2mi.so loads, exports every entry point include/gpt2mi.h
declares, and the ctypes binding (_lib._SIGS) types exactly that set. No compute calls here."""
import ctypes
import os
import re

import pytest

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "gpt2mi.h")
LIB = os.path.join(REPO, "gpt_2_distributed_amd", "libgpt2mi.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gpt2mi_\w+)\s*\(", src)))


def test_header_declares_the_entry_points():
    names = declared()
    for n in ("gpt2mi_gemm", "gpt2mi_gemm_f32", "gpt2mi_attn_fwd", "gpt2mi_attn_bwd", "gpt2mi_xent_fwd",
              "gpt2mi_adamw", "gpt2mi_layernorm_fwd", "gpt2mi_layernorm_bwd", "gpt2mi_embed_fwd"):
        assert n in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgpt2mi.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    lib.gpt2mi_abi_version.restype = ctypes.c_int
    from gpt_2_distributed_amd import _lib
    hdr = re.search(r"#define GPT2MI_ABI_VERSION (\d+)", open(HEADER).read())
    assert lib.gpt2mi_abi_version() == _lib.ABI_VERSION == int(hdr.group(1))


def test_ctypes_binding_covers_the_header():
    from gpt_2_distributed_amd import _lib
    assert sorted(_lib.EXPORTED) == declared()
