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


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgpt2mi.so not built (run __graft_entry__.build())")
def test_refuses_shapes_that_overflow_the_dropout_index():
    """The counter-based dropout hashes 32-bit element / pair indices: a dropout launch whose indices
    would wrap is refused before anything is launched (no GPU needed: argument checks only)."""
    from gpt_2_distributed_amd import _lib
    lib = _lib.load()
    # attention: B*H*T*T = 256*16*1024*1024 = 2^32
    assert lib.gpt2mi_attn_fwd(None, None, None, 256, 1024, 16, 64, 0.1, 1, None) == 22
    assert b"32-bit dropout" in lib.gpt2mi_last_error()
    assert lib.gpt2mi_attn_bwd(None, None, None, None, None, None, None, 256, 1024, 16, 64, 0.1, 1, None) == 22
    # GEMM epilogue dropout: M*N = 2^20 * 2^13 = 2^33 pairs*2
    assert lib.gpt2mi_gemm(0, 2, 1 << 20, 1 << 13, 64, None, 64, None, 64, None, 1 << 13, None, None, None, 0,
                           1.0, None, 0, 1, 0.1, 1, None, 0, None) == 22
    assert b"32-bit dropout" in lib.gpt2mi_last_error()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgpt2mi.so not built (run __graft_entry__.build())")
def test_gemm_schedule_is_a_per_call_argument():
    """ABI v8: the GEMM schedule is passed with every call (no process-global switch is exported); an unknown
    schedule value is refused before any launch."""
    from gpt_2_distributed_amd import _lib
    lib = _lib.load()
    for gone in ("gpt2mi_set_gemm_impl", "gpt2mi_set_gemm_persistent"):
        assert not hasattr(ctypes.CDLL(LIB), gone), gone
    assert lib.gpt2mi_gemm(0, 0, 256, 256, 64, None, 64, None, 64, None, 256, None, None, None, 0,
                           1.0, None, 0, 1, 0.0, 1, None, 0x200, None) == 22
    assert b"sched" in lib.gpt2mi_last_error()
    assert lib.gpt2mi_gemm_wgrad(256, 256, 64, None, 256, None, 256, None, 256, 0, 1.0, None, None, 0, 1, 0x1ff,
                                 None) == 22


def test_schedule_flags_match_the_header():
    """The GPT2MI_SCHED_* values the bindings pass (AUTO, NO_PERSISTENT, BF16_SLABS since v10) are the header's."""
    from gpt_2_distributed_amd import _lib
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    flags = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define GPT2MI_SCHED_(\w+) (0x[0-9a-fA-F]+|\d+)", src)}
    assert flags == {"AUTO": _lib.SCHED_AUTO, "NO_PERSISTENT": _lib.SCHED_NO_PERSISTENT,
                     "SHARED_CUS": _lib.SCHED_SHARED_CUS, "BF16_SLABS": _lib.SCHED_BF16_SLABS}
