#!/usr/bin/env python
"""Prices running the memory-bound cross-entropy pass beside the compute-bound lm_head GEMM on disjoint CU sets
(hipExtStreamCreateWithCUMask): if the GEMM, power-limited on the full chip, loses less than its CU share when it
runs on fewer CUs, the xent pass's HBM traffic can ride under it (a row-chunked lm_head would pipeline xent(chunk i)
under the forward GEMM of chunk i+1). Measured at cfg 2's head (65536 x 50432 x 768): the persistent forward GEMM on
the full chip, on a CU-masked stream with a grid of that many CUs (tools/variant_lib.sh builds with
-DGPT2MI_PERSIST_GRID), the xent pass alone on the remaining CUs, and both at once.

    python tools/overlap_probe.py tools/ab/lib_base.so tools/ab/lib_grid208.so tools/ab/lib_grid224.so
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lib_ab import bind  # noqa: E402

dev = "cuda"
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
NCU = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(bits):
    words = (NCU + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, m) == 0
    return torch.cuda.ExternalStream(s.value)


def main():
    base, *grids = [bind(p) for p in sys.argv[1:]]
    gsz = [int(os.path.basename(p).split("grid")[1].split(".")[0]) for p in sys.argv[2:]]
    M, C, Vp, V = 65536, 768, 50432, 50257
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(M, C, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(Vp, C, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    logits = torch.empty(M, Vp, dtype=torch.bfloat16, device=dev)
    logits2 = (torch.randn(M, Vp, device=dev, generator=g) * 2).to(torch.bfloat16)
    dlog = torch.empty_like(logits2)
    labels = torch.randint(0, V, (M,), device=dev, generator=g)
    rows, lse, loss, ic = (torch.empty(M, device=dev), torch.empty(M, device=dev), torch.empty(1, device=dev),
                           torch.empty(1, device=dev))

    def gemm(lib, st):
        assert lib.gpt2mi_gemm(0, 0, M, Vp, C, x.data_ptr(), C, w.data_ptr(), C, logits.data_ptr(), Vp, None, None,
                               None, 0, 1.0, None, 0, 1, 0.0, 5, None, 0, st.cuda_stream) == 0

    def xent(st):
        assert base.gpt2mi_xent_fwd(logits2.data_ptr(), Vp, labels.data_ptr(), rows.data_ptr(), lse.data_ptr(),
                                    dlog.data_ptr(), Vp, M, V, -100, loss.data_ptr(), ic.data_ptr(),
                                    st.cuda_stream) == 0

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    main_st = torch.cuda.current_stream()

    def timed(fns):
        """fns: [(callable, stream)], launched together; ms from a start event every stream waits for to the last end."""
        torch.cuda.synchronize()
        s = ev()
        s.record(main_st)
        ends = []
        for fn, st in fns:
            st.wait_event(s)
            fn(st)
            e = ev()
            e.record(st)
            ends.append(e)
        for e in ends:
            main_st.wait_event(e)
        f = ev()
        f.record(main_st)
        torch.cuda.synchronize()
        return s.elapsed_time(f)

    def med(fns, n=7):
        timed(fns)
        return sorted(timed(fns) for _ in range(n))[n // 2]

    full = masked_stream(range(NCU))
    print(f"CUs {NCU}", flush=True)
    tg = med([(lambda st: gemm(base, st), main_st)])
    tx = med([(xent, main_st)])
    print(f"full chip: gemm {tg * 1e3:7.1f} us, xent {tx * 1e3:7.1f} us, sequential {1e3 * (tg + tx):7.1f} us",
          flush=True)
    tgf = med([(lambda st: gemm(base, st), full)])
    print(f"full-mask stream: gemm {tgf * 1e3:7.1f} us", flush=True)
    for lib, n in zip(grids, gsz):
        free = NCU - n
        # candidate bit orders: XCD-major (bits [32x, 32x + 32) = XCD x) and XCD-interleaved (bit i on XCD i % 8)
        for name, small in (("xcd-major", [b for b in range(NCU) if b % 32 < free // 8]),
                            ("interleaved", list(range(free)))):
            big_st, small_st = masked_stream([b for b in range(NCU) if b not in small]), masked_stream(small)
            t1 = med([(lambda st: gemm(lib, st), big_st)])
            t2 = med([(xent, small_st)])
            t3 = med([(lambda st: gemm(lib, st), big_st), (xent, small_st)])
            print(f"grid {n} / {free} free ({name}): gemm {t1 * 1e3:7.1f} us, xent {t2 * 1e3:7.1f} us, "
                  f"both {t3 * 1e3:7.1f} us (vs {1e3 * (tg + tx):7.1f} sequential on the full chip)", flush=True)


if __name__ == "__main__":
    main()
