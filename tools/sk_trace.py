#!/usr/bin/env python3
"""Phase timeline of the stream-K GEMM (variant 6) per workgroup, from the
A/B build with -DHPA_SK_TRACE (s_memrealtime, 100 MHz):
  0 entry  1 wave 0's steps done  2 all waves done (barrier)
  per super-tile i (0, 1): 3+4i folded  4+4i ticket back  5+4i slabs summed  6+4i epilogue done
usage: HPA_LIB=llm.c-paged_amd/libpaged_hip_sktrace.so tools/sk_trace.py"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pagedattn as pa  # noqa: E402
from gemm_tune import shape_inputs, time_fused, dev  # noqa: E402

NAMES = {1: "w0 steps", 2: "barrier", 3: "fold0", 4: "ticket0", 5: "slabs0", 6: "epi0",
         7: "fold1", 8: "ticket1", 9: "slabs1", 10: "epi1"}


def main():
    pa.init(0)
    L = pa.lib()
    L.hpa_sk_trace_read.argtypes = [ctypes.c_void_p]
    buf = np.zeros(1024 * 16, np.uint64)
    for name, M, K, N, epi in [("124M attproj", 64, 768, 768, pa.HPA_FEPI_RESID),
                               ("124M fc", 64, 768, 3072, pa.HPA_FEPI_GELU),
                               ("XL qkv", 64, 1600, 4800, pa.HPA_FEPI_GELU),
                               ("XL attproj", 64, 1600, 1600, pa.HPA_FEPI_RESID),
                               ("XL logits", 64, 1600, 50257, pa.HPA_FEPI_LOGITS)]:
        g = shape_inputs(M, K, N, epi, False)
        nf, nc = ctypes.c_size_t(), ctypes.c_size_t()
        pa.check(L.hpa_gemm_sk_workspace(N, ctypes.byref(nf), ctypes.byref(nc)), "ws")
        g.sk_slab = dev(np.zeros(nf.value, np.float32))
        g.sk_count = dev(np.zeros(nc.value, np.int32))
        g.variant = 6
        us = time_fused(g, iters=20)
        pa.check(L.hpa_sk_trace_read(buf.ctypes.data), "trace")  # clears
        pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
        pa.check(L.hpa_sk_trace_read(buf.ctypes.data), "trace")
        t = buf.reshape(1024, 16).astype(np.int64)
        G = int((t[:, 0] > 0).sum())
        t = t[:G]
        t0 = t[:, 0].min()
        rel = np.where(t > 0, (t - t0) * 0.01, np.nan)  # us
        print(f"{name}: M={M} K={K} N={N}  {us:.2f} us/launch (events, back to back); {G} workgroups; "
              f"entry spread {np.nanmax(rel[:, 0]):.2f} us; last phase {np.nanmax(rel):.2f} us")
        for i in range(1, 11):
            col = rel[:, i]
            v = col[~np.isnan(col)]
            if len(v) == 0:
                continue
            print(f"   {NAMES[i]:9s} n={len(v):4d}  min {v.min():7.2f}  p50 {np.median(v):7.2f}  "
                  f"max {v.max():7.2f} us")


if __name__ == "__main__":
    main()
