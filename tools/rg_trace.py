#!/usr/bin/env python3
"""Per-workgroup timeline of the ring logits kernel (hpa_logits.hip) from the
trace build's stamps (make XFLAGS=-DHPA_RG_TRACE): iteration starts, the
shader clock (s_memtime over s_memrealtime), and per-iteration averages of
the loader's vmcnt wait, wave 0's barrier wait and the compute sections.
usage: HPA_LIB=<trace build .so> python tools/rg_trace.py [B] [iters]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sys.argv = [sys.argv[0], str(B), "768"]
import gemm_tune as gt  # noqa: E402

gt.pa.init(0)
L = gt.pa.lib()
name, M, K, N, epi, ln = {s[0]: s for s in gt.SHAPES}["logits"]
g = gt.shape_inputs(M, K, N, epi, ln)
g.variant = 4
for _ in range(iters):
    gt.pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
gt.pa.check(L.hpa_synchronize())
buf2 = np.zeros((2, 256, 24), np.uint64)
if L.hpa_logits_trace(buf2.ctypes.data_as(ctypes.c_void_p)) != 0:
    raise SystemExit("not a trace build")
t = buf2[0].astype(np.int64)
live = t[:, 0] > 0
t = t[live]
clk = buf2[1].astype(np.int64)[live]
t0 = t[:, 0].min()
us = (t[:, :18] - t0) / 100.0
print(f"B={B}: {live.sum()} workgroups; span {us[:, 17].max():.2f} us")
for k, nm in [(0, "start"), (1, "prologue done")] + [(2 + i, f"iter {i}") for i in range(14)] + [(16, "loop end"),
                                                                                                   (17, "end")]:
    v = us[:, k][t[:, k] > 0]
    if len(v):
        print(f"{nm:14s} n={len(v):4d} min {v.min():7.2f} med {np.median(v):7.2f} max {v.max():7.2f}")
d = np.diff(us[:, 2:14], axis=1)
dc = np.diff(clk[:, 2:14], axis=1)
print(f"iteration length (iters 1..11): med {np.median(d):.3f} us, mean {d.mean():.3f}; "
      f"shader clock {np.median(dc / d):.0f} MHz (median)")
nit = np.where(t[:, 2:16] > 0, 1, 0).sum(1)  # iterations stamped (<= 14) -- use the loop count instead
n_iter = np.where(us[:, 16] > 0, 0, 0) + 12.27
for k, nm in [(18, "loader vmcnt wait"), (19, "wave0 barrier wait"), (20, "wave0 compute"), (21, "loader DMA issue")]:
    v = t[:, k] / 100.0 / n_iter
    print(f"{nm:20s} per iteration: med {np.median(v):.3f} us")
