#!/usr/bin/env python3
"""Run ONE fused-GEMM configuration N times (for rocprofv3 --pmc passes).
usage: gemm_one.py shape waves row_blocks variant col_tiles [B] [iters] [C]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
shape, waves, rb, variant, ct = sys.argv[1], *[int(a) for a in sys.argv[2:6]]
B = int(sys.argv[6]) if len(sys.argv) > 6 else 64
iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
C = int(sys.argv[8]) if len(sys.argv) > 8 else 768
sys.argv = [sys.argv[0], str(B), str(C)]
import gemm_tune as gt  # noqa: E402

gt.pa.init(0)
name, M, K, N, epi, ln = {s[0]: s for s in gt.SHAPES}[shape]
g = gt.shape_inputs(M, K, N, epi, ln)
g.waves, g.row_blocks, g.variant, g.col_tiles = waves, rb, variant, ct
for _ in range(iters):
    gt.pa.check(gt.pa.lib().hpa_gemm_fused(ctypes.byref(g)), "gemm")
gt.pa.check(gt.pa.lib().hpa_synchronize())
print("done", shape, waves, rb, variant, ct, B)
