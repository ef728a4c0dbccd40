#!/usr/bin/env python3
"""Launch-shape sweep of the bf16-weight fused GEMM (w_dtype = HPA_BF16,
hpa_gemm_bf16.hip) on the GPT-2 decode shapes at a given batch, next to the
fp32 kernel's default shape; outputs checked equal across shapes (a row's sum
depends on the waves only).
Usage: tools/gemm_tune_bf16.py [B] [C]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import gemm_tune as gt  # noqa: E402  (its B, C come from the same argv)

pa = gt.pa


def main():
    pa.init(0)
    L = pa.lib()
    print(f"bf16 weights  B={gt.B} C={gt.C}")
    tot_best = tot_auto = tot_f32 = 0.0
    for name, M, K, N, epi, ln in gt.SHAPES:
        g = gt.shape_inputs(M, K, N, epi, ln)
        g.waves = g.row_blocks = g.col_tiles = g.variant = 0
        f32 = gt.time_fused(g)
        wb = pa.DeviceBuffer(L.hpa_frag_bf16_elems(N, K) * 2)
        gt.keep.append(wb)
        W = np.random.default_rng(1).uniform(-0.05, 0.05, (N, K)).astype(np.float32)
        pa.check(L.hpa_pack_frag_bf16(gt.dev(W), N, K, K, wb.ptr), "pack")
        g.w, g.w_dtype = wb.ptr, pa.HPA_BF16
        res, ref = [], {}
        shapes = [(1, w_, rb, ct) for w_ in (4, 8) for rb, ct in ((1, 1), (2, 1), (4, 1), (2, 2), (4, 2))]
        shapes += [(5, w_, rb, r) for w_ in (4, 8) for rb in (1, 2, 4) for r in (1, 2, 4, 8)
                   if rb * K <= 3200 and not (rb == 4 and K > 768)]
        for variant, waves, rb, ct in shapes:
            if ((M + 15) // 16) % rb:
                continue
            g.variant, g.waves, g.row_blocks, g.col_tiles = variant, waves, rb, ct
            try:
                us = gt.time_fused(g)
            except RuntimeError:
                continue
            o = gt.out_copy(g, M, N, epi)
            key = (variant, waves)
            ref.setdefault(key, o)
            res.append((us, (variant, waves, rb, ct), float(np.abs(o - ref[key]).max())))
        g.variant = g.waves = g.row_blocks = g.col_tiles = 0
        auto_us = gt.time_fused(g)
        best = min(res)
        tot_best += best[0]
        tot_auto += auto_us
        tot_f32 += f32
        print(f"{name:8s} M={M} K={K} N={N}  fp32 default {f32:8.2f} us   bf16 auto {auto_us:8.2f} us")
        for us, shp, err in sorted(res):
            print(f"   {us:8.2f} us  (variant, waves, rb, ct|rounds)={shp}  {2.0 * M * K * N / us / 1e6:7.1f} TF/s  "
                  f"{2.0 * N * K / us / 1e3:7.1f} GB/s(W)  maxdiff={err:.2e}")
    print(f"sum: fp32 default {tot_f32:.1f} us  bf16 best {tot_best:.1f} us  bf16 auto {tot_auto:.1f} us")


if __name__ == '__main__':
    main()
