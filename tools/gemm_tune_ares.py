#!/usr/bin/env python3
"""fp32 A-resident GEMM (variant 5, hpa_gemm_ares.hip) against the fp32
default launch on the GPT-2 decode shapes: every (waves, row blocks, rounds),
outputs checked equal across A-resident shapes (one k chain per wave).
Usage: tools/gemm_tune_ares.py [B] [C]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import gemm_tune as gt  # noqa: E402

pa = gt.pa


def main():
    pa.init(0)
    print(f"fp32 A-resident  B={gt.B} C={gt.C}")
    tot_def = tot_best = 0.0
    for name, M, K, N, epi, ln in gt.SHAPES:
        if K > 1600:
            continue
        g = gt.shape_inputs(M, K, N, epi, ln)
        g.waves = g.row_blocks = g.col_tiles = 0
        g.variant = 4 if epi == pa.HPA_FEPI_LOGITS else 0
        dflt = gt.time_fused(g)
        res, ref = [], None
        for waves in (4, 8):
            for rb in (1, 2):
                if rb == 2 and (K > 768 or ((M + 15) // 16) % 2):
                    continue
                for rounds in (1, 2, 4, 8):
                    g.variant, g.waves, g.row_blocks, g.col_tiles = 5, waves, rb, rounds
                    try:
                        us = gt.time_fused(g)
                    except RuntimeError:
                        continue
                    o = gt.out_copy(g, M, N, epi)
                    ref = o if ref is None else ref
                    res.append((us, (waves, rb, rounds), float(np.abs(o - ref).max())))
        best = min(res)
        tot_def += dflt
        tot_best += min(best[0], dflt)
        print(f"{name:8s} M={M} K={K} N={N}  fp32 default {dflt:8.2f} us")
        for us, shp, err in sorted(res)[:6]:
            print(f"   {us:8.2f} us  (waves, rb, rounds)={shp}  {2.0 * M * K * N / us / 1e6:7.1f} TF/s  "
                  f"maxdiff={err:.2e}")
    print(f"sum: default {tot_def:.1f} us  with A-resident where faster {tot_best:.1f} us")


if __name__ == '__main__':
    main()
