#!/usr/bin/env python3
"""Infinity-Cache probe: does reading part of a layer's K/V pool slab just
before its decode attention make the attention faster?  Per batch size, the
attention of layer l timed after hpa_l3_prefetch of the first `frac` of that
layer's slab (per-iteration HIP events; frac 0 = attention alone in the same
form).  GPT-2 124M shapes, page 16, ctx 1020.  usage: l3_probe.py [batches...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

batches = [int(x) for x in sys.argv[1:]] or [64, 8]
pa.init(0)
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in batches:
    m.decode_init(B, 16, 1024)
    m.fill_random(1020, seed=3)
    m.step(np.zeros(B, np.int32))
    kv = 2.0 * B * 1020 * cfg["C"] * 4
    for grid in (1024, 256):
        for frac in (0.0, 0.125, 0.25, 0.375, 0.5, 0.75, 1.0):
            a, p = m.time_attention_pf(frac, 24, grid)
            print(f"B={B:3d} grid={grid:4d} frac={frac:5.3f} attention {a * 1e3:7.2f} us ({kv / a / 1e6:6.0f} GB/s)"
                  f"  prefetch {p * 1e3:7.2f} us", flush=True)
m.close()
