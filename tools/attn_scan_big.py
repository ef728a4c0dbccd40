#!/usr/bin/env python3
"""Attention alone at B = 64 / 128 (124M, page 16, ctx 1024) for split counts 1-4."""
import sys
sys.path.insert(0, "llm.c-paged_amd")
import numpy as np
import pagedattn as pa
pa.init(0)
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in (64, 128):
    m.decode_init(B, 16, 1024)
    m.fill_random(1022, seed=3)
    m.step(np.zeros(B, np.int32))
    for s in (1, 2, 3, 4):
        m.set_attn_splits(s)
        ms, by = m.time_attention(48)
        print(f"B={B} splits={s}: {ms*1e3:8.2f} us {by/ms/1e6:8.1f} GB/s", flush=True)
