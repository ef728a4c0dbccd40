#!/usr/bin/env python3
"""Attention alone vs waves per workgroup and split count at the XL (page 32)
and 124M (page 16) B = 64 shapes (HIP-event timing of back-to-back launches)."""
import os, sys
sys.path.insert(0, "llm.c-paged_amd")
import numpy as np
import pagedattn as pa
pa.init(0)
L = pa.lib()
for name, cfg, P, B in (("XL", dict(pa.GPT2_XL), 32, 64), ("124M", dict(pa.GPT2_124M), 16, 64)):
    m = pa.Model(cfg, seed=1)
    m.decode_init(B, P, 1024)
    m.fill_random(1022, seed=3)
    m.step(np.zeros(B, np.int32))
    for waves in (2, 4, 8):
        pa.check(L.hpa_set_attention_waves(waves), "waves")
        for s in (1, 2):
            m.set_attn_splits(s)
            ms, by = m.time_attention(48)
            print(f"{name} B={B} page {P} waves={waves} splits={s}: {ms*1e3:8.2f} us {by/ms/1e6:8.1f} GB/s", flush=True)
    pa.check(L.hpa_set_attention_waves(0), "waves")  # back to the callers' choice
    m.close()
