#!/usr/bin/env python3
"""Decode attention alone vs batch and split count at GPT-2 124M shapes (ctx
1020, page 16): HIP-event timing of back-to-back launches
(gpt2_decode_time_attention), the split kernel with its in-kernel merge,
S = 1, 2, 4, 8, and the engine's pick marked; then 8 waves per workgroup
(hpa_set_attention_waves) at the small batches.  usage: attn_scan_r3.py [batches...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

batches = [int(x) for x in sys.argv[1:]] or [8, 16, 32, 64]
pa.init(0)
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in batches:
    m.decode_init(B, 16, 1024)
    m.fill_random(1020, seed=3)
    m.step(np.zeros(B, np.int32))
    auto = m.attn_splits()
    for nw in ((4, 8) if B <= 32 else (4,)):
        pa.check(pa.lib().hpa_set_attention_waves(nw), "waves")
        for s in (1, 2, 4, 8):
            m.set_attn_splits(s)
            ms, by = m.time_attention(48)
            tag = " (engine)" if s == auto and nw == pa.lib().hpa_attn_pick_waves(B, cfg["NH"], s, 0) else ""
            print(f"B={B:3d} waves={nw} S={s}{tag:9s} {ms * 1e3:7.2f} us {by / ms / 1e6:7.1f} GB/s", flush=True)
    pa.check(pa.lib().hpa_set_attention_waves(0), "waves")  # back to the engine's pick
m.close()
