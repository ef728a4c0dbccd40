#!/usr/bin/env python3
"""Decode attention alone at small batches, every split count 1..8 with 4
and 8 waves (GPT-2 124M shapes, ctx 1020, page 16; HIP-event timing of
back-to-back launches).  usage: attn_scan_s3.py [batches...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

batches = [int(x) for x in sys.argv[1:]] or [8, 16]
pa.init(0)
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in batches:
    m.decode_init(B, 16, 1024)
    m.fill_random(1020, seed=3)
    m.step(np.zeros(B, np.int32))
    auto = m.attn_splits()
    for nw in (4, 8):
        pa.check(pa.lib().hpa_set_attention_waves(nw), "waves")
        for s in range(1, 9):
            m.set_attn_splits(s)
            ms, by = m.time_attention(48)
            tag = " (engine)" if s == auto and nw == pa.lib().hpa_attn_pick_waves(B, cfg["NH"], s, 0) else ""
            print(f"B={B:3d} waves={nw} S={s}{tag:9s} {ms * 1e3:7.2f} us {by / ms / 1e6:7.1f} GB/s", flush=True)
    pa.check(pa.lib().hpa_set_attention_waves(0), "waves")
m.close()
