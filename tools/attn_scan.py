#!/usr/bin/env python3
"""Paged decode attention alone vs batch size: GPT-2 124M shapes, synthetic
K/V to ctx, back-to-back launches timed with HIP events
(gpt2_decode_time_attention).  For every B: the engine's split count (auto,
hpa_attn_pick_splits) and the single pass (splits 1), then a splits sweep at
the small batches.  usage: attn_scan.py [ctx]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pa.init(0)
L = pa.lib()
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in (8, 16, 32, 64, 128):
    m.decode_init(B, 16, ctx)
    m.fill_random(ctx - 2, seed=3)
    m.step(np.zeros(B, np.int32))
    auto = m.attn_splits()
    sweep = sorted({1, auto} | ({2, 4, 8, 16} if B <= 32 else set()))
    for s in sweep:
        m.set_attn_splits(s)
        ms, by = m.time_attention(48)
        tag = " (engine)" if s == auto else ""
        print(f"B={B:4d} splits={s:2d}{tag:9s} {ms * 1e3:8.2f} us  {by / ms / 1e6:8.1f} GB/s", flush=True)
