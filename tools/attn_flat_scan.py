#!/usr/bin/env python3
"""Decode attention alone at GPT-2 124M shapes (ctx 1020, page 16): the
balanced form (gpt2_decode_set_attn_flat(2): flattened tiles, one workgroup
per CU) against the (sequence, head, range) grid at the engine's split count,
4 and 8 waves, HIP-event timing of back-to-back launches
(gpt2_decode_time_attention).  usage: attn_flat_scan.py [batches...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

batches = [int(x) for x in sys.argv[1:]] or [4, 8, 16, 21, 32]
pa.init(0)
cfg = dict(pa.GPT2_124M)
m = pa.Model(cfg, seed=1)
for B in batches:
    m.decode_init(B, 16, 1024)
    m.fill_random(1020, seed=3)
    m.step(np.zeros(B, np.int32))
    auto = m.attn_flat()
    for flat in (1, 2):
        m.set_attn_flat(flat)
        for nw in ((4, 8) if flat == 1 else (0, 4, 8)):  # balanced, 0: the 16-wave kernel where it fits
            pa.check(pa.lib().hpa_set_attention_waves(nw), "waves")
            ms, by = m.time_attention(48)
            form = "balanced" if flat == 2 else f"grid S={m.attn_splits()}"
            print(f"B={B:3d} {form:10s} waves={nw} {ms * 1e3:7.2f} us {by / ms / 1e6:7.1f} GB/s"
                  f"{'  (engine auto: balanced)' if auto and flat == 2 else ''}", flush=True)
        pa.check(pa.lib().hpa_set_attention_waves(0), "waves")
    m.set_attn_flat(0)
m.close()
