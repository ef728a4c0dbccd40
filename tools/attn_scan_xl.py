#!/usr/bin/env python3
"""Decode attention alone at GPT-2 XL shapes (NH = 25, page 32, ctx 1020),
B = 64: split counts 1-8 x waves 2/4/8 (HIP-event timing of back-to-back
launches, gpt2_decode_time_attention).  B x NH = 1600 (sequence, head)
workgroups are 6.25 per CU; S = 4 makes them a whole 25 per CU.
usage: attn_scan_xl.py [B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pa.init(0)
m = pa.Model(dict(pa.GPT2_XL), seed=1)
m.decode_init(B, 32, 1024)
m.fill_random(1020, seed=3)
m.step(np.zeros(B, np.int32))
auto = m.attn_splits()
for nw in (2, 4, 8):
    pa.check(pa.lib().hpa_set_attention_waves(nw), "waves")
    for s in (1, 2, 3, 4, 8):
        m.set_attn_splits(s)
        ms, by = m.time_attention(24)
        tag = " (engine)" if s == auto and nw == 4 else ""
        print(f"XL B={B} waves={nw} S={s}{tag:9s} {ms * 1e3:8.2f} us {by / ms / 1e6:7.1f} GB/s", flush=True)
pa.check(pa.lib().hpa_set_attention_waves(0), "waves")
m.close()
