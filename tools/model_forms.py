#!/usr/bin/env python3
"""Decode step time of a GPT-2 size on the engine's auto layer form vs five
launches per layer (graph replay, synthetic weights and K/V at ctx ~1000).
usage: model_forms.py medium|large|xl|124M [B]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import numpy as np  # noqa: E402
import pagedattn as pa  # noqa: E402

SIZES = {"124M": dict(L=12, NH=12, C=768), "medium": dict(L=24, NH=16, C=1024),
         "large": dict(L=36, NH=20, C=1280), "xl": dict(L=48, NH=25, C=1600)}
name = sys.argv[1] if len(sys.argv) > 1 else "medium"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = dict(maxT=1024, V=50257, **SIZES[name])
pa.init(0)
m = pa.Model(cfg, seed=1)
steps, ctx = 20, 1000
for mode in (1, 0, 1):
    m.decode_init(B, 32 if name == "xl" else 16, 1024)
    m.set_layer_kernel(mode)
    form = m.layer_form()
    m.set_graph(True)
    m.fill_random(ctx, seed=3)
    m.step(np.zeros(B, np.int32))
    for _ in range(3):
        m.step_async(None)
    pa.check(pa.lib().hpa_device_synchronize(), "sync")
    m.set_positions(np.full(B, ctx, np.int32))
    pa.check(pa.lib().hpa_device_synchronize(), "sync")
    t0 = time.perf_counter()
    for _ in range(steps):
        m.step_async(None)
    pa.check(pa.lib().hpa_device_synchronize(), "sync")
    ms = (time.perf_counter() - t0) * 1e3 / steps
    m.status()
    print(f"GPT-2 {name} B={B}: layer_kernel {mode} (form {form}) {ms:.3f} ms/step {B / ms * 1e3:.0f} tok/s",
          flush=True)
m.close()
