"""Per-wave timeline of chain form 8's fc phase (GPT-2 XL, layer 5) from the
trace build's s_memtime stamps (hpa_decode_cx_wave_trace): for each wave, the
shader cycles from its A loads' issue to each half-tile's MFMAs issued.
Prints the median / max over the waves of all workgroups holding an fc unit
of the per-half-tile increments, against the MFMA issue a half-tile needs
(5 k16 steps x 4 MFMAs of 32 cycles, x 3 waves sharing a SIMD).

usage: HPA_LIB=llm.c-paged_amd/libpaged_hip_trace.so python tools/cx_wave_trace.py [B] [ctx]
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "llm.c-paged_amd")]
import pagedattn as hip  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    cfg = dict(maxT=1024, V=50257, L=48, NH=25, C=1600)
    hip.init(0)
    m = hip.Model(cfg, params=hip.synthetic_params(cfg, seed=3))
    m.decode_init(B, 32, ctx + 16)
    assert m.set_layer_kernel(6), "chain form 8 not in use"
    m.set_graph(True)
    m.fill_random(ctx, seed=5)
    toks = np.random.default_rng(1).integers(0, cfg["V"], B).astype(np.int32)
    for _ in range(3):
        m.step(toks)
    L = hip.lib()
    if L.hpa_decode_cx_wave_trace(None) != 0:
        raise SystemExit("not a trace build (make XFLAGS=-DHPA_LAYER_TRACE)")
    m.step(toks)
    m.status()
    buf = np.zeros((256, 12, 16), np.uint64)
    hip.check(L.hpa_decode_cx_wave_trace(buf.ctypes.data_as(ctypes.c_void_p)), "trace")
    t = buf.astype(np.int64)
    live = (t[:, :, 0] > 0) & (t[:, :, 15] > 0)
    n = int(live.sum())
    print(f"XL B={B} ctx={ctx}: fc phase of layer 5, {n} waves with stamps")
    w = t[live]
    base = w[:, 0:1]
    nq = int(((w[:, 1:15] > 0).sum(axis=1)).max())
    rel = np.where(w[:, 1:1 + nq] > 0, w[:, 1:1 + nq] - base, -1)
    prev = np.concatenate([np.zeros((rel.shape[0], 1), np.int64), rel[:, :-1]], axis=1)
    inc = np.where(rel > 0, rel - prev, -1)
    print("half-tile  cycles since A issue (median / max)   increment (median / max)")
    for q in range(nq):
        c = rel[:, q][rel[:, q] > 0]
        d = inc[:, q][inc[:, q] > 0]
        if len(c):
            print(f"{q:9d}  {int(np.median(c)):10d} / {int(c.max()):8d}        {int(np.median(d)):8d} / {int(d.max()):8d}")
    tot = (w[:, 15] - w[:, 0])
    print(f"loop total: median {int(np.median(tot))} cycles, max {int(tot.max())}; "
          f"MFMA issue per half-tile per SIMD (3 waves): {5 * 4 * 32 * 3} cycles")
    m.close()


if __name__ == "__main__":
    main()
