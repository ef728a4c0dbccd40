"""Timeline of the pipelined halves (hpa_pipe.hip) from the trace build's
per-(layer, half, workgroup) s_memrealtime stamps.

usage: HPA_LIB=llm.c-paged_amd/libpl_pt.so python tools/pipe_trace.py [B] [ctx] [g_cus]
  (the library: make -C llm.c-paged_amd BUILD=build_pt LIB=libpl_pt.so XFLAGS=-DHPA_PIPE_TRACE)

Prints, for every (layer, half) of the last step, the A role's attention
window (first wait done .. last unit done over the A workgroups) and the G
role's phases (max over G workgroups of each phase's wait-done and done),
in us since the launch's first stamp.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "llm.c-paged_amd"), os.path.join(HERE, "..", "tests")]
import pagedattn as hip  # noqa: E402
import synth  # noqa: E402

G_EV = ["B wait", "B done", "C wait", "C done", "D wait", "D done", "E wait", "E done"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 990
    g_cus = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cfg = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    hip.init(0)
    m = hip.Model(cfg, params=synth.params(cfg, seed=3))
    m.decode_init(B, 16, cfg["maxT"])
    assert m.set_layer_kernel(7) and m.layer_form() == 5, "pipelined halves not in use"
    if g_cus:
        m.set_pipe_split(g_cus)
    m.set_graph(True)
    hip.check(hip.lib().gpt2_decode_fill_random(m.h, ctx, 5), "fill")
    toks = np.random.default_rng(1).integers(0, cfg["V"], B).astype(np.int32)
    L = hip.lib()
    L.hpa_decode_pipe_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for _ in range(8):
        m.step(toks)
    if L.hpa_decode_pipe_trace(None, 0) != 0:
        raise SystemExit("not a trace build (XFLAGS=-DHPA_PIPE_TRACE)")
    m.step(toks)
    m.status()
    nl = cfg["L"]
    buf = np.zeros((2 * nl, 256, 12), np.uint64)
    hip.check(L.hpa_decode_pipe_trace(buf.ctypes.data_as(ctypes.c_void_p), nl), "trace")
    t = buf.astype(np.int64)
    ng = g_cus or 64
    t0 = t[0, :, 10][t[0, :, 10] > 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    print(f"B={B} ctx={ctx} G CUs={ng}: launch span {us(t[..., :10][t[..., :10] > 0].max()):.1f} us")
    print(f"{'l h':5s} {'A start':>8s} {'A end':>8s} {'A med':>8s} | " + " ".join(f"{e:>7s}" for e in G_EV))
    for lh in range(2 * nl):
        a_w = t[lh, ng:, 0]
        a_d = t[lh, ng:, 1]
        a_w, a_d = a_w[a_w > 0], a_d[a_d > 0]
        row = f"{lh // 2:2d} {lh % 2} {us(a_w.min()):8.1f} {us(a_d.max()):8.1f} {us(np.median(a_d)):8.1f} |"
        for k in range(2, 10):
            v = t[lh, :ng, k]
            v = v[v > 0]
            row += f" {us(v.max()):7.1f}" if len(v) else "       -"
        print(row)
    m.close()


if __name__ == "__main__":
    main()
