"""Phase timeline of the persistent decode layer (hpa_layer.hip), from the
trace build's per-(layer, workgroup) s_memrealtime stamps.

usage: HPA_LIB=llm.c-paged_amd/libpaged_hip_trace.so python tools/pl_trace.py [B] [ctx] [mode] [XL|b16]
(mode = gpt2_decode_set_layer_kernel: 2 full persistent layer, default; 3
attention launch + persistent chain; 4 wide units; 5 chain form 6; 6 chain
form 8; XL: GPT-2 XL, page 32; b16: the bf16-weight chain, hpa_chain_b16.hip,
at config 5's pool -- maxT 2048, page 8, bf16 KV -- with any nonzero mode)

Prints, per event, the min / median / max over workgroups of the time since
the earliest kernel-start stamp of that layer (us), averaged over layers 1..L-2
of the last step, plus the span of one launch.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "llm.c-paged_amd"), os.path.join(HERE, "..", "tests")]
import pagedattn as hip  # noqa: E402
import synth  # noqa: E402

EVENTS = ["start", "A issued", "A unit done", "A barrier", "B wait done", "B done", "C wait done", "C done",
          "D wait done", "D done", "E wait done", "end",
          # chain form 6 only: stores issued (before the drain) / E folded
          "B stored", "C stored", "D part stored", "E folded"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 990
    mode = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    xl = len(sys.argv) > 4 and sys.argv[4] == "XL"
    b16 = len(sys.argv) > 4 and sys.argv[4] == "b16"
    cfg = dict(maxT=1024, V=50257, L=48, NH=25, C=1600) if xl else dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    if b16:
        cfg["maxT"] = 2048
    hip.init(0)
    m = hip.Model(cfg, params=hip.synthetic_params(cfg, seed=3) if xl or b16 else synth.params(cfg, seed=3))
    if b16:
        m.decode_init(B, 8, cfg["maxT"], kv_dtype=hip.HPA_BF16, w_dtype=hip.HPA_BF16)
    else:
        m.decode_init(B, 32 if xl else 16, cfg["maxT"])
    assert m.set_layer_kernel(mode), "persistent layer not in use"
    m.set_graph(True)
    hip.check(hip.lib().gpt2_decode_fill_random(m.h, ctx, 5), "fill")
    toks = np.random.default_rng(1).integers(0, cfg["V"], B).astype(np.int32)
    for _ in range(8):
        m.step(toks)
    L = hip.lib()
    read = L.hpa_decode_chain_b16_trace if b16 else L.hpa_decode_layer_trace
    if read(None, 0) != 0:
        raise SystemExit("not a trace build (make XFLAGS=-DHPA_LAYER_TRACE)")
    m.step(toks)
    m.status()
    buf = np.zeros((cfg["L"], 256, 16), np.uint64)  # 16 event slots per (layer, workgroup)
    hip.check(read(buf.ctypes.data_as(ctypes.c_void_p), cfg["L"]), "trace")
    rows = {k: [] for k in range(len(EVENTS))}
    spans = []
    for layer in range(1, cfg["L"] - 1):
        t = buf[layer].astype(np.int64)
        t0 = t[:, 0][t[:, 0] > 0].min()
        spans.append((t[:, 11][t[:, 11] > 0].max() - t0) / 100.0)
        for k in range(len(EVENTS)):
            v = t[:, k]
            v = v[v > 0]
            if len(v):
                rows[k].append(((v - t0) / 100.0))
    print(f"B={B} ctx={ctx} mode={mode}: launch span (first start -> last end) {np.mean(spans):.1f} us "
          f"(layers 1..{cfg['L'] - 2}, last step)")
    print(f"{'event':14s} {'n':>4s} {'min':>7s} {'med':>7s} {'max':>7s}  us")
    for k, name in enumerate(EVENTS):
        if not rows[k]:
            continue
        n = int(np.mean([len(r) for r in rows[k]]))
        mn = np.mean([r.min() for r in rows[k]])
        md = np.mean([np.median(r) for r in rows[k]])
        mx = np.mean([r.max() for r in rows[k]])
        print(f"{name:14s} {n:4d} {mn:7.2f} {md:7.2f} {mx:7.2f}")
    if len(sys.argv) > 5:  # "active N": also over workgroups 0..N-1 only (the units of a phase at one row block)
        na = int(sys.argv[6]) if len(sys.argv) > 6 else 48
        print(f"-- workgroups 0..{na - 1} only")
        for k, name in enumerate(EVENTS):
            vals = []
            for layer in range(1, cfg["L"] - 1):
                t = buf[layer].astype(np.int64)
                t0 = t[:, 0][t[:, 0] > 0].min()
                v = t[:na, k]
                v = v[v > 0]
                if len(v):
                    vals.append((v - t0) / 100.0)
            if vals:
                print(f"{name:14s} {na:4d} {np.mean([r.min() for r in vals]):7.2f} "
                      f"{np.mean([np.median(r) for r in vals]):7.2f} {np.mean([r.max() for r in vals]):7.2f}")
    m.close()


if __name__ == "__main__":
    main()
