"""Probe: does one half of the batch's attention overlap the other half's
GEMM chain when the two halves run as two engines on two HIP streams?

usage: python tools/overlap_probe.py [B] [ctx] [layer_form] [steps]

Times, at GPT-2 124M and the same synthetic KV fill:
  one   - one engine of B rows (the bench's configuration)
  serial- two engines of B/2 rows on ONE stream (no overlap possible)
  two   - two engines of B/2 rows on TWO streams (overlap if the hardware
          runs the two queues' kernels side by side)
and checks that the two-stream tokens equal the serial ones.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "llm.c-paged_amd")]
import pagedattn as hip  # noqa: E402

CFG = dict(maxT=1024, V=50257, L=12, NH=12, C=768)


def engine(B, ctx, form, offset):
    m = hip.Model(CFG, seed=1337)
    m.decode_init(B, 16, CFG["maxT"])
    m.set_layer_kernel(form)
    m.reserve(ctx + 64)
    hip.check(hip.lib().gpt2_decode_fill_random_ex(m.h, ctx, 77, offset), "fill")
    return m


def run(models, streams, steps, first):
    L = hip.lib()
    for m, s, f in zip(models, streams, first):  # capture + warm
        L.hpa_set_stream(s)
        m.set_graph(True)
        m.step_async(f)
    for _ in range(4):
        for m, s in zip(models, streams):
            L.hpa_set_stream(s)
            m.step_async(None)
    hip.check(L.hpa_device_synchronize(), "sync")
    t0 = time.perf_counter()
    for _ in range(steps):
        for m, s in zip(models, streams):
            L.hpa_set_stream(s)
            m.step_async(None)
    hip.check(L.hpa_device_synchronize(), "sync")
    ms = (time.perf_counter() - t0) * 1e3 / steps
    toks = []
    for m, s in zip(models, streams):
        L.hpa_set_stream(s)
        out = np.zeros(m.B, np.int32)
        hip.check(L.hpa_memcpy(out.ctypes.data, m.next_ptr(), out.nbytes), "next")
        toks.append(out)
    L.hpa_set_stream(None)
    return ms, np.concatenate(toks)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ctx = int(sys.argv[2]) if len(sys.argv) > 2 else 960
    form = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    hip.init(0)
    L = hip.lib()
    first = np.random.default_rng(1).integers(0, CFG["V"], B).astype(np.int32)
    h = B // 2
    res = {}
    m1 = engine(B, ctx, form, 0)
    res["one"] = run([m1], [L.hpa_get_stream()], steps, [first])
    m1.close()
    ms = [engine(h, ctx, form, 0), engine(h, ctx, form, h)]
    s0 = L.hpa_get_stream()
    res["serial"] = run(ms, [s0, s0], steps, [first[:h], first[h:]])
    for m in ms:
        m.close()
    ms = [engine(h, ctx, form, 0), engine(h, ctx, form, h)]
    s1 = L.hpa_stream_create()
    res["two"] = run(ms, [s0, s1], steps, [first[:h], first[h:]])
    for m in ms:
        m.close()
    for k, (t, _) in res.items():
        print(f"{k:7s} B={B} ctx={ctx} form={form}: {t:.4f} ms/step  {B / t * 1e3:.0f} tok/s")
    same = np.array_equal(res["two"][1], res["serial"][1])
    agree = float(np.mean(res["two"][1] == res["one"][1]))
    print(f"two-stream tokens == serial: {same}; agreement with one engine {agree:.3f}")
    if not same:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
