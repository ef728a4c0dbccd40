#!/usr/bin/env python3
"""GPT-2 XL layer GEMMs at B = 64 (C = 1600): the looped kernel with the
engine's launch shape against the loader / MFMA-wave ring kernel (variant 3,
hpa_gemm_ring.hip).  qkv / fc with LayerNorm folded (hpa_ln_fold_pack), as in
the engine; HIP-event timing of back-to-back launches; max |diff| between the
two kernels' outputs; the ring at K parts S = 1..4 (S > 1: two
workgroups per CU, the last part of a column pair sums the parts).  HPA_RING_MODE=1 / 2 (set before the run) times the
ring's no-MFMA / no-DMA diagnostic forms.  usage: ring_tune.py [B] [C]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import pagedattn as pa  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
C = int(sys.argv[2]) if len(sys.argv) > 2 else 1600
rng = np.random.default_rng(0)
keep = []


def dev(a):
    b = pa.DeviceBuffer.from_array(np.ascontiguousarray(a))
    keep.append(b)
    return b.ptr


def inputs(M, K, N, epi, fold):
    L = pa.lib()
    Mp = (M + 15) // 16 * 16
    g = pa.HpaFusedGemm()
    x = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    g.x = dev(pa.to_frag(x))
    g.M, g.K, g.N = M, K, N
    W = rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32)
    bias = rng.uniform(-0.1, 0.1, N).astype(np.float32)
    g.w, g.bias = dev(pa.to_frag(W)), dev(bias)
    if fold:
        g.ln_w = dev(rng.uniform(0.8, 1.2, K).astype(np.float32))
        g.ln_b = dev(rng.uniform(-0.1, 0.1, K).astype(np.float32))
        st = np.zeros((K // 16, Mp, 2), np.float32)
        g.ln_stats, g.ln_ntiles = dev(st), K // 16
        wf = pa.DeviceBuffer(L.hpa_frag_elems(N, K) * 4)
        c1, c2 = pa.DeviceBuffer(N * 4), pa.DeviceBuffer(N * 4)
        keep.extend([wf, c1, c2])
        pa.check(L.hpa_ln_fold_pack(dev(W), N, K, g.ln_w, g.ln_b, g.bias, wf.ptr, c1.ptr, c2.ptr), "fold")
        g.w, g.bias, g.ln_fold_c1 = wf.ptr, c2.ptr, c1.ptr
    g.epilogue = epi
    out = pa.DeviceBuffer(Mp * N * 4)
    keep.append(out)
    g.out = out.ptr
    if epi == pa.HPA_FEPI_RESID:
        g.res_in = dev(rng.uniform(-1, 1, Mp * N).astype(np.float32))
    keep.append(g)
    return g, out, Mp * N


def run(g, iters=50):
    L = pa.lib()
    for _ in range(3):
        pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
    t = pa.Timer()
    t.start()
    for _ in range(iters):
        pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
    return t.stop() * 1000.0 / iters


pa.init(0)
print(f"B={B} C={C} HPA_RING_MODE={os.environ.get('HPA_RING_MODE', '0')} HPA_RING_ROT={os.environ.get('HPA_RING_ROT', '0')}")
tot = [0.0, 0.0]
for name, K, N, epi, fold in (("qkv", C, 3 * C, pa.HPA_FEPI_GELU, True), ("attproj", C, C, pa.HPA_FEPI_RESID, False),
                              ("fc", C, 4 * C, pa.HPA_FEPI_GELU, True), ("fcproj", 4 * C, C, pa.HPA_FEPI_RESID, False)):
    g, out, n = inputs(B, K, N, epi, fold)
    pk = (ctypes.c_int * 3)()
    pa.lib().hpa_fused_pick(B, N, K, ctypes.cast(pk, pa._I))
    g.waves, g.row_blocks, g.col_tiles, g.variant = pk[0], pk[1], pk[2], 1
    t_loop = run(g)
    a = np.empty(n, np.float32)
    pa.check(pa.lib().hpa_memcpy(a.ctypes.data, g.out, a.nbytes))
    g.variant = 3
    line = f"{name:8s} K={K:5d} N={N:5d}  looped {tuple(pk)} {t_loop:7.2f} us  ring"
    best = None
    for parts in (1, 2, 3, 4):
        if parts > 1:
            if (K // 16 + 3) // 4 < parts:
                continue
            nf, nc = ctypes.c_size_t(), ctypes.c_size_t()
            pa.check(pa.lib().hpa_gemm_ring_workspace(N, parts, ctypes.byref(nf), ctypes.byref(nc)), "ws")
            slab = pa.DeviceBuffer(nf.value * 4)
            cnt = pa.DeviceBuffer.from_array(np.zeros(nc.value, np.int32))
            keep.extend([slab, cnt])
            g.sk_slab, g.sk_count = slab.ptr, cnt.ptr
        g.waves = parts
        t = run(g)
        b = np.empty(n, np.float32)
        pa.check(pa.lib().hpa_memcpy(b.ctypes.data, g.out, b.nbytes))
        line += f"  S={parts} {t:6.2f} ({float(np.abs(a - b).max()):.1e})"
        best = t if best is None else min(best, t)
    tot[0] += t_loop
    tot[1] += best
    print(line, flush=True)
print(f"layer GEMMs: looped {tot[0]:.1f} us, ring (best S) {tot[1]:.1f} us")
