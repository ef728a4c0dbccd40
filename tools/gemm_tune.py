#!/usr/bin/env python3
"""Microbenchmark of the fused decode GEMM (hpa_gemm_fused) on the GPT-2
shapes at a given batch: every (waves, row blocks) per workgroup, HIP-event timing
on the library stream, outputs checked equal-within-fp32 across settings.
Usage: tools/gemm_tune.py [B] [C]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import pagedattn as pa  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
C = int(sys.argv[2]) if len(sys.argv) > 2 else 768
V = 50257
rng = np.random.default_rng(0)
keep = []


def dev(a):
    b = pa.DeviceBuffer.from_array(np.ascontiguousarray(a))
    keep.append(b)
    return b.ptr


def shape_inputs(M, K, N, epi, ln):
    Mp = (M + 15) // 16 * 16
    g = pa.HpaFusedGemm()
    g.x = dev(pa.to_frag(rng.uniform(-1, 1, (M, K)).astype(np.float32)))
    g.M, g.K, g.N = M, K, N
    g.w = dev(pa.to_frag(rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32)))
    if ln:
        st = np.zeros((K // 16, Mp, 2), np.float32)
        st[:, :M, 0] = 1.0
        st[:, :M, 1] = 20.0
        g.ln_stats = dev(st)
        g.ln_ntiles = K // 16
        g.ln_w = dev(np.ones(K, np.float32))
        g.ln_b = dev(np.zeros(K, np.float32))
    if epi != pa.HPA_FEPI_LOGITS:
        g.bias = dev(rng.uniform(-0.1, 0.1, N).astype(np.float32))
    g.epilogue = epi
    if epi == pa.HPA_FEPI_RESID:
        g.res_in = dev(np.zeros(Mp * N, np.float32))
        g.out = dev(np.zeros(Mp * N, np.float32))
        g.stats_out = dev(np.zeros((N // 16) * Mp * 2, np.float32))
    elif epi == pa.HPA_FEPI_GELU:
        g.out = dev(np.zeros(Mp * N, np.float32))
    else:
        g.out = dev(np.zeros(M * N, np.float32))
        g.part_out = dev(np.zeros(((N + 15) // 16) * Mp * 2, np.float32))
    return g


def out_copy(g, M, N, epi):
    n = M * N if epi == pa.HPA_FEPI_LOGITS else ((M + 15) // 16 * 16) * N
    a = np.empty(n, np.float32)
    pa.check(pa.lib().hpa_memcpy(a.ctypes.data, g.out, a.nbytes))
    return a


def time_fused(g, iters=50):
    L = pa.lib()
    for _ in range(3):
        pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
    t = pa.Timer()
    t.start()
    for _ in range(iters):
        pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
    return t.stop() * 1000.0 / iters


SHAPES = [("qkv", B, C, 3 * C, pa.HPA_FEPI_GELU, True), ("attproj", B, C, C, pa.HPA_FEPI_RESID, False),
          ("fc", B, C, 4 * C, pa.HPA_FEPI_GELU, True), ("fcproj", B, 4 * C, C, pa.HPA_FEPI_RESID, False),
          ("logits", B, C, V, pa.HPA_FEPI_LOGITS, True)]


ONESHOT = {(4, 48), (8, 48), (16, 48), (8, 192), (16, 192), (10, 100)}  # hpa_fused.hip launch_os instances


def main():
    pa.init(0)
    L = pa.lib()
    print(f"B={B} C={C}")
    total_best = total_auto = 0.0
    for name, M, K, N, epi, ln in SHAPES:
        g = shape_inputs(M, K, N, epi, ln)
        pk = (ctypes.c_int * 3)()
        L.hpa_fused_pick(M, N, K, ctypes.cast(pk, pa._I))
        rb_eff = pk[1]
        while ((M + 15) // 16) % rb_eff:
            rb_eff //= 2
        oneshot = rb_eff == 1 and (N + 15) // 16 < 1024 and (pk[0], K // 16) in ONESHOT and pk[2] <= 1
        auto = (pk[0], rb_eff, 2 if oneshot else 1, pk[2])
        res = []
        ref = None
        for waves in (4, 8, 10, 16):
            for rb in (1, 2, 4):
                for variant in (1, 2, 3, 4):
                    for ct in (1, 2, 4):
                        if ((M + 15) // 16) % rb or (variant == 2 and (rb != 1 or ct != 1)):
                            continue
                        if variant == 3 and (waves == 16 or ct == 4):  # deep = looped there
                            continue
                        if variant == 4 and (epi != pa.HPA_FEPI_LOGITS or (waves, rb, ct) != (4, 1, 1)):
                            continue  # resident logits kernel: one launch shape
                        if ct > 1 and (waves == 16 or rb == 1 or (ct == 4 and (rb != 4 or waves != 4))):
                            continue
                        g.waves, g.row_blocks, g.variant, g.col_tiles = waves, rb, variant, ct
                        try:
                            us = time_fused(g)
                        except RuntimeError:
                            continue
                        o = out_copy(g, M, N, epi)
                        if ref is None:
                            ref = o
                        res.append((us, (waves, rb, variant, ct), float(np.abs(o - ref).max())))
        flops = 2.0 * M * K * N
        wbytes = 4.0 * N * K
        best = min(res)
        total_best += best[0]
        total_auto += ([r for r in res if r[1] == auto] or [best])[0][0]
        print(f"{name:8s} M={M} K={K} N={N} auto (waves, row_blocks, variant, col_tiles)={auto}")
        for us, waves, err in sorted(res):
            print(f"   {us:8.2f} us  (waves, rb, variant, ct)={waves}  {flops / us / 1e6:7.1f} TF/s "
                  f"{wbytes / us / 1e3:7.1f} GB/s(W)  maxdiff={err:.2e}")
    print(f"sum best {total_best:.1f} us   sum auto {total_auto:.1f} us")


if __name__ == '__main__':
    main()
