#!/usr/bin/env python3
"""Microbenchmark of the bf16-weight logits GEMM (BASELINE config 5: M = 256,
N = 50257, K = 768, LNf on the operand path, argmax partials) in isolation:
every launch shape of the bf16 kernels (variant 0 looped, variant 5
A-resident), HIP-event timing per launch with the weights either L2/MALL-warm
(back to back) or cold (a 512 MiB buffer read between launches, as in the
decode step where the last attention streams the K/V cache before the
logits).  Outputs checked equal within bf16-operand rounding across shapes.
usage: tools/b16_logits.py [M] [iters] [variant waves row_blocks]  (the last three: one shape only, e.g.
for rocprofv3 --pmc passes)"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
import pagedattn as pa  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
K, N = 768, 50257
rng = np.random.default_rng(0)
keep = []


def dev(a):
    b = pa.DeviceBuffer.from_array(np.ascontiguousarray(a))
    keep.append(b)
    return b.ptr


def main():
    pa.init(0)
    L = pa.lib()
    Mp = (M + 15) // 16 * 16
    g = pa.HpaFusedGemm()
    g.x = dev(pa.to_frag(rng.uniform(-1, 1, (M, K)).astype(np.float32)))
    g.M, g.K, g.N = M, K, N
    w32 = dev(rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32))
    nb = int(L.hpa_frag_bf16_elems(N, K)) * 2
    wb = pa.DeviceBuffer(nb)
    keep.append(wb)
    pa.check(L.hpa_pack_frag_bf16(w32, N, K, K, wb.ptr), "pack")
    g.w = wb.ptr
    g.w_dtype = pa.HPA_BF16
    st = np.zeros((K // 16, Mp, 2), np.float32)
    st[:, :M, 0] = 1.0
    st[:, :M, 1] = 20.0
    g.ln_stats = dev(st)
    g.ln_ntiles = K // 16
    g.ln_w = dev(np.ones(K, np.float32))
    g.ln_b = dev(np.zeros(K, np.float32))
    g.epilogue = pa.HPA_FEPI_LOGITS
    g.out = dev(np.zeros(M * N, np.float32))
    g.part_out = dev(np.zeros(((N + 15) // 16) * Mp * 2, np.float32))
    flush = pa.DeviceBuffer(512 << 20)
    keep.append(flush)
    pk = (ctypes.c_int * 3)()
    L.hpa_fused_pick_bf16(M, N, K, ctypes.cast(pk, pa._I))
    pa5 = (ctypes.c_int * 3)()
    ares = L.hpa_fused_pick_bf16_ares(M, N, K, ctypes.cast(pa5, pa._I))
    print(f"M={M} N={N} K={K}: pick variant {'5 (ares) ' + str(list(pa5)) if ares else '0 ' + str(list(pk))}")
    ev0, ev1 = L.hpa_event_create(), L.hpa_event_create()

    def run(cold):
        ts = []
        for _ in range(ITERS):
            if cold:
                pa.check(L.hpa_l3_prefetch(flush.ptr, ctypes.c_size_t(512 << 20), 1024), "flush")
            L.hpa_event_record(ev0)
            pa.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm")
            L.hpa_event_record(ev1)
            ts.append(L.hpa_event_elapsed_ms(ev0, ev1) * 1000.0)
        return float(np.median(ts))

    ref = None
    shapes = [(5, w, rb, rd) for w in (4, 8) for rb in (1, 2, 4) for rd in (0,)]
    shapes += [(0, w, rb, ct) for w in (4, 8) for rb in (1, 2, 4) for ct in (1, 2) if (rb, ct) != (1, 2)]
    if len(sys.argv) > 5:
        shapes = [(int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), 0)]
    for variant, waves, rb, ct in shapes:
        if (Mp // 16) % rb:
            continue
        g.variant, g.waves, g.row_blocks, g.col_tiles = variant, waves, rb, ct
        try:
            warm = run(False)
            cold = run(True)
        except RuntimeError as e:
            print(f"variant {variant} waves {waves} rb {rb} ct/rounds {ct}: {e}")
            continue
        o = np.empty(M * N, np.float32)
        pa.check(L.hpa_memcpy(o.ctypes.data, g.out, o.nbytes))
        if ref is None:
            ref = o
        d = float(np.abs(o - ref).max())
        print(f"variant {variant} waves {waves} rb {rb} ct/rounds {ct}: warm {warm:7.2f} us  cold {cold:7.2f} us  "
              f"max|d| {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
