#!/usr/bin/env python3
"""Stream-K (variant 6) against the engine's auto launch shape on the GPT-2
layer GEMM shapes: HIP-event timing of back-to-back launches, identical
inputs, max |difference|.  usage: tools/sk_tune.py [C] [B ...]"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pagedattn as pa  # noqa: E402
from gemm_tune import out_copy, shape_inputs, time_fused, dev  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 1600
Bs = [int(x) for x in sys.argv[2:]] or [64]
V = 50257


def main():
    pa.init(0)
    L = pa.lib()
    tot = {}
    for B in Bs:
        shapes = [("qkv", B, C, 3 * C, pa.HPA_FEPI_GELU), ("attproj", B, C, C, pa.HPA_FEPI_RESID),
                  ("fc", B, C, 4 * C, pa.HPA_FEPI_GELU), ("fcproj", B, 4 * C, C, pa.HPA_FEPI_RESID),
                  ("logits", B, C, V, pa.HPA_FEPI_LOGITS)]
        for name, M, K, N, epi in shapes:
            g = shape_inputs(M, K, N, epi, False)
            auto_us = time_fused(g)
            ref = out_copy(g, M, N, epi)
            nf, nc = ctypes.c_size_t(), ctypes.c_size_t()
            pa.check(L.hpa_gemm_sk_workspace(N, ctypes.byref(nf), ctypes.byref(nc)), "ws")
            g.sk_slab = dev(np.zeros(nf.value, np.float32))
            g.sk_count = dev(np.zeros(nc.value, np.int32))
            g.variant = 6
            try:
                sk_us = time_fused(g)
                diff = float(np.abs(out_copy(g, M, N, epi) - ref).max())
            except RuntimeError as e:
                sk_us, diff = float("nan"), str(e)
            fl = 2.0 * M * K * N
            tot.setdefault(B, [0.0, 0.0])
            tot[B][0] += auto_us if name != "logits" else 0
            tot[B][1] += sk_us if name != "logits" else 0
            print(f"B={B:3d} {name:8s} K={K:5d} N={N:6d}  auto {auto_us:8.2f} us ({fl / auto_us / 1e6:6.1f} TF/s)  "
                  f"stream-K {sk_us:8.2f} us ({fl / sk_us / 1e6:6.1f} TF/s)  maxdiff {diff}", flush=True)
        print(f"B={B}: layer GEMMs auto {tot[B][0]:.1f} us, stream-K {tot[B][1]:.1f} us", flush=True)


if __name__ == '__main__':
    main()
