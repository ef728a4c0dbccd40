"""The fused decode-layer GEMM (hpa_gemm_fused) and frag-layout helpers vs
float64 numpy references of the same ops, each epilogue, at every
waves-per-workgroup setting (the K range split over 4/8/16 waves and folded
in LDS).

Tolerance: |gpu - f64| <= 4e-6 * sum_k |a||w| + 2e-6 (fp32 MFMA chains; the
LayerNorm on the A operand uses one-pass statistics, so LN'ed cases compare
against the f64 LN of the same inputs).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gelu_tanh(a):
    """the reference's tanh GELU (paged_infer.c gelu_forward) in float64; numpy
    rather than torch: torch's bundled HIP runtime beside the library's
    /opt/rocm one aborts the process at exit (double free)"""
    a = np.asarray(a, np.float64)
    return 0.5 * a * (1 + np.tanh(np.sqrt(2 / np.pi) * (a + 0.044715 * a ** 3)))


def _ln(x, w, b):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + 1e-5) * w + b


def _stats_tiles(x, Mp):
    """per-row partial (sum, sum of squares) over 16-column tiles: [tiles][Mp][2]"""
    M, C = x.shape
    t = C // 16
    st = np.zeros((t, Mp, 2), np.float32)
    for i in range(t):
        blk = x[:, 16 * i:16 * (i + 1)].astype(np.float64)
        st[i, :M, 0] = blk.sum(1)
        st[i, :M, 1] = (blk * blk).sum(1)
    return st


def _rbf16(x):
    """fp32 -> bf16 value (round to nearest even, finite inputs), as fp32"""
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def _bf16_ambiguous(a64):
    """elements within 1e-5 relative of a bf16 rounding midpoint"""
    a32 = a64.astype(np.float32)
    lo = a32.view(np.uint32) & np.uint32(0xFFFF0000)
    mid = (lo | np.uint32(0x8000)).view(np.float32).astype(np.float64)
    return np.abs(a64 - mid) <= 1e-5 * np.abs(a64)


def test_pack_frag_bf16_layout(hip):
    """bf16 frag layout (hip_paged_attn.h): element (m, k) at
    ((m/16 * K/32 + k/32) * 64 + m%16 + 16*((k%16)/4)) * 8 + k%4 + 4*((k%32)/16), RNE values"""
    L = hip.lib()
    rng = np.random.default_rng(5)
    rows, K = 70, 96
    a = rng.standard_normal((rows, K)).astype(np.float32)
    d_a = hip.DeviceBuffer.from_array(a)
    n = L.hpa_frag_bf16_elems(rows, K)
    assert n == 80 * K
    d_f = hip.DeviceBuffer(n * 2)
    hip.check(L.hpa_pack_frag_bf16(d_a.ptr, rows, K, K, d_f.ptr))
    f = d_f.download(n, np.uint16)
    m, k = np.meshgrid(np.arange(rows), np.arange(K), indexing="ij")
    idx = (((m >> 4) * (K >> 5) + (k >> 5)) * 64 + (m & 15) + 16 * ((k >> 2) & 3)) * 8 + (k & 3) + 4 * ((k >> 4) & 1)
    want = (_rbf16(a).view(np.uint32) >> 16).astype(np.uint16)
    assert np.array_equal(f[idx], want)
    mask = np.ones(n, bool)
    mask[idx.ravel()] = False
    assert np.all(f[mask] == 0)  # padded rows


@pytest.mark.parametrize("epi,M,K,N,waves,rb,ct,ln,variant", [
    ("RESID", 64, 768, 768, 4, 4, 2, True, 1), ("RESID", 80, 3072, 768, 8, 4, 1, False, 1),
    ("RESID", 64, 1600, 1600, 8, 2, 2, True, 1), ("RESID", 37, 768, 768, 4, 1, 1, False, 1),
    ("GELU", 256, 768, 3072, 4, 4, 2, True, 1), ("GELU", 64, 768, 3072, 8, 2, 1, True, 1),
    ("LOGITS", 64, 768, 50257, 4, 4, 2, True, 1), ("LOGITS", 256, 768, 50257, 0, 0, 0, True, 0),
    # A-resident kernel (variant 5; ct = rounds of `waves` column tiles per workgroup)
    ("RESID", 64, 768, 768, 8, 4, 1, True, 5), ("RESID", 80, 3072, 768, 4, 1, 2, False, 5),
    ("RESID", 48, 1600, 1600, 8, 2, 3, True, 5), ("RESID", 37, 768, 784, 4, 1, 1, True, 5),
    ("GELU", 256, 768, 3072, 8, 4, 2, True, 5), ("GELU", 64, 768, 3072, 4, 2, 1, True, 5),
    ("LOGITS", 64, 768, 50257, 8, 4, 4, True, 5), ("LOGITS", 256, 768, 50257, 8, 2, 8, True, 5),
    # automatic rounds at config 5's batch, and 50 rows (padded rows 50..63 of the last row group)
    ("LOGITS", 256, 768, 50257, 8, 4, 0, True, 5), ("LOGITS", 50, 768, 50257, 8, 4, 0, True, 5)])
def test_fused_bf16_weights(hip, epi, M, K, N, waves, rb, ct, ln, variant):
    """w_dtype = HPA_BF16: every epilogue against the f64 product of the
    bf16-rounded operands (LN applied before the rounding)"""
    L = hip.lib()
    e = dict(RESID=hip.HPA_FEPI_RESID, GELU=hip.HPA_FEPI_GELU, LOGITS=hip.HPA_FEPI_LOGITS)[epi]
    rng = np.random.default_rng(M + K + waves)
    res = rng.uniform(-1, 1, (M, N)).astype(np.float32)
    out, acc, bound, keep = _run(hip, e, M, K, N, waves, ln=ln, rng=rng, res=res, rb=rb, ct=ct, w_bf16=True,
                                 variant=variant)
    Mp = (M + 15) // 16 * 16
    if epi == "RESID":
        got = hip.from_frag(out.download(Mp * N), M, N)
        assert np.all(np.abs(got - (res + acc)) <= bound + 1e-6)
    elif epi == "GELU":
        got = hip.from_frag(out.download(Mp * N), M, N)
        ref = _gelu_tanh(acc)
        assert np.all(np.abs(got - ref) <= 1.2 * bound + 2e-5)  # |gelu'| <= 1.13
    else:
        got = out.download((M, N))
        assert np.all(np.abs(got - acc) <= bound)
        part = keep[-3]
        nxt = hip.DeviceBuffer(M * 4)
        hip.check(L.hpa_argmax_final(part.ptr, (N + 15) // 16, Mp, M, nxt.ptr, None, None, None))
        assert np.array_equal(nxt.download(M, np.int32), got.argmax(-1))


def test_fused_bf16_ares_relaunch_r5j_case(hip):
    """the case one intermediate round-5 suite failed once
    (RESID, M=48, K=N=1600, 8 waves, rb 2 -> 1 (3 row blocks), 3 rounds, LN,
    A-resident variant 5).  Same inputs, 24 launches in one process: every
    launch within the f64 bound and bit-identical to the first (a race in the
    kernel's LDS reuse across rounds would show as a launch-to-launch change)"""
    L = hip.lib()
    M, K, N, waves, rb, ct = 48, 1600, 1600, 8, 2, 3
    first = None
    for it in range(24):
        rng = np.random.default_rng(M + K + waves)
        res = rng.uniform(-1, 1, (M, N)).astype(np.float32)
        out, acc, bound, keep = _run(hip, hip.HPA_FEPI_RESID, M, K, N, waves, ln=True, rng=rng, res=res, rb=rb,
                                     ct=ct, w_bf16=True, variant=5)
        got = hip.from_frag(out.download(M * N), M, N)
        err = np.abs(got - (res + acc)) - (bound + 1e-6)
        assert np.all(err <= 0), (it, int(np.argmax(err)), float(err.max()))
        if first is None:
            first = got
        else:
            assert np.array_equal(got, first), (it, int(np.sum(got != first)))
    del L


def test_fused_bf16_rows_independent_of_shape(hip):
    """a row's bf16 result depends on the waves only, never on row blocks,
    column tiles or M (bit-identical)"""
    rng = np.random.default_rng(21)
    K, N = 768, 768
    fixed = dict(x=rng.uniform(-1, 1, (64, K)).astype(np.float32),
                 W=rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=rng.uniform(-0.1, 0.1, N).astype(np.float32),
                 lw=rng.uniform(0.8, 1.2, K).astype(np.float32), lb=rng.uniform(-0.1, 0.1, K).astype(np.float32))
    res = np.zeros((64, N), np.float32)
    for variant, shapes in [(1, [(4, 64, 4, 2), (4, 64, 1, 1), (4, 64, 2, 2), (4, 48, 1, 1)]),
                            (5, [(8, 64, 4, 1), (4, 64, 1, 3), (8, 64, 2, 2), (4, 48, 1, 1)])]:
        outs = []
        for waves, M, rb, ct in shapes:
            out, _, _, keep = _run(hip, hip.HPA_FEPI_RESID, M, K, N, waves, ln=True, rng=rng, res=res[:M], rb=rb,
                                   ct=ct, fixed=fixed, w_bf16=True, variant=variant)
            outs.append(hip.from_frag(out.download((M + 15) // 16 * 16 * N), M, N))
        for o in outs[1:]:
            assert np.array_equal(o, outs[0][:o.shape[0]])


def test_pack_unpack_roundtrip(hip):
    L = hip.lib()
    rng = np.random.default_rng(0)
    a = rng.standard_normal((70, 96)).astype(np.float32)
    d_a = hip.DeviceBuffer.from_array(a)
    n = L.hpa_frag_elems(70, 96)
    d_f = hip.DeviceBuffer(n * 4)
    hip.check(L.hpa_pack_frag(d_a.ptr, 70, 96, 96, d_f.ptr))
    f = d_f.download(n)
    assert np.array_equal(f, hip.to_frag(a))
    d_b = hip.DeviceBuffer(a.nbytes)
    hip.check(L.hpa_unpack_frag(d_f.ptr, 70, 96, d_b.ptr, 96))
    assert np.array_equal(d_b.download(a.shape), a)


def _run(hip, epi, M, K, N, waves, ln, rng, res=None, pool_args=None, rb=0, fixed=None, variant=0, ct=0,
         fold=False, w_bf16=False, sk_ws=False):
    L = hip.lib()
    x = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    W = rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32)
    bias = rng.uniform(-0.1, 0.1, N).astype(np.float32)
    if fixed is not None:  # caller-provided operands (rows of x: the first M)
        x, W, bias = fixed["x"][:M], fixed["W"], fixed["bias"]
    Mp = (M + 15) // 16 * 16
    keep = []

    def dev(a):
        b = hip.DeviceBuffer.from_array(np.ascontiguousarray(a))
        keep.append(b)
        return b.ptr

    g = hip.HpaFusedGemm()
    g.x = dev(hip.to_frag(x))
    g.M, g.K, g.N = M, K, N
    if ln:
        lw = rng.uniform(0.8, 1.2, K).astype(np.float32)
        lb = rng.uniform(-0.1, 0.1, K).astype(np.float32)
        if fixed is not None:
            lw, lb = fixed["lw"], fixed["lb"]
        g.ln_stats = dev(_stats_tiles(x, Mp))
        g.ln_ntiles = K // 16
        g.ln_w, g.ln_b = dev(lw), dev(lb)
        a = _ln(x.astype(np.float64), lw, lb)
    else:
        a = x.astype(np.float64)
    g.w = dev(hip.to_frag(W))
    if w_bf16:  # bf16 weights (hpa_gemm_bf16.hip): packed on the device from fp32 W
        wb = hip.DeviceBuffer(L.hpa_frag_bf16_elems(N, K) * 2)
        keep.append(wb)
        hip.check(L.hpa_pack_frag_bf16(dev(W), N, K, K, wb.ptr), "pack bf16")
        g.w, g.w_dtype = wb.ptr, hip.HPA_BF16
        # reference: bf16-rounded operands, exact products, f64 sums; an A element
        # whose f64 value sits within 1e-5 relative of a bf16 rounding midpoint may
        # round either way on the GPU (fp32 LN): one bf16 ulp (2^-7 |a| bound) there
        a32 = a.astype(np.float32)
        amb = _bf16_ambiguous(a)
        ab = _rbf16(a32).astype(np.float64)
        Wb = _rbf16(W).astype(np.float64)
        extra = (amb * np.abs(a) * 2.0 ** -7) @ np.abs(Wb).T
        a, W = ab, Wb
    g.bias = dev(bias) if epi != hip.HPA_FEPI_LOGITS else None
    if fold:  # LN folded into the packed weights (hpa_ln_fold_pack)
        assert ln
        wf = hip.DeviceBuffer(L.hpa_frag_elems(N, K) * 4)
        c1, c2 = hip.DeviceBuffer(N * 4), hip.DeviceBuffer(N * 4)
        keep.extend([wf, c1, c2])
        hip.check(L.hpa_ln_fold_pack(dev(W), N, K, g.ln_w, g.ln_b, g.bias, wf.ptr, c1.ptr, c2.ptr), "fold")
        hip.check(L.hpa_synchronize())
        g.w, g.bias, g.ln_fold_c1 = wf.ptr, c2.ptr, c1.ptr
        Wg = (W * lw).astype(np.float64)  # the packed products (fp32-rounded: within the bound's slack)
        x64 = x.astype(np.float64)
        mu = x64.mean(-1)
        rs = 1 / np.sqrt(((x64 - mu[:, None]) ** 2).mean(-1) + 1e-5)
        c1h = Wg.sum(1)
        fold_bound = 4e-6 * rs[:, None] * (np.abs(x64) @ np.abs(Wg).T + np.abs(mu)[:, None] * np.abs(c1h)) + 2e-6
    g.waves = waves
    g.row_blocks = rb
    g.variant = variant
    g.col_tiles = ct
    g.epilogue = epi
    acc = a @ W.astype(np.float64).T
    bound = 4e-6 * (np.abs(a) @ np.abs(W.astype(np.float64)).T) + 2e-6
    if w_bf16:
        bound = bound + extra
    if fold:
        bound = np.maximum(bound, fold_bound)
    if epi != hip.HPA_FEPI_LOGITS:
        acc = acc + bias
    if epi == hip.HPA_FEPI_RESID:
        g.res_in = dev(hip.to_frag(res))
        out = hip.DeviceBuffer(Mp * N * 4)
        st = hip.DeviceBuffer(N // 16 * Mp * 2 * 4)
        g.out, g.stats_out = out.ptr, st.ptr
        keep.append(st)
    elif epi == hip.HPA_FEPI_GELU:
        out = hip.DeviceBuffer(Mp * N * 4)
        g.out = out.ptr
    elif epi == hip.HPA_FEPI_LOGITS:
        out = hip.DeviceBuffer(M * N * 4)
        part = hip.DeviceBuffer((N + 15) // 16 * Mp * 2 * 4)
        g.out, g.part_out = out.ptr, part.ptr
        keep.append(part)
    else:
        out = hip.DeviceBuffer(M * (N // 3) * 4)
        g.out = out.ptr
        pool, bt, pos = pool_args
        g.pool = ctypes.pointer(pool.s)
        g.layer = 0
        g.block_table, g.bt_stride, g.pos = dev(bt), bt.shape[1], dev(pos)
    keep.append(out)
    keep.append(g)  # the descriptor (LOGITS: hpa_logits_partials)
    if variant == 3 and waves > 1:  # K-split ring: slab + counters (zeroed once; every launch leaves them zero)
        nf, nc = ctypes.c_size_t(), ctypes.c_size_t()
        hip.check(L.hpa_gemm_ring_workspace(N, waves, ctypes.byref(nf), ctypes.byref(nc)), "ring workspace")
        slab = hip.DeviceBuffer(nf.value * 4)
        cnt = hip.DeviceBuffer.from_array(np.zeros(nc.value, np.int32))
        keep.extend([slab, cnt])
        g.sk_slab, g.sk_count = slab.ptr, cnt.ptr
    if variant == 6 or sk_ws:  # stream-K: slab + counters (zeroed once; every launch leaves them zero)
        nf, nc = ctypes.c_size_t(), ctypes.c_size_t()
        hip.check(L.hpa_gemm_sk_workspace(N, ctypes.byref(nf), ctypes.byref(nc)), "sk workspace")
        slab = hip.DeviceBuffer(nf.value * 4)
        cnt = hip.DeviceBuffer.from_array(np.zeros(nc.value, np.int32))
        keep.extend([slab, cnt])
        g.sk_slab, g.sk_count = slab.ptr, cnt.ptr
    hip.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm_fused")
    hip.check(L.hpa_synchronize())
    return out, acc, bound, keep


@pytest.mark.parametrize("M,K,N,waves,rb,ct", [(64, 256, 128, 4, 4, 1), (64, 256, 128, 16, 1, 1),
                                               (8, 768, 768, 16, 2, 1), (40, 3072, 768, 8, 1, 1),
                                               (100, 512, 96, 16, 4, 1), (3, 48, 32, 16, 1, 1),
                                               (130, 768, 768, 0, 0, 0), (64, 3072, 768, 4, 2, 1),
                                               (48, 1600, 1600, 8, 4, 1), (64, 768, 768, 4, 4, 2),
                                               (64, 768, 80, 4, 4, 4)])
def test_fused_resid_with_stats(hip, M, K, N, waves, rb, ct):
    rng = np.random.default_rng(M + waves + rb)
    res = rng.uniform(-1, 1, (M, N)).astype(np.float32)
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_RESID, M, K, N, waves, ln=(K == N), rng=rng, res=res, rb=rb,
                                 ct=ct)
    Mp = (M + 15) // 16 * 16
    got = hip.from_frag(out.download(Mp * N), M, N)
    ref = res + acc
    assert np.all(np.abs(got - ref) <= bound + 1e-6)
    # padded rows stay zero
    full = out.download(Mp * N)
    if Mp > M:
        assert np.all(hip.from_frag(full, Mp, N)[M:] == 0)


@pytest.mark.parametrize("waves,rb", [(4, 1), (8, 2), (16, 4), (16, 1)])
def test_fused_gelu_with_ln(hip, waves, rb):
    rng = np.random.default_rng(waves + rb)
    M, K, N = 64, 768, 3072
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_GELU, M, K, N, waves, ln=True, rng=rng, rb=rb)
    got = hip.from_frag(out.download(M * N), M, N)
    ref = _gelu_tanh(acc)
    assert np.abs(got - ref).max() <= 2e-5


@pytest.mark.parametrize("M,waves,rb,ct", [(64, 4, 4, 1), (37, 8, 1, 1), (64, 16, 2, 1), (64, 4, 4, 2),
                                           (64, 4, 4, 4), (40, 8, 2, 2), (64, 8, 4, 2)])
def test_fused_logits_argmax(hip, M, waves, rb, ct):
    L = hip.lib()
    rng = np.random.default_rng(3)
    K, N = 768, 50257
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, waves, ln=True, rng=rng, rb=rb, ct=ct)
    got = out.download((M, N))
    assert np.all(np.abs(got - acc) <= bound)
    part = keep[-3]
    nxt = hip.DeviceBuffer(M * 4)
    Mp = (M + 15) // 16 * 16
    hip.check(L.hpa_argmax_final(part.ptr, (N + 15) // 16, Mp, M, nxt.ptr, None, None, None))
    ids = nxt.download(M, np.int32)
    assert np.array_equal(ids, got.argmax(-1))


@pytest.mark.parametrize("form", [0, 12, 16])
@pytest.mark.parametrize("M", [64, 37, 16, 1])
def test_logits_resident_kernel(hip, M, form):
    """variant 4 (activation-resident, hpa_logits.hip; form 12 = ring, 16 =
    16-wave K split, 0 = by M): logits within the fp32 bound of the float64
    reference, argmax partials consistent, and within rounding of the looped
    kernel"""
    L = hip.lib()
    rng = np.random.default_rng(11)
    K, N = 768, 50257
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, form, ln=True, rng=rng, variant=4)
    got = out.download((M, N))
    assert np.all(np.abs(got - acc) <= bound)
    part, g = keep[-3], keep[-1]
    # one running (max, argmax) partial per row per workgroup (grid <= CUs)
    npart = L.hpa_logits_partials(ctypes.byref(g))
    assert 0 < npart <= 256
    nxt = hip.DeviceBuffer(M * 4)
    Mp = (M + 15) // 16 * 16
    hip.check(L.hpa_argmax_final(part.ptr, npart, Mp, M, nxt.ptr, None, None, None))
    assert np.array_equal(nxt.download(M, np.int32), got.argmax(-1))
    rng = np.random.default_rng(11)
    out1, _, _, keep1 = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, 4, ln=True, rng=rng, rb=1, variant=1)
    got1 = out1.download((M, N))
    assert np.abs(got1 - got).max() <= 2e-5
    # the looped kernel: one partial per 16-column tile
    assert L.hpa_logits_partials(ctypes.byref(keep1[-1])) == (N + 15) // 16
    hip.check(L.hpa_argmax_final(keep1[-3].ptr, (N + 15) // 16, Mp, M, nxt.ptr, None, None, None))
    assert np.array_equal(nxt.download(M, np.int32), got1.argmax(-1))


@pytest.mark.parametrize("form", [12, 16])
def test_logits_resident_rows_independent_of_batch(hip, form):
    """variant 4, each form of the resident kernel (waves 12: the ring form,
    rows split over waves, 1 or 2 K parts per wave; waves 16: K split over 16
    waves): a row's logits and argmax are bit-identical at 64, 48, 32, 16 and
    5 rows -- the same sum at every row count, which is what keeps a sharded
    decode equal to the unsharded one (the engine picks the form by the
    global batch)"""
    L = hip.lib()
    rng = np.random.default_rng(23)
    K, N = 768, 50257
    fixed = dict(x=rng.uniform(-1, 1, (64, K)).astype(np.float32),
                 W=rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=np.zeros(N, np.float32),
                 lw=rng.uniform(0.8, 1.2, K).astype(np.float32), lb=rng.uniform(-0.1, 0.1, K).astype(np.float32))
    outs, ids = [], []
    for M in (64, 48, 32, 16, 5):
        out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, form, ln=True, rng=np.random.default_rng(0),
                                     fixed=fixed, variant=4)
        got = out.download((M, N))
        assert np.all(np.abs(got - acc) <= bound)
        npart = L.hpa_logits_partials(ctypes.byref(keep[-1]))
        nxt = hip.DeviceBuffer(M * 4)
        hip.check(L.hpa_argmax_final(keep[-3].ptr, npart, (M + 15) // 16 * 16, M, nxt.ptr, None, None, None))
        outs.append(got)
        ids.append(nxt.download(M, np.int32))
        assert np.array_equal(ids[-1], got.argmax(-1))
    for o, i in zip(outs[1:], ids[1:]):
        assert np.array_equal(o, outs[0][:o.shape[0]])
        assert np.array_equal(i, ids[0][:i.shape[0]])


@pytest.mark.parametrize("form", [0, 12])
def test_logits_resident_argmax_ties_first_index(hip, form):
    """equal maxima in several column tiles and workgroups: the lowest column
    wins, as the reference's strict-> scan (paged_infer.c:937-951); form 0 =
    by rows (the 16-wave form at 16 rows), 12 = the ring form"""
    L = hip.lib()
    M, K, N = 16, 768, 50257
    x = np.zeros((M, K), np.float32)
    x[:, 0] = 1.0
    W = np.zeros((N, K), np.float32)
    # logit = W[:, 0] * LN(x)[0]; LN of a one-hot row is a fixed positive value at k = 0
    cols = [7, 4000, 4001, 25000, 50256]
    W[cols, 0] = 0.5
    fixed = dict(x=x, W=W, bias=np.zeros(N, np.float32), lw=np.ones(K, np.float32), lb=np.zeros(K, np.float32))
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, form, ln=True, rng=np.random.default_rng(0),
                                 fixed=fixed, variant=4)
    got = out.download((M, N))
    assert np.all(got[:, cols] == got[0, 7]) and got[0, 7] > got[0, 8]
    npart = L.hpa_logits_partials(ctypes.byref(keep[-1]))
    nxt = hip.DeviceBuffer(M * 4)
    hip.check(L.hpa_argmax_final(keep[-3].ptr, npart, 16, M, nxt.ptr, None, None, None))
    assert np.array_equal(nxt.download(M, np.int32), np.full(M, 7, np.int32))


@pytest.mark.parametrize("M,form,variant", [(64, 12, 4), (37, 12, 4), (16, 16, 4), (5, 0, 4), (20, 0, 1)])
def test_logits_in_launch_pick(hip, M, form, variant):
    """HpaFusedGemm.pick_next: the resident logits kernel's last workgroup
    reduces the argmax partials in the launch (both forms), other LOGITS paths
    pick with hpa_argmax_final after it -- either way next = tokens = the
    argmax of each row (lowest column among equals), pos += 1, and the arrival
    counter is left at zero for the next launch (three launches back to back)"""
    L = hip.lib()
    rng = np.random.default_rng(41 + M)
    K, N = 768, 50257
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, form, ln=True, rng=rng, variant=variant)
    got = out.download((M, N))
    ids = got.argmax(-1).astype(np.int32)
    g = keep[-1]
    nxt = hip.DeviceBuffer.from_array(np.full(M, -7, np.int32))
    tok = hip.DeviceBuffer.from_array(np.full(M, -7, np.int32))
    pos = hip.DeviceBuffer.from_array(np.arange(M, dtype=np.int32))
    cnt = hip.DeviceBuffer.from_array(np.zeros(1, np.int32))
    g.pick_next, g.pick_tokens, g.pick_pos, g.pick_count = nxt.ptr, tok.ptr, pos.ptr, cnt.ptr
    for it in range(3):
        hip.check(L.hpa_gemm_fused(ctypes.byref(g)), "gemm_fused pick")
        hip.check(L.hpa_synchronize())
        assert np.array_equal(out.download((M, N)), got)
        assert np.array_equal(nxt.download(M, np.int32), ids), it
        assert np.array_equal(tok.download(M, np.int32), ids)
        assert np.array_equal(pos.download(M, np.int32), np.arange(M) + it + 1)
        assert cnt.download(1, np.int32)[0] == 0
    g.pick_next = g.pick_tokens = g.pick_pos = g.pick_count = None


def test_fused_qkv_appends_into_pages(hip):
    rng = np.random.default_rng(9)
    NH, P = 2, 16
    C = NH * 64
    M, K, N = 5, C, 3 * C
    pool = hip.Pool(1, NH, P, 20)
    bt = rng.permutation(20).astype(np.int32)[:20].reshape(5, 4)
    pos = np.array([0, 15, 16, 33, 63], np.int32)
    out, acc, bound, keep = _run(hip, hip.HPA_FEPI_QKV, M, K, N, 8, ln=True, rng=rng,
                                 pool_args=(pool, bt, pos))
    q = out.download((M, C))
    assert np.all(np.abs(q - acc[:, :C]) <= bound[:, :C])
    for b in range(M):
        k, v = pool.read_tokens(0, bt[b], pos[b] + 1)
        assert np.all(np.abs(k[pos[b]] - acc[b, C:2 * C]) <= bound[b, C:2 * C])
        assert np.all(np.abs(v[pos[b]] - acc[b, 2 * C:]) <= bound[b, 2 * C:])


def test_fused_fold_deterministic(hip):
    """the LDS fold sums the waves' partials in wave order: bit-identical
    across repeated launches"""
    rng = np.random.default_rng(4)
    res = rng.uniform(-1, 1, (64, 768)).astype(np.float32)
    outs = []
    for _ in range(3):
        out, acc, bound, keep = _run(hip, hip.HPA_FEPI_RESID, 64, 3072, 768, 16, ln=False,
                                     rng=np.random.default_rng(4), res=res)
        outs.append(out.download(64 * 768))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])


def test_fused_rejects_bad_launch_shape(hip):
    rng = np.random.default_rng(5)
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 16, 64, 64, 2, ln=False, rng=rng)
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 16, 64, 64, 4, ln=False, rng=rng, rb=3)
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 64, 64, 64, 4, ln=False, rng=rng, rb=4, ct=3)
    with pytest.raises(RuntimeError):  # LN'ed A operand wider than the LDS copy of w, b
        _run(hip, hip.HPA_FEPI_GELU, 16, 2064, 64, 4, ln=True, rng=rng)


@pytest.mark.parametrize("epi", ["RESID", "LOGITS"])
def test_fused_rows_independent_of_split(hip, epi):
    """a row's result depends only on the waves (per-wave K ranges): equal
    bit for bit across row_blocks 1/2/4 and across M (the micro-batch lanes
    rely on this)"""
    e = getattr(hip, "HPA_FEPI_" + epi)
    N = 768 if epi == "RESID" else 4000
    r = np.random.default_rng(7)
    K = 768
    fixed = dict(x=r.uniform(-1, 1, (64, K)).astype(np.float32),
                 W=r.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=r.uniform(-0.1, 0.1, N).astype(np.float32),
                 lw=r.uniform(0.8, 1.2, K).astype(np.float32), lb=r.uniform(-0.1, 0.1, K).astype(np.float32))
    res = r.uniform(-1, 1, (64, N)).astype(np.float32)
    outs = []
    for M, rb, ct in [(64, 1, 1), (64, 2, 1), (64, 4, 1), (16, 1, 1), (32, 2, 1), (64, 4, 2), (32, 2, 2)]:
        out, _, _, keep = _run(hip, e, M, K, N, 8, ln=True, rng=np.random.default_rng(7),
                               res=res[:M], rb=rb, fixed=fixed, ct=ct)
        if epi == "RESID":
            got = hip.from_frag(out.download(((M + 15) // 16 * 16) * N), M, N)
        else:
            got = out.download((M, N))
        outs.append(got[:16])
    for o in outs[1:]:
        assert np.array_equal(outs[0], o)


@pytest.mark.parametrize("epi,K,N,waves", [("RESID", 768, 768, 4), ("GELU", 768, 3072, 8), ("RESID", 768, 768, 16),
                                           ("RESID", 3072, 768, 8), ("QKV", 768, 2304, 4)])
@pytest.mark.parametrize("M", [64, 37])
def test_fused_oneshot_bit_identical_to_looped(hip, epi, K, N, waves, M):
    """the one-shot kernel (all operand loads up front) keeps the looped
    kernel's per-wave K ranges, k order and LN statistics order: equal bit
    for bit, and within the f64 bound"""
    e = getattr(hip, "HPA_FEPI_" + epi)
    r = np.random.default_rng(11)
    fixed = dict(x=r.uniform(-1, 1, (M, K)).astype(np.float32),
                 W=r.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=r.uniform(-0.1, 0.1, N).astype(np.float32),
                 lw=r.uniform(0.8, 1.2, K).astype(np.float32), lb=r.uniform(-0.1, 0.1, K).astype(np.float32))
    res = r.uniform(-1, 1, (M, N)).astype(np.float32)
    ln = K == 768
    outs = []
    for variant in (1, 2):
        pool_args = None
        if epi == "QKV":
            NH, P = N // 3 // 64, 16
            pool = hip.Pool(1, NH, P, 4 * M)
            bt = np.arange(4 * M, dtype=np.int32).reshape(M, 4)
            pos = (np.arange(M, dtype=np.int32) * 7) % 64
            pool_args = (pool, bt, pos)
        out, acc, bound, keep = _run(hip, e, M, K, N, waves, ln=ln, rng=np.random.default_rng(0), res=res,
                                     rb=1, fixed=fixed, variant=variant, pool_args=pool_args)
        if epi == "QKV":
            q = out.download((M, N // 3))
            k, v = pool.read_tokens(0, bt[M - 1], pos[M - 1] + 1)
            outs.append((q, k[pos[M - 1]].copy(), v[pos[M - 1]].copy()))
            assert np.all(np.abs(q - acc[:, :N // 3]) <= bound[:, :N // 3])
        else:
            Mp = (M + 15) // 16 * 16
            got = hip.from_frag(out.download(Mp * N), M, N)
            outs.append((got,))
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_fused_oneshot_rejects_unsupported_shape(hip):
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 16, 512, 64, 4, ln=False, rng=np.random.default_rng(1), variant=2)


@pytest.mark.parametrize("epi,N,waves,variant,rb,ct", [("GELU", 3072, 4, 2, 1, 1), ("GELU", 3072, 4, 1, 1, 1),
                                                       ("QKV", 2304, 4, 2, 1, 1), ("QKV", 2304, 8, 1, 4, 2),
                                                       ("GELU", 3072, 8, 1, 4, 2)])
@pytest.mark.parametrize("M", [64, 37])
def test_fused_ln_fold(hip, epi, N, waves, variant, rb, ct, M):
    """LayerNorm folded into the packed weights (hpa_ln_fold_pack, the
    engine's qkv / fc): within the f64 bound of LN(x) . W^T + b, for the
    one-shot (decode) and looped multi-tile (prefill) kernels; the two
    kernels agree bit for bit"""
    e = getattr(hip, "HPA_FEPI_" + epi)
    K = 768
    r = np.random.default_rng(13)
    fixed = dict(x=(r.uniform(-1, 1, (M, K)) + r.uniform(-0.5, 0.5, (M, 1))).astype(np.float32),  # mean != 0
                 W=r.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=r.uniform(-0.1, 0.1, N).astype(np.float32),
                 lw=r.uniform(0.8, 1.2, K).astype(np.float32), lb=r.uniform(-0.1, 0.1, K).astype(np.float32))
    pool_args = None
    if epi == "QKV":
        pool = hip.Pool(1, N // 3 // 64, 16, 4 * M)
        bt = np.arange(4 * M, dtype=np.int32).reshape(M, 4)
        pos = (np.arange(M, dtype=np.int32) * 7) % 64
        pool_args = (pool, bt, pos)
    out, acc, bound, keep = _run(hip, e, M, K, N, waves, ln=True, rng=np.random.default_rng(0), rb=rb,
                                 fixed=fixed, variant=variant, ct=ct, pool_args=pool_args, fold=True)
    if epi == "QKV":
        C = N // 3
        q = out.download((M, C))
        assert np.all(np.abs(q - acc[:, :C]) <= bound[:, :C])
        for b in (0, M - 1):
            k, v = pool.read_tokens(0, bt[b], pos[b] + 1)
            assert np.all(np.abs(k[pos[b]] - acc[b, C:2 * C]) <= bound[b, C:2 * C])
            assert np.all(np.abs(v[pos[b]] - acc[b, 2 * C:]) <= bound[b, 2 * C:])
        got = q
    else:
        Mp = (M + 15) // 16 * 16
        got = hip.from_frag(out.download(Mp * N), M, N)
        ref = 0.5 * acc * (1 + np.tanh(np.sqrt(2 / np.pi) * (acc + 0.044715 * acc ** 3)))
        assert np.all(np.abs(got - ref) <= bound + 1e-6)
    if variant == 2:  # the looped kernel with the same waves: same bits
        out1, _, _, keep1 = _run(hip, e, M, K, N, waves, ln=True, rng=np.random.default_rng(0), rb=1,
                                 fixed=fixed, variant=1, ct=1, pool_args=pool_args, fold=True)
        got1 = out1.download((M, N // 3)) if epi == "QKV" else hip.from_frag(out1.download(Mp * N), M, N)
        assert np.array_equal(got, got1)


@pytest.mark.parametrize("epi,K,N,fold", [("GELU", 1600, 6400, True), ("QKV", 1600, 4800, True),
                                          ("RESID", 6400, 1600, False), ("RESID", 1600, 1600, False),
                                          ("LOGITS", 1600, 1000, False), ("GELU", 768, 3072, True),
                                          ("RESID", 3072, 768, False), ("GELU", 256, 80, False),
                                          ("LOGITS", 1600, 1000, "apply"), ("GELU", 768, 3072, "apply"),
                                          ("LOGITS", 1600, 50257, "apply")])
@pytest.mark.parametrize("M", [64, 37, 16, 1])
def test_fused_stream_k(hip, epi, K, N, fold, M):
    """stream-K kernel (variant 6, hpa_gemm_sk.hip): every epilogue within the
    f64 bound; LayerNorm folded with the producer's row statistics (True) or
    applied to the A fragments on load ("apply": the XL logits' LNf);
    odd column-tile counts (N = 1000, 80: a half-filled last super-tile);
    tiles split between workgroups summed by the last to arrive; a relaunch is
    bit identical and leaves the counters zero"""
    e = getattr(hip, "HPA_FEPI_" + epi)
    rng = np.random.default_rng(K + N + M)
    res = rng.uniform(-1, 1, (M, N)).astype(np.float32) if epi == "RESID" else None
    pool_args = None
    if epi == "QKV":
        pool = hip.Pool(1, N // 3 // 64, 16, 4 * M)
        bt = np.arange(4 * M, dtype=np.int32).reshape(M, 4)
        pos = (np.arange(M, dtype=np.int32) * 7) % 64
        pool_args = (pool, bt, pos)
    out, acc, bound, keep = _run(hip, e, M, K, N, 8, ln=bool(fold), rng=rng, res=res, pool_args=pool_args,
                                 variant=6, fold=fold is True)
    Mp = (M + 15) // 16 * 16
    if epi == "QKV":
        C = N // 3
        got = out.download((M, C))
        assert np.all(np.abs(got - acc[:, :C]) <= bound[:, :C])
        for b in (0, M - 1):
            k, v = pool.read_tokens(0, bt[b], pos[b] + 1)
            assert np.all(np.abs(k[pos[b]] - acc[b, C:2 * C]) <= bound[b, C:2 * C])
            assert np.all(np.abs(v[pos[b]] - acc[b, 2 * C:]) <= bound[b, 2 * C:])
    elif epi == "LOGITS":
        got = out.download((M, N))
        assert np.all(np.abs(got - acc) <= bound)
    else:
        got = hip.from_frag(out.download(Mp * N), M, N)
        if epi == "GELU":
            ref = 0.5 * acc * (1 + np.tanh(np.sqrt(2 / np.pi) * (acc + 0.044715 * acc ** 3)))
            assert np.all(np.abs(got - ref) <= bound + 1e-6)
        else:
            assert np.all(np.abs(got - (acc + res)) <= bound + 1e-6)
    # relaunch: bit-identical (fixed summation order), counters back at zero
    g = [k for k in keep if isinstance(k, hip.HpaFusedGemm)][0]
    hip.check(hip.lib().hpa_gemm_fused(ctypes.byref(g)), "relaunch")
    hip.check(hip.lib().hpa_synchronize())
    again = out.download((M, N // 3)) if epi == "QKV" else out.download((M, N)) if epi == "LOGITS" else \
        hip.from_frag(out.download(Mp * N), M, N)
    assert np.array_equal(again, got)
    cnt = [k for k in keep if isinstance(k, hip.DeviceBuffer)][-1]
    assert not cnt.download((cnt.nbytes // 4,), np.int32).any()


def test_fused_stream_k_rejects_wide_layernorm(hip):
    """LN applied on load stages its weights in LDS: K > 2048 is refused"""
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 16, 3072, 768, 8, ln=True, rng=np.random.default_rng(1), variant=6)


def test_logits_variant4_takes_stream_k_with_workspace(hip):
    """variant 4 at K = 1600 (not the resident kernel's shape): with a stream-K
    workspace it runs stream-K (bit-identical to variant 6), without one the
    looped kernel; both within the f64 bound"""
    M, K, N = 64, 1600, 3000
    outs = []
    for variant, ws in ((6, True), (4, True), (4, False)):
        out, acc, bound, keep = _run(hip, hip.HPA_FEPI_LOGITS, M, K, N, 8, ln=True,
                                     rng=np.random.default_rng(5), variant=variant, sk_ws=ws)
        got = out.download((M, N))
        assert np.all(np.abs(got - acc) <= bound)
        outs.append(got)
    assert np.array_equal(outs[0], outs[1])



@pytest.mark.parametrize("epi,K,N,fold", [("GELU", 1600, 6400, True), ("QKV", 1600, 4800, True),
                                          ("RESID", 6400, 1600, False), ("RESID", 1600, 1600, False),
                                          ("GELU", 768, 3072, True), ("GELU", 256, 80, False),
                                          ("RESID", 48, 1616, False), ("QKV", 768, 2304, False)])
@pytest.mark.parametrize("M", [64, 49, 20, 5])
@pytest.mark.parametrize("parts", [1, 3])
def test_fused_ring(hip, epi, K, N, fold, M, parts):
    """loader / MFMA-wave ring kernel (variant 3, hpa_gemm_ring.hip): every
    epilogue within the f64 bound at 16-64 padded rows; LN folded or absent;
    K not a multiple of the 8-step stage (K16 = 100, 3); an odd column-tile
    count (N = 80, 1616: the last workgroup's second tile past N); the RESID
    epilogue's 16-column LN partial sums; a relaunch is bit identical; K split
    in 3 parts over workgroups (the last part of a column pair sums them and
    rewinds its counter)"""
    if parts > 1 and K < 48 * parts:
        pytest.skip("fewer 4-step stages than K parts")
    e = getattr(hip, "HPA_FEPI_" + epi)
    rng = np.random.default_rng(K + N + M + 3)
    res = rng.uniform(-1, 1, (M, N)).astype(np.float32) if epi == "RESID" else None
    pool_args = None
    if epi == "QKV":
        pool = hip.Pool(1, N // 3 // 64, 16, 4 * M)
        bt = np.arange(4 * M, dtype=np.int32).reshape(M, 4)
        pos = (np.arange(M, dtype=np.int32) * 7) % 64
        pool_args = (pool, bt, pos)
    out, acc, bound, keep = _run(hip, e, M, K, N, parts, ln=fold, rng=rng, res=res, pool_args=pool_args,
                                 variant=3, fold=fold)
    Mp = (M + 15) // 16 * 16
    if epi == "QKV":
        C = N // 3
        got = out.download((M, C))
        assert np.all(np.abs(got - acc[:, :C]) <= bound[:, :C])
        for b in (0, M // 2, M - 1):
            k, v = pool.read_tokens(0, bt[b], pos[b] + 1)
            assert np.all(np.abs(k[pos[b]] - acc[b, C:2 * C]) <= bound[b, C:2 * C])
            assert np.all(np.abs(v[pos[b]] - acc[b, 2 * C:]) <= bound[b, 2 * C:])
    else:
        full = out.download(Mp * N)
        got = hip.from_frag(full, M, N)
        if epi == "GELU":
            ref = 0.5 * acc * (1 + np.tanh(np.sqrt(2 / np.pi) * (acc + 0.044715 * acc ** 3)))
            assert np.all(np.abs(got - ref) <= bound + 1e-6)
        else:
            assert np.all(np.abs(got - (acc + res)) <= bound + 1e-6)
            assert not hip.from_frag(full, Mp, N)[M:].any()  # padded rows stay zero
            st = [k for k in keep if isinstance(k, hip.DeviceBuffer) and k.nbytes == N // 16 * Mp * 2 * 4][0]
            st = st.download((N // 16, Mp, 2))
            g16 = got.astype(np.float64).reshape(M, N // 16, 16)
            assert np.allclose(st[:, :M, 0].T, g16.sum(-1), rtol=1e-5, atol=1e-4)
            assert np.allclose(st[:, :M, 1].T, (g16 ** 2).sum(-1), rtol=1e-5, atol=1e-4)
    g = [k for k in keep if isinstance(k, hip.HpaFusedGemm)][0]
    hip.check(hip.lib().hpa_gemm_fused(ctypes.byref(g)), "relaunch")
    hip.check(hip.lib().hpa_synchronize())
    again = out.download((M, N // 3)) if epi == "QKV" else hip.from_frag(out.download(Mp * N), M, N)
    assert np.array_equal(again, got)
    if parts > 1:
        cnt = [k for k in keep if isinstance(k, hip.DeviceBuffer)][-1]
        assert not cnt.download((cnt.nbytes // 4,), np.int32).any()


def test_fused_ring_rows_independent_of_batch(hip):
    """a row's result depends only on K (the ring's two fixed chains), never
    on M: the rows of a 20-row launch equal the same rows of a 64-row one"""
    rng = np.random.default_rng(12)
    K, N = 1600, 4800
    fixed = dict(x=rng.uniform(-1, 1, (64, K)).astype(np.float32),
                 W=rng.uniform(-0.05, 0.05, (N, K)).astype(np.float32),
                 bias=rng.uniform(-0.1, 0.1, N).astype(np.float32),
                 lw=rng.uniform(0.8, 1.2, K).astype(np.float32), lb=rng.uniform(-0.1, 0.1, K).astype(np.float32))
    for parts in (1, 3):
        outs = []
        for M in (64, 20):
            out, _, _, keep = _run(hip, hip.HPA_FEPI_GELU, M, K, N, parts, ln=True, rng=rng, fixed=fixed, variant=3,
                                   fold=True)
            outs.append(hip.from_frag(out.download((M + 15) // 16 * 16 * N), M, N))
        assert np.array_equal(outs[0][:20], outs[1])


def test_fused_ring_rejects_unsupported_shape(hip):
    """variant 3 needs <= 64 padded rows and no LayerNorm applied on load"""
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 65, 768, 256, 1, ln=False, rng=np.random.default_rng(1), variant=3)
    with pytest.raises(RuntimeError):
        _run(hip, hip.HPA_FEPI_GELU, 64, 768, 256, 1, ln=True, rng=np.random.default_rng(1), variant=3)
    with pytest.raises(RuntimeError):  # 5 K parts
        _run(hip, hip.HPA_FEPI_GELU, 64, 768, 256, 5, ln=False, rng=np.random.default_rng(1), variant=3)
