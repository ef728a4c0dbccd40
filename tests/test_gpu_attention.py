"""Paged decode attention kernel (hpa_paged_attention_decode) vs the oracle's
restatement of attention_paged (paged_infer.c:163-240) on identical inputs.

Tolerance (BASELINE.json north star): 1e-4 max-abs on the attention output.
Inputs: K/V ~ U(-1,1), q ~ U(-2,2); pages handed out in a random permutation
so every block table is non-contiguous; ragged context lengths that cross
tile (64) and page boundaries.
"""
import numpy as np
import pytest

import oracle_ctypes as oc

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _run_case(hip, P, ctxs, NH, waves=4, seed=0, q_scale=2.0, kv=None, splits=0, bf16=False, repeat=1):
    rng = np.random.default_rng(seed)
    L = hip.lib()
    C = NH * 64
    B = len(ctxs)
    maxp = max((c + P - 1) // P for c in ctxs)
    num_pages = B * maxp + 3
    pool = hip.Pool(1, NH, P, num_pages, dtype=hip.HPA_BF16 if bf16 else hip.HPA_F32)
    perm = rng.permutation(num_pages).astype(np.int32)
    bt = np.full((B, maxp), -1, np.int32)
    ks, vs = [], []
    k_next = 0
    for b, ctx in enumerate(ctxs):
        n = (ctx + P - 1) // P
        bt[b, :n] = perm[k_next:k_next + n]
        k_next += n
        if kv is None:
            k = rng.uniform(-1, 1, (ctx, C)).astype(np.float32)
            v = rng.uniform(-1, 1, (ctx, C)).astype(np.float32)
        else:
            k, v = kv(ctx, C)
        if bf16:  # the values a bf16 pool stores; the oracle sees exactly these
            k, v = hip.round_bf16(k), hip.round_bf16(v)
        pool.write_tokens(0, bt[b, :n], k, v)
        ks.append(k)
        vs.append(v)
    q = rng.uniform(-q_scale, q_scale, (B, C)).astype(np.float32)
    pos = np.array([c - 1 for c in ctxs], np.int32)
    d_q = hip.DeviceBuffer.from_array(q)
    d_bt = hip.DeviceBuffer.from_array(bt)
    d_pos = hip.DeviceBuffer.from_array(pos)
    if splits:  # split-context form, frag output, repeated launches over one workspace
        Mp = (B + 15) // 16 * 16
        d_out = hip.DeviceBuffer(Mp * C * 4)
        wsb = L.hpa_attn_ws_bytes(B, NH, splits)
        d_ws = hip.DeviceBuffer(max(wsb, 4))
        hip.check(L.hpa_memset_async(d_ws.ptr, 0, wsb))
        hip.check(L.hpa_set_attention_waves(waves))
        outs = []
        for _ in range(repeat):
            hip.check(L.hpa_paged_attention_decode_split(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr,
                                                         B, splits, d_ws.ptr if wsb else None, 1), "split attention")
            hip.check(L.hpa_synchronize())
            outs.append(hip.from_frag(d_out.download(Mp * C), B, C))
        hip.check(L.hpa_set_attention_waves(0))  # back to the callers' choice
        for o in outs[1:]:  # fixed merge order: bit-identical every launch
            assert np.array_equal(o, outs[0])
        # the counters are left zero for the next launch
        cnt = d_ws.download(B * NH, np.int32, offset=B * NH * splits * 68 * 4) if wsb else np.zeros(1)
        assert not cnt.any()
        out = outs[0]
    else:
        d_out = hip.DeviceBuffer(q.nbytes)
        hip.check(L.hpa_set_attention_waves(waves))
        hip.check(L.hpa_paged_attention_decode(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr, B))
        hip.check(L.hpa_synchronize())
        hip.check(L.hpa_set_attention_waves(0))  # back to the callers' choice
        out = d_out.download((B, C))
    ref = np.zeros_like(out)
    for b, ctx in enumerate(ctxs):
        n = (ctx + P - 1) // P
        kp = [np.zeros((P, C), np.float32) for _ in range(n)]
        vp = [np.zeros((P, C), np.float32) for _ in range(n)]
        for t in range(ctx):
            kp[t // P][t % P] = ks[b][t]
            vp[t // P][t % P] = vs[b][t]
        ref[b] = oc.attention_decode(q[b], kp, vp, ctx, NH)
    return out, ref


@pytest.mark.parametrize("P", [8, 16, 32])
def test_decode_attention_ragged(hip, P):
    ctxs = [1, 2, 5, 63, 64, 65, 127, 200, 257, 1024]
    out, ref = _run_case(hip, P, ctxs, NH=3, seed=P)
    err = np.abs(out - ref).max()
    assert err <= TOL, err


@pytest.mark.parametrize("waves", [1, 2, 4, 8])
def test_decode_attention_waves(hip, waves):
    out, ref = _run_case(hip, 16, [1, 70, 333, 1000], NH=2, waves=waves, seed=11)
    assert np.abs(out - ref).max() <= TOL


def test_decode_attention_peaked_softmax(hip):
    """large q: softmax concentrated on few keys (exercises the online max
    rescaling across tiles and waves)"""
    out, ref = _run_case(hip, 16, [300, 999, 64], NH=2, seed=5, q_scale=40.0)
    assert np.abs(out - ref).max() <= TOL


def test_decode_attention_all_scores_below_reference_floor(hip):
    """every score < -10000: the reference's expsum == 0 branch gives 0"""

    def kv(ctx, C):
        return np.full((ctx, C), 10.0, np.float32), np.ones((ctx, C), np.float32)

    rng_q = -1000.0
    ctxs = [5, 80]
    out, ref = _run_case(hip, 16, ctxs, NH=1, seed=1, kv=kv, q_scale=1e-6)
    assert np.abs(out - ref).max() <= TOL
    # and with an explicitly hugely negative q
    L = hip.lib()
    P, NH, C = 16, 1, 64
    pool = hip.Pool(1, NH, P, 8)
    k, v = kv(40, C)
    pool.write_tokens(0, [3, 1, 6], k, v)
    q = np.full((1, C), rng_q, np.float32)
    d_q = hip.DeviceBuffer.from_array(q)
    d_bt = hip.DeviceBuffer.from_array(np.array([[3, 1, 6]], np.int32))
    d_pos = hip.DeviceBuffer.from_array(np.array([39], np.int32))
    d_out = hip.DeviceBuffer(q.nbytes)
    hip.check(L.hpa_paged_attention_decode(d_q.ptr, pool.ref, 0, d_bt.ptr, 3, d_pos.ptr, d_out.ptr, 1))
    assert np.all(d_out.download((1, C)) == 0.0)


def test_decode_attention_full_size_subset_and_determinism(hip):
    """BASELINE config 2 shape (B=64, NH=12, ctx 1024, page 16): random fill
    through the library, a sample of sequences checked against the oracle,
    and two launches bit-identical."""
    L = hip.lib()
    B, NH, P, ctx = 64, 12, 16, 1024
    C = NH * 64
    maxp = ctx // P
    pool = hip.Pool(1, NH, P, B * maxp)
    rng = np.random.default_rng(7)
    bt = rng.permutation(B * maxp).astype(np.int32).reshape(B, maxp)
    d_bt = hip.DeviceBuffer.from_array(bt)
    hip.check(L.hpa_pool_fill_random(pool.ref, d_bt.ptr, maxp, B, ctx, 1234))
    q = rng.uniform(-2, 2, (B, C)).astype(np.float32)
    pos = np.full(B, ctx - 1, np.int32)
    d_q = hip.DeviceBuffer.from_array(q)
    d_pos = hip.DeviceBuffer.from_array(pos)
    d_out = hip.DeviceBuffer(q.nbytes)
    hip.check(L.hpa_paged_attention_decode(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr, B))
    o1 = d_out.download((B, C))
    hip.check(L.hpa_paged_attention_decode(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr, B))
    o2 = d_out.download((B, C))
    assert np.array_equal(o1, o2)
    assert np.isfinite(o1).all()
    for b in (0, 17, 63):
        k, v = pool.read_tokens(0, bt[b], ctx)
        kp = [k[i * P:(i + 1) * P].copy() for i in range(maxp)]
        vp = [v[i * P:(i + 1) * P].copy() for i in range(maxp)]
        ref = oc.attention_decode(q[b], kp, vp, ctx, NH)
        assert np.abs(o1[b] - ref).max() <= TOL


@pytest.mark.parametrize("P", [8, 16, 32])
@pytest.mark.parametrize("splits", [1, 2, 3, 4, 8, 16])
def test_split_context_attention(hip, P, splits):
    """flash-decoding form: each (sequence, head) cut into
    `splits` context ranges, merged by the last range in range order; ragged
    contexts leave ranges empty (ctx 1, 2), repeated launches are bit-identical
    and leave the arrival counters zero"""
    ctxs = [1, 2, 5, 63, 64, 65, 200, 257, 1024]
    out, ref = _run_case(hip, P, ctxs, NH=3, seed=P + splits, splits=splits, repeat=3)
    assert np.abs(out - ref).max() <= TOL


@pytest.mark.parametrize("waves", [1, 2, 8])
def test_split_context_attention_waves(hip, waves):
    out, ref = _run_case(hip, 16, [1, 70, 333, 1000], NH=2, waves=waves, seed=13, splits=4, repeat=2)
    assert np.abs(out - ref).max() <= TOL


def test_split_context_attention_floor_and_peaked(hip):
    """every score below the -10000 floor (zero output, as the reference) and a
    peaked softmax, across ranges"""
    def kv(ctx, C):
        return np.full((ctx, C), 10.0, np.float32), np.ones((ctx, C), np.float32)

    out, ref = _run_case(hip, 16, [5, 80, 300], NH=1, seed=1, kv=kv, q_scale=1e-6, splits=4)
    assert np.abs(out - ref).max() <= TOL
    out, ref = _run_case(hip, 16, [300, 999, 64], NH=2, seed=5, q_scale=40.0, splits=8)
    assert np.abs(out - ref).max() <= TOL


@pytest.mark.parametrize("splits", [2, 4, 8])
def test_split_context_attention_bf16_pool(hip, splits):
    ctxs = [1, 2, 7, 63, 64, 65, 200, 257, 1024]
    out, ref = _run_case(hip, 8, ctxs, NH=3, seed=splits, bf16=True, splits=splits, repeat=2)
    assert np.abs(out - ref).max() <= TOL


@pytest.mark.parametrize("B", [8, 16, 32])
def test_split_context_attention_strong_scaling_shapes(hip, B):
    """the per-GPU batches of the metric's B = 64 at 8/4/2 GPUs (GPT-2 124M,
    ctx 1024, page 16) at the engine's split count: every sequence vs the
    oracle on a head subset, bit-identical on relaunch"""
    L = hip.lib()
    NH, P, ctx = 12, 16, 1024
    C = NH * 64
    S = L.hpa_attn_pick_splits(B, NH, ctx, 256)
    assert S == {8: 2, 16: 1, 32: 2}[B]
    maxp = ctx // P
    pool = hip.Pool(1, NH, P, B * maxp)
    rng = np.random.default_rng(B)
    bt = rng.permutation(B * maxp).astype(np.int32).reshape(B, maxp)
    d_bt = hip.DeviceBuffer.from_array(bt)
    hip.check(L.hpa_pool_fill_random(pool.ref, d_bt.ptr, maxp, B, ctx, 99))
    q = rng.uniform(-2, 2, (B, C)).astype(np.float32)
    pos = np.full(B, ctx - 1, np.int32)
    pos[::3] = rng.integers(0, ctx, len(pos[::3]))  # ragged
    d_q = hip.DeviceBuffer.from_array(q)
    d_pos = hip.DeviceBuffer.from_array(pos)
    Mp = (B + 15) // 16 * 16
    d_out = hip.DeviceBuffer(Mp * C * 4)
    wsb = L.hpa_attn_ws_bytes(B, NH, S)
    d_ws = hip.DeviceBuffer(max(wsb, 4))
    hip.check(L.hpa_memset_async(d_ws.ptr, 0, wsb))
    outs = []
    for _ in range(2):
        hip.check(L.hpa_paged_attention_decode_split(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr, B,
                                                     S, d_ws.ptr if wsb else None, 1))
        outs.append(hip.from_frag(d_out.download(Mp * C), B, C))
    assert np.array_equal(outs[0], outs[1])
    for b in range(B):
        n = int(pos[b]) + 1
        k, v = pool.read_tokens(0, bt[b], n)
        np_ = (n + P - 1) // P
        kp = [np.zeros((P, C), np.float32) for _ in range(np_)]
        vp = [np.zeros((P, C), np.float32) for _ in range(np_)]
        for i in range(np_):
            m = min(P, n - i * P)
            kp[i][:m] = k[i * P:i * P + m]
            vp[i][:m] = v[i * P:i * P + m]
        ref = oc.attention_decode(q[b], kp, vp, n, NH)
        assert np.abs(outs[0][b] - ref).max() <= TOL, b


@pytest.mark.parametrize("P", [8, 16, 32])
@pytest.mark.parametrize("waves", [1, 4, 8])
def test_bf16_pool_attention(hip, P, waves):
    """bf16 KV storage (BASELINE config 5), fp32 arithmetic: exact same
    K/V values on both sides, so the fp32 1e-4 bar holds"""
    ctxs = [1, 2, 7, 63, 64, 65, 200, 257, 1024]
    out, ref = _run_case(hip, P, ctxs, NH=3, seed=P + waves, waves=waves, bf16=True)
    assert np.abs(out - ref).max() <= TOL


def test_bf16_pool_roundtrip(hip):
    rng = np.random.default_rng(1)
    pool = hip.Pool(2, 2, 8, 6, dtype=hip.HPA_BF16)
    k = rng.standard_normal((13, 128)).astype(np.float32)
    v = rng.standard_normal((13, 128)).astype(np.float32)
    pool.write_tokens(1, [4, 1], k, v)
    k2, v2 = pool.read_tokens(1, [4, 1], 13)
    assert np.array_equal(k2, hip.round_bf16(k)) and np.array_equal(v2, hip.round_bf16(v))
