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


def _run_case(hip, P, ctxs, NH, waves=4, seed=0, q_scale=2.0, kv=None, chunks=0, bf16=False):
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
    if chunks:  # context chunks with carried softmax state (the pipelined decode)
        import ctypes
        Mp = (B + 15) // 16 * 16
        d_out = hip.DeviceBuffer(Mp * C * 4)
        d_state = hip.DeviceBuffer(L.hpa_attn_state_elems(B, NH) * 4)
        a = hip.HpaAttnChunk(q=d_q.ptr, pool=ctypes.addressof(pool.s), layer=0, block_table=d_bt.ptr,
                             bt_stride=maxp, pos=d_pos.ptr, state=d_state.ptr, out_frag=d_out.ptr, B=B,
                             nchunks=chunks)
        for c in range(chunks):
            a.chunk = c
            hip.check(L.hpa_attn_chunk_with_gemm(ctypes.byref(a), None), "attn chunk")
        hip.check(L.hpa_synchronize())
        out = hip.from_frag(d_out.download(Mp * C), B, C)
    else:
        d_out = hip.DeviceBuffer(q.nbytes)
        hip.check(L.hpa_set_attention_waves(waves))
        hip.check(L.hpa_paged_attention_decode(d_q.ptr, pool.ref, 0, d_bt.ptr, maxp, d_pos.ptr, d_out.ptr, B))
        hip.check(L.hpa_synchronize())
        hip.check(L.hpa_set_attention_waves(4))
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
@pytest.mark.parametrize("chunks", [1, 3, 4])
def test_chunked_attention_with_carried_state(hip, P, chunks):
    """the pipelined decode's attention: context chunks in separate launches,
    (m, l, acc) carried through memory; ctx 1 and 2 leave most chunks empty"""
    ctxs = [1, 2, 5, 63, 64, 65, 200, 257, 1024]
    out, ref = _run_case(hip, P, ctxs, NH=3, seed=P + chunks, chunks=chunks)
    assert np.abs(out - ref).max() <= TOL


def test_chunked_attention_all_scores_below_reference_floor(hip):
    def kv(ctx, C):
        return np.full((ctx, C), 10.0, np.float32), np.ones((ctx, C), np.float32)

    out, ref = _run_case(hip, 16, [5, 80, 300], NH=1, seed=1, kv=kv, q_scale=1e-6, chunks=4)
    assert np.abs(out - ref).max() <= TOL


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
