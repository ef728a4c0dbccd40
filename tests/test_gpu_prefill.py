"""Prefill: the multi-query causal paged attention on
MFMA and the engine's one-pass prefill, against the oracle.

* attention: every query row (b, t) of a prefill block must equal the
  oracle's attention_paged arithmetic for one query at position start[b]+t
  over keys 0..start[b]+t (tolerance 1e-4, the north-star bar);
* engine: gpt2_decode_prefill(T tokens) must equal T token-by-token decode
  steps of the oracle with the same tokens (logits 2e-4 as the decode tests;
  greedy ids bit-exact where the top-2 margin exceeds 1e-3), and decode must
  continue from it.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu
TOL = 1e-4
LOGIT_TOL = 2e-4
TIE_MARGIN = 1e-3
SMALL = dict(maxT=256, V=1000, L=2, NH=2, C=128)


def _attn_case(hip, P, starts, T, NH, bf16=False, seed=0):
    rng = np.random.default_rng(seed)
    L = hip.lib()
    C = NH * 64
    B = len(starts)
    ctxs = [s + T for s in starts]
    maxp = max((c + P - 1) // P for c in ctxs)
    num_pages = B * maxp + 2
    pool = hip.Pool(1, NH, P, num_pages, dtype=hip.HPA_BF16 if bf16 else hip.HPA_F32)
    perm = rng.permutation(num_pages).astype(np.int32)
    bt = np.full((B, maxp), -1, np.int32)
    ks, vs, k_next = [], [], 0
    for b, ctx in enumerate(ctxs):
        n = (ctx + P - 1) // P
        bt[b, :n] = perm[k_next:k_next + n]
        k_next += n
        k = rng.uniform(-1, 1, (ctx, C)).astype(np.float32)
        v = rng.uniform(-1, 1, (ctx, C)).astype(np.float32)
        if bf16:
            k, v = hip.round_bf16(k), hip.round_bf16(v)
        pool.write_tokens(0, bt[b, :n], k, v)
        ks.append(k)
        vs.append(v)
    q = rng.uniform(-2, 2, (B * T, C)).astype(np.float32)
    R = B * T
    Rp = (R + 15) // 16 * 16
    d_q = hip.DeviceBuffer.from_array(q)
    d_bt = hip.DeviceBuffer.from_array(bt)
    d_start = hip.DeviceBuffer.from_array(np.array(starts, np.int32))
    d_out = hip.DeviceBuffer(Rp * C * 4)
    import ctypes
    F = ctypes.POINTER(ctypes.c_float)
    I = ctypes.POINTER(ctypes.c_int)
    hip.check(L.hpa_paged_attention_prefill(ctypes.cast(d_q.ptr, F), ctypes.addressof(pool.s), 0,
                                            ctypes.cast(d_bt.ptr, I), maxp, ctypes.cast(d_start.ptr, I), B, T,
                                            ctypes.cast(d_out.ptr, F)), "prefill attention")
    hip.check(L.hpa_synchronize())
    out = hip.from_frag(d_out.download(Rp * C), R, C)
    worst = 0.0
    for b in range(B):
        n = (ctxs[b] + P - 1) // P
        kp = [np.zeros((P, C), np.float32) for _ in range(n)]
        vp = [np.zeros((P, C), np.float32) for _ in range(n)]
        for t in range(ctxs[b]):
            kp[t // P][t % P] = ks[b][t]
            vp[t // P][t % P] = vs[b][t]
        for t in range(T):
            ref = oc.attention_decode(q[b * T + t], kp, vp, starts[b] + t + 1, NH)
            worst = max(worst, float(np.abs(out[b * T + t] - ref).max()))
    return worst


@pytest.mark.parametrize("P", [8, 16, 32])
def test_prefill_attention_matches_oracle(hip, P):
    """ragged starts (fresh, mid-page, past a 64-token block), T not a
    multiple of 64 or 16"""
    assert _attn_case(hip, P, [0, 5, 70], 83, NH=3, seed=P) <= TOL


def test_prefill_attention_bf16_pool(hip):
    assert _attn_case(hip, 16, [0, 17], 50, NH=2, bf16=True, seed=3) <= TOL


def test_prefill_attention_single_token(hip):
    """T = 1 is a decode step through the prefill kernel"""
    assert _attn_case(hip, 16, [0, 100, 255], 1, NH=2, seed=5) <= TOL


def _margins(logits):
    s = np.sort(logits, axis=-1)
    return s[:, -1] - s[:, -2]


def _run(hip, cfgd, B, P, T, seed, pre_steps=0, post_steps=8, graph=False, kv_bf16=False, tol=LOGIT_TOL,
         w_bf16=False, tie=TIE_MARGIN):
    params = synth.params(cfgd, seed=seed)
    model = hip.Model(cfgd, params=params)
    model.decode_init(B, P, cfgd["maxT"], kv_dtype=hip.HPA_BF16 if kv_bf16 else hip.HPA_F32,
                      w_dtype=hip.HPA_BF16 if w_bf16 else hip.HPA_F32)
    model.set_graph(graph)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    orc = oc.PagedDecoder(params, c, B, P, cfgd["maxT"], page_seed=seed + 1, kv_bf16=kv_bf16, w_bf16=w_bf16)
    rng = np.random.default_rng(seed)
    worst = 0.0

    def check(g_next, o_next, o_logits):
        nonlocal worst
        worst = max(worst, float(np.abs(model.logits() - o_logits).max()))
        clear = _margins(o_logits) > tie
        assert np.array_equal(g_next[clear], o_next[clear])

    for _ in range(pre_steps):  # decode steps before the prefill (prefill at a nonzero start)
        tok = rng.integers(0, cfgd["V"], B).astype(np.int32)
        o_next, o_logits = orc.step(tok)
        check(model.step(tok), o_next, o_logits)
    toks = rng.integers(0, cfgd["V"], (B, T)).astype(np.int32)
    for t in range(T):
        o_next, o_logits = orc.step(toks[:, t])
    check(model.prefill(toks), o_next, o_logits)
    assert np.array_equal(model.positions(), np.full(B, pre_steps + T, np.int32))
    tok = o_next
    for _ in range(post_steps):  # decode continues from the prefilled pages, greedy fed back
        o_next, o_logits = orc.step(tok)
        check(model.step(tok), o_next, o_logits)
        tok = o_next
    assert worst <= tol, worst
    model.close()
    orc.close()
    return worst


@pytest.mark.parametrize("P,T", [(16, 37), (8, 64), (32, 130)])
def test_prefill_then_decode_matches_oracle(hip, P, T):
    _run(hip, SMALL, B=4, P=P, T=T, seed=P + T)


def test_prefill_after_decode_steps(hip):
    _run(hip, SMALL, B=3, P=16, T=45, seed=9, pre_steps=7, graph=True)


def test_prefill_twice(hip):
    """two prefills back to back (chunked prefill) equal one long one"""
    params = synth.params(SMALL, seed=2)
    outs = []
    for chunks in ([60], [25, 35]):
        m = hip.Model(SMALL, params=params)
        m.decode_init(3, 16, SMALL["maxT"])
        toks = np.random.default_rng(2).integers(0, SMALL["V"], (3, 60)).astype(np.int32)
        t0 = 0
        for n in chunks:
            nxt = m.prefill(toks[:, t0:t0 + n])
            t0 += n
        outs.append((nxt, m.logits()))
        m.close()
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.abs(outs[0][1] - outs[1][1]).max() <= LOGIT_TOL


def test_prefill_gpt2_124m_shapes(hip):
    cfgd = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    worst = _run(hip, cfgd, B=2, P=16, T=70, seed=4, post_steps=4)
    print(f"124M prefill: worst logit diff {worst:.3e}")


def test_prefill_bf16_kv(hip):
    _run(hip, SMALL, B=3, P=16, T=50, seed=6, kv_bf16=True, tol=5e-3)


@pytest.mark.parametrize("B,T", [(3, 50), (4, 40)])
def test_prefill_bf16_weights(hip, B, T):
    """bf16 weights: B*T rows through the bf16 GEMMs (looped and, at B*T > 112
    rows, the A-resident kernel) against the oracle's bf16-weights decode
    (tolerance as test_gpu_decode.py BF16W_*)"""
    _run(hip, SMALL, B=B, P=16, T=T, seed=8 + B, w_bf16=True, kv_bf16=True, tol=2e-2, tie=4e-2)


def test_prefill_rejects_overflow(hip):
    m = hip.Model(SMALL)
    m.decode_init(2, 16, 64)
    with pytest.raises(RuntimeError):
        m.prefill(np.zeros((2, 65), np.int32))
    m.close()
