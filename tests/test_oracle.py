"""The CPU oracle against the reference's own outputs (tests/golden/, made by
tests/golden/gen_golden.py from the reference sources) and against its own
properties.  These pin the oracle before it is trusted as the GPU checker.

Tolerance: exact (0.0 max-abs).  The oracle is built -O2 -fno-fast-math
-ffp-contract=off like the golden generator, with the reference's arithmetic
order, so any difference is a restatement bug.
"""
import os

import numpy as np
import pytest

import oracle_ctypes as oc
import synth

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name))  # allow_pickle=False (default)


def test_attention_paged_matches_reference_golden():
    g = load("attn_paged_golden.npz")
    for ci in range(int(g["ncases"])):
        B, T, C, NH, off, bs = [int(x) for x in g[f"c{ci}_shape"]]
        out, pre, att = oc.attention_paged(g[f"c{ci}_inp"], g[f"c{ci}_kpool"], g[f"c{ci}_vpool"],
                                           g[f"c{ci}_order"], B, T, C, NH, off, bs)
        assert np.array_equal(out, g[f"c{ci}_out"]), ci
        assert np.array_equal(pre, g[f"c{ci}_preatt"]), ci
        assert np.array_equal(att, g[f"c{ci}_att"]), ci


def test_matmul_forward_and_cached_match_reference_golden():
    g = load("matmul_golden.npz")
    B, T, C, OC = [int(x) for x in g["shape"]]
    L = oc.lib()
    out = np.zeros((B, T, OC), np.float32)
    L.oracle_matmul_forward(oc.fp(out), oc.fp(g["inp"]), oc.fp(g["w"]), oc.fp(g["b"]), B, T, C, OC)
    assert np.array_equal(out, g["fwd"])
    out = np.zeros((B, T, OC), np.float32)
    L.oracle_matmul_cached(oc.fp(out), oc.fp(g["inp"]), oc.fp(g["w"]), oc.fp(g["b"]), B, T, C, OC)
    assert np.array_equal(out, g["cached"])
    # matmul_cached == matmul_forward on Q of every row and K,V of the last row
    # (the reference's test_matmul.c property)
    assert np.array_equal(g["cached"][:, :, :C], g["fwd"][:, :, :C])
    assert np.array_equal(g["cached"][:, -1, C:], g["fwd"][:, -1, C:])


def test_full_forward_matches_reference_train_scratch():
    g = load("forward_golden.npz")
    c = oc.cfg(*[int(x) for x in g["cfg"]])
    logits = oc.gpt2_forward(g["params"], c, g["tokens"])
    assert np.array_equal(logits, g["logits"])


@pytest.mark.parametrize("page_size", [4, 8, 16, 32])
def test_paged_decode_equals_full_recompute(page_size):
    """incremental paged decode (absolute positions, all
    layers, per-sequence permuted block tables) == full recompute, every step."""
    g = load("forward_golden.npz")
    c = oc.cfg(*[int(x) for x in g["cfg"]])
    tokens = g["tokens"]
    B, T = tokens.shape
    d = oc.PagedDecoder(g["params"], c, B, page_size, 64, page_seed=page_size + 1)
    for t in range(T):
        nxt, logits = d.step(tokens[:, t])
        assert np.array_equal(logits, g["logits"][:, t]), t
        assert np.array_equal(nxt, g["logits"][:, t].argmax(-1)), t
    d.close()


@pytest.mark.parametrize("block_size", [1, 2, 5, 8, 16])
def test_paged_equals_contiguous_attention(block_size):
    """test_paged_attn.c's property (paged == contiguous attention), seeded,
    exact, over several page sizes and permuted page placement."""
    rng = np.random.default_rng(block_size)
    B, T, C, NH = 2, 20, 12, 3
    inp = rng.uniform(0, 100, (B, T, 3 * C)).astype(np.float32)
    # the reference test shares pages across b: use b = 0's K/V for all b
    inp[1, :, C:] = inp[0, :, C:]
    npages = (T + block_size - 1) // block_size
    kpool = np.zeros((npages, block_size, C), np.float32)
    vpool = np.zeros((npages, block_size, C), np.float32)
    order = rng.permutation(npages).astype(np.int32)
    for t in range(T):
        kpool[order[t // block_size], t % block_size] = inp[0, t, C:2 * C]
        vpool[order[t // block_size], t % block_size] = inp[0, t, 2 * C:]
    out_p, pre_p, att_p = oc.attention_paged(inp, kpool, vpool, order, B, T, C, NH, 0, block_size)
    out_c = np.zeros((B, T, C), np.float32)
    pre = np.zeros((B, NH, T, T), np.float32)
    att = np.zeros((B, NH, T, T), np.float32)
    oc.lib().oracle_attention_forward(oc.fp(out_c), oc.fp(pre), oc.fp(att), oc.fp(inp), B, T, C, NH)
    assert np.array_equal(out_p, out_c)
    assert np.array_equal(att_p, att)


def test_attention_decode_row_equals_paged_last_row():
    rng = np.random.default_rng(3)
    C, NH, bs, ctx = 64, 4, 8, 37
    npages = (ctx + bs - 1) // bs
    kp = [rng.uniform(-1, 1, (bs, C)).astype(np.float32) for _ in range(npages)]
    vp = [rng.uniform(-1, 1, (bs, C)).astype(np.float32) for _ in range(npages)]
    q = rng.uniform(-1, 1, C).astype(np.float32)
    out = oc.attention_decode(q, kp, vp, ctx, NH)
    # the same row through attention_paged: T = ctx rows at offset 0, row ctx-1
    inp = np.zeros((1, ctx, 3 * C), np.float32)
    inp[0, ctx - 1, :C] = q
    kpool = np.stack(kp)
    vpool = np.stack(vp)
    o2, _, _ = oc.attention_paged(inp, kpool, vpool, np.arange(npages, dtype=np.int32), 1, ctx, C,
                                  NH, 0, bs)
    assert np.array_equal(out, o2[0, ctx - 1])


def test_argmax_first_max_wins():
    x = np.array([0.5, 2.0, -1.0, 2.0, 2.0], np.float32)
    assert oc.lib().oracle_argmax(oc.fp(x), 5) == 1


def test_reference_all_negative_scores_give_zero_output():
    """expsum == 0 branch of paged_infer.c:213: scores below -10000 -> 0."""
    C, NH, bs, ctx = 64, 1, 8, 9
    kp = [np.full((bs, C), 10.0, np.float32) for _ in range(2)]
    vp = [np.ones((bs, C), np.float32) for _ in range(2)]
    q = np.full(C, -1000.0, np.float32)
    out = oc.attention_decode(q, kp, vp, ctx, NH)
    assert np.all(out == 0.0)


def test_oracle_bf16_rounding_matches_numpy_rne():
    """oracle_round_bf16 == round-to-nearest-even on the upper 16 bits (the
    GPU pool's hpa::f32_to_bf16), ties to even included"""
    L = oc.lib()
    xs = np.array([1.0, 1.00390625, 1.01171875, -2.5e-3, 3.14159, 65504.0, 1e-30, -0.0], np.float32)
    u = xs.view(np.uint32).astype(np.uint64)
    want = (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)
    got = np.array([L.oracle_round_bf16(float(x)) for x in xs], np.float32)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_oracle_bf16_kv_decode_is_close_to_fp32():
    """bf16 KV storage perturbs the decode by bf16 rounding only"""
    cfgd = dict(maxT=64, V=300, L=2, NH=2, C=128)
    params = synth.params(cfgd, seed=2)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    a = oc.PagedDecoder(params, c, 3, 8, 64, page_seed=1)
    b = oc.PagedDecoder(params, c, 3, 8, 64, page_seed=1, kv_bf16=True)
    rng = np.random.default_rng(0)
    worst = 0.0
    for _ in range(10):
        tok = rng.integers(0, 300, 3).astype(np.int32)
        _, la = a.step(tok)
        _, lb = b.step(tok)
        worst = max(worst, float(np.abs(la - lb).max()))
    a.close()
    b.close()
    assert 0.0 < worst < 5e-2


@pytest.mark.parametrize("w_bf16", [False, True])
def test_forced_step_on_own_stream_is_the_plain_step(w_bf16):
    """oracle_paged_step_ex fed its own residual stream (embedding, then each
    layer's output) reproduces the plain step bit for bit: the forced input is
    the only thing it changes, so a per-layer GPU check through it measures
    one layer's arithmetic at a time"""
    g = load("forward_golden.npz")
    c = oc.cfg(*[int(x) for x in g["cfg"]])
    params = g["params"]
    tokens = g["tokens"]
    B, T = tokens.shape
    Cn = c.channels
    off = (ctypes_offsets(c))
    wte = params[off[0]:off[0] + c.vocab_size * Cn].reshape(c.vocab_size, Cn)
    wpe = params[off[1]:off[1] + c.max_seq_len * Cn].reshape(c.max_seq_len, Cn)
    a = oc.PagedDecoder(params, c, B, 8, 64, page_seed=3, w_bf16=w_bf16)
    b = oc.PagedDecoder(params, c, B, 8, 64, page_seed=3, w_bf16=w_bf16)
    for t in range(T):
        na, la, outs = a.step_forced(tokens[:, t], None)
        emb = wte[tokens[:, t]] + wpe[t]
        xs = np.concatenate([emb[None], outs], axis=0)
        nb, lb, outs_b = b.step_forced(tokens[:, t], xs)
        assert np.array_equal(la, lb) and np.array_equal(na, nb) and np.array_equal(outs, outs_b), t
        if not w_bf16:
            assert np.array_equal(la, g["logits"][:, t]), t
    a.close()
    b.close()


def ctypes_offsets(c):
    import ctypes
    off = (ctypes.c_size_t * 16)()
    oc.lib().oracle_param_offsets(c, off)
    return [int(x) for x in off]
