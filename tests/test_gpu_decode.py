"""End-to-end decode on the MI355X path (gpt2_decode_*) vs the oracle's
paged incremental decode (absolute positions, all L layers; the oracle is
pinned bit-exact to the reference's full-L forward in test_oracle.py).

Tolerances: logits <= 2e-4 max-abs (fp32, different summation order: MFMA
k-chains + parallel LN reductions vs the reference's sequential dots).
Greedy ids bit-exact on every row except where the oracle's top-2 logit
margin is within 2x the measured max |logit difference| of that run (a
genuine near-tie: an order-of-summation difference of that size can flip
it); the exempt rows are counted, printed and asserted to be few.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu
LOGIT_TOL = 2e-4

SMALL = dict(maxT=128, V=1000, L=2, NH=2, C=128)
GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)


def _margins(logits):
    s = np.sort(logits, axis=-1)
    return s[:, -1] - s[:, -2]


class IdCheck:
    """greedy ids vs the oracle's, with the near-tie rule above"""

    def __init__(self):
        self.rows = []  # (oracle margins, ids equal) per step
        self.worst = 0.0

    def add(self, g_logits, o_logits, g_next, o_next):
        self.worst = max(self.worst, float(np.abs(g_logits - o_logits).max()))
        self.rows.append((_margins(o_logits), np.asarray(g_next) == np.asarray(o_next)))

    def verify(self, tol, max_exempt_frac=0.02):
        tie = 2.0 * self.worst
        exempt = total = 0
        for margin, same in self.rows:
            clear = margin > tie
            assert same[clear].all(), (margin[clear & ~same], tie)
            exempt += int((~clear).sum())
            total += len(margin)
        print(f"max |logit diff| {self.worst:.3e}; tie margin {tie:.3e}; exempt rows {exempt}/{total}")
        assert self.worst <= tol, self.worst
        assert exempt <= max(1, max_exempt_frac * total), (exempt, total)
        return exempt


def _compare_run(hip, cfgd, B, P, steps, seed, graph=False, feed_greedy=False, kv_bf16=False, tol=LOGIT_TOL,
                 w_bf16=False, splits=0, max_exempt_frac=0.02):
    params = synth.params(cfgd, seed=seed)
    model = hip.Model(cfgd, params=params)
    model.decode_init(B, P, cfgd["maxT"], kv_dtype=hip.HPA_BF16 if kv_bf16 else hip.HPA_F32,
                      w_dtype=hip.HPA_BF16 if w_bf16 else hip.HPA_F32)
    if splits:
        assert model.set_attn_splits(splits) == splits
    model.set_graph(graph)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    orc = oc.PagedDecoder(params, c, B, P, cfgd["maxT"], page_seed=seed + 3, kv_bf16=kv_bf16, w_bf16=w_bf16)
    rng = np.random.default_rng(seed)
    tok = rng.integers(0, cfgd["V"], B).astype(np.int32)
    chk = IdCheck()
    for t in range(steps):
        o_next, o_logits = orc.step(tok)
        g_next = model.step(tok)
        chk.add(model.logits(), o_logits, g_next, o_next)
        tok = o_next if feed_greedy else rng.integers(0, cfgd["V"], B).astype(np.int32)
    ties = chk.verify(tol, max_exempt_frac)
    assert np.array_equal(model.positions(), np.full(B, steps, np.int32))
    model.close()
    orc.close()
    return chk.worst, ties


@pytest.mark.parametrize("P", [8, 16, 32])
def test_decode_small_model_matches_oracle(hip, P):
    _compare_run(hip, SMALL, B=3, P=P, steps=70, seed=P)


@pytest.mark.parametrize("splits", [2, 8, 16])
def test_decode_with_split_context_attention_matches_oracle(hip, splits):
    """the engine with its attention's context cut into ranges (the strong-
    scaling shapes' path), graph replay, contexts crossing many ranges"""
    _compare_run(hip, SMALL, B=4, P=16, steps=100, seed=80 + splits, graph=True, splits=splits)


def test_decode_batch_over_64_rows(hip):
    """B > 64: two 64-row groups in every GEMM, padded rows in the second"""
    _compare_run(hip, SMALL, B=70, P=16, steps=12, seed=70)


def test_decode_graph_replay_matches_oracle_greedy(hip):
    _compare_run(hip, SMALL, B=5, P=16, steps=40, seed=9, graph=True, feed_greedy=True)


def test_graph_and_eager_bit_identical(hip):
    params = synth.params(SMALL, seed=4)
    outs = []
    for graph in (False, True):
        m = hip.Model(SMALL, params=params)
        m.decode_init(4, 16, 128)
        m.set_graph(graph)
        rng = np.random.default_rng(0)
        seq = []
        for _ in range(20):
            seq.append(m.step(rng.integers(0, 1000, 4).astype(np.int32)))
        seq.append(m.logits())
        outs.append(seq)
        m.close()
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_decode_gpt2_124m_shapes(hip):
    """GPT-2 124M shapes (L=12, C=768, NH=12, V=50257), B=4, 24 steps"""
    worst, ties = _compare_run(hip, GPT2_124M, B=4, P=16, steps=24, seed=21)
    print(f"124M: worst logit diff {worst:.3e}, near-ties {ties}")


def test_device_greedy_feedback(hip):
    """tokens=None feeds the device-side argmax ids back without a host
    round trip; must equal feeding the same ids from the host"""
    params = synth.params(SMALL, seed=12)
    m1 = hip.Model(SMALL, params=params)
    m1.decode_init(3, 16, 128)
    m2 = hip.Model(SMALL, params=params)
    m2.decode_init(3, 16, 128)
    first = np.array([1, 2, 3], np.int32)
    a = m1.step(first)
    b = m2.step(first)
    for _ in range(10):
        a = m1.step(None)
        b = m2.step(b)
        assert np.array_equal(a, b)


def test_fill_random_then_decode_is_finite(hip):
    m = hip.Model(SMALL)
    m.decode_init(8, 16, 128)
    m.fill_random(100, seed=3)
    assert np.array_equal(m.positions(), np.full(8, 100, np.int32))
    nxt = m.step(np.arange(8, dtype=np.int32))
    assert np.isfinite(m.logits()).all()
    assert nxt.min() >= 0 and nxt.max() < 1000
    tot, att = m.step_bytes()
    assert att > 0 and tot > att
    m.close()


def test_context_full_is_an_error(hip):
    m = hip.Model(SMALL)
    m.decode_init(2, 16, 20)
    for _ in range(20):
        m.step(np.zeros(2, np.int32))
    with pytest.raises(RuntimeError):
        m.step(np.zeros(2, np.int32))
    m.close()


def test_decode_xl_width_matches_oracle(hip):
    """GPT-2 XL layer shapes (C=1600, NH=25 -> K/16 = 100 and 400: the looped
    GEMM path; page 32 as BASELINE config 3) on a 2-layer model"""
    cfgd = dict(maxT=128, V=1000, L=2, NH=25, C=1600)
    worst, ties = _compare_run(hip, cfgd, B=20, P=32, steps=20, seed=33, graph=True)
    print(f"XL width: worst logit diff {worst:.3e}, near-ties {ties}")


# bf16 KV: the GPU and the oracle round their own fp32 K/V (which differ by
# ~1e-6) to bf16, so an element within 1e-6 of a rounding boundary can land on
# the neighbouring bf16 value on one side; the logit bar is widened for that
# (the attention kernel itself keeps 1e-4 on identical
# inputs, test_gpu_attention.py::test_bf16_pool_attention)
BF16_LOGIT_TOL = 5e-3  # measured 2.6e-3 at 124M shapes (12 layers amplify single-ulp flips)
# bf16 rounding of values that differ by fp32 summation order flips single
# bf16 ulps on one side only, so near-ties are far more common than in fp32
# (measured 4/96 rows exempt with bf16 KV at 124M, 56/800 with bf16 weights
# on the small model, 18/96 with bf16 weights + KV at 124M): the exempt share
# is bounded at 25 % here, 2 % for fp32.  These runs compound the flips over
# all layers; the per-layer pinned runs (test_gpu_configs.py
# test_config5_layer_pinned_full_context: each layer on the GPU's own input)
# hold bf16 ids to the fp32 2 % bar.
BF16_EXEMPT = 0.25


@pytest.mark.parametrize("P", [8, 16])
def test_decode_bf16_kv_matches_oracle(hip, P):
    _compare_run(hip, SMALL, B=20, P=P, steps=50, seed=40 + P, graph=True, kv_bf16=True, tol=BF16_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)


def test_decode_bf16_kv_124m_shapes(hip):
    cfgd = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    worst, ties = _compare_run(hip, cfgd, B=8, P=8, steps=12, seed=7, graph=True, kv_bf16=True,
                               tol=BF16_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)
    print(f"124M bf16 KV: worst logit diff {worst:.3e}, near-ties {ties}")


def test_bf16_kv_guards(hip):
    m = hip.Model(SMALL)
    m.decode_init(40, 16, 64, kv_dtype=hip.HPA_BF16)
    m.fill_random(30, seed=2)
    m.step(np.zeros(40, np.int32))
    assert np.isfinite(m.logits()).all()
    tot, att = m.step_bytes()
    assert att == 2.0 * SMALL["L"] * 40 * 32 * SMALL["C"] * 2  # ctx = pos + 1 = 32; 2 bytes per element
    m.close()


@pytest.mark.parametrize("cfg_name,B,steps", [("small", 6, 30), ("124m", 4, 8)])
def test_sampling_matches_reference_sampler(hip, cfg_name, B, steps):
    """device multinomial sampling == the reference's softmax_forward +
    sample_mult with random_f32 coins (oracle) on the same logits, stream
    b seeded 1337 + b; sampled ids fed back on the device"""
    cfgd = SMALL if cfg_name == "small" else dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    m = hip.Model(cfgd, params=synth.params(cfgd, seed=3))
    m.decode_init(B, 16, cfgd["maxT"])
    m.set_sampling(True, seed=1337)
    m.set_graph(True)
    sampler = oc.Sampler(B, seed=1337)
    tok = np.random.default_rng(1).integers(0, cfgd["V"], B).astype(np.int32)
    seen = set()
    for s in range(steps):
        g = m.step(tok if s == 0 else None)
        want = sampler.sample(m.logits())
        assert np.array_equal(g, want), (s, g, want)
        seen.update(int(x) for x in g)
    assert len(seen) > B  # a multinomial draw, not a greedy one
    m.close()


def test_sampling_off_is_greedy(hip):
    m = hip.Model(SMALL, params=synth.params(SMALL, seed=3))
    m.decode_init(3, 16, 64)
    m.set_sampling(True, seed=5)
    m.set_sampling(False)
    g = m.step(np.array([1, 2, 3], np.int32))
    assert np.array_equal(g, m.logits().argmax(-1))
    m.close()


# bf16 weights ("bf16 decode", gpt2_decode_init_w): the GPU and the oracle both
# round the GEMM weights and the GEMM input rows (after LN / attention / GELU)
# to bf16 and sum in fp32.  The weights round identically; an input row is
# rounded from fp32 values that differ by ~1e-6 (summation order), so an
# element within that of a bf16 rounding boundary lands one bf16 ulp
# (2^-8 relative) apart -- the same effect as the bf16 KV case, in more
# places; the bar and the tie margin are widened for it.
BF16W_LOGIT_TOL = 2e-2


@pytest.mark.parametrize("P", [8, 16])
def test_decode_bf16_weights_matches_oracle(hip, P):
    worst, ties = _compare_run(hip, SMALL, B=20, P=P, steps=40, seed=60 + P, graph=True, w_bf16=True,
                               tol=BF16W_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)
    print(f"bf16 weights (small): worst logit diff {worst:.3e}, near-ties {ties}")


def test_decode_bf16_weights_and_kv_124m_shapes(hip):
    """BASELINE config 5's numerics (bf16 weights + bf16 KV) at 124M shapes"""
    cfgd = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    worst, ties = _compare_run(hip, cfgd, B=8, P=8, steps=10, seed=9, graph=True, kv_bf16=True, w_bf16=True,
                               tol=BF16W_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)
    print(f"124M bf16 weights + KV: worst logit diff {worst:.3e}, near-ties {ties}")


def test_decode_bf16_weights_batch_over_64_rows(hip):
    """several row groups per GEMM (M = 80: 5 row blocks, row_blocks falls back to 1)"""
    _compare_run(hip, SMALL, B=80, P=16, steps=6, seed=71, graph=False, w_bf16=True,
                 tol=BF16W_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)


def test_bf16_weights_guards(hip):
    m = hip.Model(SMALL)
    m.decode_init(40, 16, 64, w_dtype=hip.HPA_BF16)
    tot, _ = m.step_bytes()
    tot32 = None
    m.close()
    m = hip.Model(SMALL)
    m.decode_init(40, 16, 64)
    tot32, _ = m.step_bytes()
    C, L, V = SMALL["C"], SMALL["L"], SMALL["V"]
    assert tot32 - tot == 2.0 * (L * 12 * C * C + V * C)  # weight matrices at 2 bytes instead of 4
    m.close()
