"""The persistent decode layer (hpa_layer.hip: attention -> attproj -> fc ->
fcproj -> next qkv as one launch per layer) against the five-launch layer and
the oracle.

* Decode parity vs the oracle runs through every test of test_gpu_decode.py /
  test_gpu_configs.py, where the persistent layer is the engine's default for
  B <= 64; here the two engine paths are compared directly at GPT-2 124M
  shapes with ~1000-token contexts (the bench's regime), at batches 64, 32,
  16 and 8 (split counts 1, 2, 4, 8), fp32 and bf16 pools.
* Tolerance: the qkv and fc rows are bit-identical to the launch path by
  construction (same per-row summation order); attproj / fcproj are summed
  over K parts here (4 partial tiles added in part order) instead of 4 or 8
  waves, so logits differ by fp32 reassociation only: <= 2e-5 max-abs.
* Rows never depend on the batch: engines of B = 6 and of its two halves give
  bit-identical logits at the same split count (the sharded-decode property).
* The chain's wide units (form 4: per phase 12-wave units, one per
  workgroup, or 6-wave, two per workgroup, where the phase has fewer units
  than 4-wave slots; a unit's K over its waves) at B = 64 / 40 / 32 / 20 /
  16 / 8 / 5: within the same bound of the launch
  path, rows independent of the batch (12 vs 5 + 7; 28 vs 20), eager =
  graph.
* Every step reports status 0 (no in-launch wait timed out).
* Forms 2 (the full persistent layer) and 4 (wide units) measured slower than
  the forms the engine picks and are in A/B builds only (make XFLAGS=-DHPA_AB,
  HPA_LIB=...; hpa_build_flags): their cases skip on the product library.
  The small model's tests run form 3 (the 4-wave chain), its product form.
"""
import os

import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu

SMALL = dict(maxT=256, V=1000, L=2, NH=2, C=128)
GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)


def _ab_only(hip, mode):
    if mode in (2, 4) and not hip.lib().hpa_build_flags() & 1:
        pytest.skip("layer form %d: A/B builds only (-DHPA_AB)" % mode)


def _model(hip, cfgd, params, B, P, layer, kv_dtype=0, splits_env=None, mode=3):
    _ab_only(hip, mode if layer else 0)
    if splits_env is not None:
        os.environ["HPA_LAYER_SPLITS"] = str(splits_env)
    try:
        m = hip.Model(cfgd, params=params)
        m.decode_init(B, P, cfgd["maxT"], kv_dtype=kv_dtype)
    finally:
        os.environ.pop("HPA_LAYER_SPLITS", None)
    # mode 2: the full persistent layer at every batch it supports; 3: the
    # attention's own launch + the persistent GEMM chain; 4: that chain with
    # wide units (per-phase widths by the batch's row blocks; C = 768); 5:
    # chain form 6 (12-wave units of T tiles, one per workgroup; C = 768)
    assert m.set_layer_kernel(mode if layer else 0) == bool(layer)
    if layer and mode in (4, 5, 6):
        assert m.layer_form() == 3
    m.set_graph(True)
    return m


@pytest.mark.parametrize("B,mode", [(64, 2), (32, 2), (16, 2), (8, 2), (64, 3), (40, 3), (8, 3), (16, 4), (8, 4),
                                    (5, 4), (32, 4), (20, 4), (40, 4), (64, 4), (64, 5), (48, 5), (33, 5), (32, 5),
                                    (20, 5), (16, 5), (8, 5), (5, 5), (64, 6), (33, 6), (17, 6), (1, 6)])
def test_persistent_layer_matches_launch_path_124m(hip, B, mode):
    params = synth.params(GPT2_124M, seed=31)
    ctx = 990
    rng = np.random.default_rng(B)
    toks = rng.integers(0, GPT2_124M["V"], (6, B)).astype(np.int32)
    out = []
    for layer in (1, 0):
        m = _model(hip, GPT2_124M, params, B, 16, layer, mode=mode)
        hip.check(hip.lib().gpt2_decode_fill_random(m.h, ctx, 5), "fill_random")
        lg, ids = [], []
        for t in range(toks.shape[0]):
            ids.append(m.step(toks[t]))
            lg.append(m.logits())
        m.status()
        assert np.array_equal(m.positions(), np.full(B, ctx + toks.shape[0], np.int32))
        m.close()
        out.append((np.stack(lg), np.stack(ids)))
    (lp, ip), (ll, il) = out
    diff = float(np.abs(lp - ll).max())
    s = np.sort(ll, axis=-1)
    margin = s[..., -1] - s[..., -2]
    clear = margin > 4 * diff
    print(f"B={B} mode {mode}: max |logit diff| persistent vs launches {diff:.3e}; near-ties {int((~clear).sum())}")
    assert diff <= 2e-5, diff
    assert np.array_equal(ip[clear], il[clear])


@pytest.mark.parametrize("P,mode", [(8, 2), (16, 2), (32, 2), (64, 2), (8, 3), (16, 3), (32, 3), (64, 3)])
def test_persistent_layer_small_model_matches_oracle(hip, P, mode):
    """greedy decode across page boundaries and many 64-token attention tiles"""
    params = synth.params(SMALL, seed=40 + P)
    B, steps = 5, 150
    m = _model(hip, SMALL, params, B, P, 1, mode=mode)
    c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
    orc = oc.PagedDecoder(params, c, B, P, SMALL["maxT"], page_seed=P)
    tok = np.random.default_rng(P).integers(0, SMALL["V"], B).astype(np.int32)
    worst = 0.0
    for t in range(steps):
        o_next, o_logits = orc.step(tok)
        g_next = m.step(tok)
        g_logits = m.logits()
        worst = max(worst, float(np.abs(g_logits - o_logits).max()))
        s = np.sort(o_logits, axis=-1)
        clear = (s[:, -1] - s[:, -2]) > 4e-4
        assert np.array_equal(g_next[clear], o_next[clear]), t
        tok = o_next
    m.status()
    print(f"P={P}: max |logit diff| vs oracle {worst:.3e}")
    assert worst <= 2e-4
    m.close()
    orc.close()


@pytest.mark.parametrize("splits,mode", [(1, 3), (3, 3), (16, 3), (1, 2), (3, 2), (16, 2)])
def test_persistent_layer_split_counts(hip, splits, mode):
    """context ranges per (sequence, head) forced: 1, a count that does not
    divide the tiles, and the maximum (ranges with no tile at short context);
    form 3 through the attention launch's split count, form 2 (A/B) through
    its own ranges (HPA_LAYER_SPLITS)"""
    params = synth.params(SMALL, seed=60 + splits)
    B = 4
    m = _model(hip, SMALL, params, B, 16, 1, splits_env=splits if mode == 2 else None, mode=mode)
    if mode == 3:
        m.set_attn_splits(splits)
    c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
    orc = oc.PagedDecoder(params, c, B, 16, SMALL["maxT"], page_seed=splits)
    rng = np.random.default_rng(splits)
    worst = 0.0
    for t in range(140):
        tok = rng.integers(0, SMALL["V"], B).astype(np.int32)
        _, o_logits = orc.step(tok)
        m.step(tok)
        worst = max(worst, float(np.abs(m.logits() - o_logits).max()))
    m.status()
    assert worst <= 2e-4, worst
    m.close()
    orc.close()


def test_persistent_layer_bf16_pool_matches_launch_path(hip):
    params = synth.params(SMALL, seed=77)
    B, steps = 9, 40
    rng = np.random.default_rng(77)
    toks = rng.integers(0, SMALL["V"], (steps, B)).astype(np.int32)
    res = []
    for layer in (1, 0):
        m = _model(hip, SMALL, params, B, 8, layer, kv_dtype=hip.HPA_BF16)
        lg = []
        for t in range(steps):
            m.step(toks[t])
            lg.append(m.logits())
        m.status()
        m.close()
        res.append(np.stack(lg))
    diff = float(np.abs(res[0] - res[1]).max())
    assert diff <= 1e-4, diff  # fp32 reassociation of attproj / fcproj (3e-5 measured)


def test_persistent_layer_rows_independent_of_batch(hip):
    """B = 6 vs its halves B = 3 + 3 at the same split count: bit-identical
    logits (what makes sequence-sharded decode equal the unsharded run)"""
    params = synth.params(SMALL, seed=90)
    steps = 30
    toks = np.random.default_rng(90).integers(0, SMALL["V"], (steps, 6)).astype(np.int32)

    def run(lo, hi):
        m = _model(hip, SMALL, params, hi - lo, 16, 1)
        m.set_attn_splits(4)
        lg = []
        for t in range(steps):
            m.step(toks[t, lo:hi])
            lg.append(m.logits())
        m.status()
        m.close()
        return np.stack(lg)

    full = run(0, 6)
    assert np.array_equal(full[:, :3], run(0, 3))
    assert np.array_equal(full[:, 3:], run(3, 6))


def test_persistent_layer_eager_equals_graph(hip):
    params = synth.params(SMALL, seed=5)
    toks = np.random.default_rng(5).integers(0, SMALL["V"], (12, 7)).astype(np.int32)
    outs = []
    for graph in (False, True):
        m = _model(hip, SMALL, params, 7, 16, 1)
        m.set_graph(graph)
        lg = []
        for t in range(12):
            m.step(toks[t])
            lg.append(m.logits())
        m.status()
        m.close()
        outs.append(np.stack(lg))
    assert np.array_equal(outs[0], outs[1])


def test_persistent_chain_wide_rows_independent_of_batch_and_graph(hip):
    """wide units at GPT-2 124M shapes: B = 12 vs its halves 5 + 7 give
    bit-identical logits (attention split count and waves fixed, as a sharded
    engine takes them from the global batch), and eager equals graph (form 4:
    A/B builds only)"""
    _ab_only(hip, 4)
    params = synth.params(GPT2_124M, seed=93)
    steps = 4
    toks = np.random.default_rng(93).integers(0, GPT2_124M["V"], (steps, 28)).astype(np.int32)

    def run(lo, hi, graph=True):
        m = _model(hip, GPT2_124M, params, hi - lo, 16, 1, mode=4)
        m.set_graph(graph)
        m.set_attn_splits(2)
        m.fill_random(300, seed=9, seq_offset=lo)
        lg = []
        for t in range(steps):
            m.step(toks[t, lo:hi])
            lg.append(m.logits())
        m.status()
        m.close()
        return np.stack(lg)

    hip.check(hip.lib().hpa_set_attention_waves(8), "waves")
    try:
        full = run(0, 12)
        assert np.array_equal(full[:, :5], run(0, 5))
        assert np.array_equal(full[:, 5:], run(5, 12))
        assert np.array_equal(full, run(0, 12, graph=False))
        full = run(0, 28)  # 6-wave units (17-32 rows): the first 20 rows of 28 = a 20-row engine
        assert np.array_equal(full[:, :20], run(0, 20))
    finally:
        hip.check(hip.lib().hpa_set_attention_waves(0), "waves")


def test_chain6_rows_independent_of_batch_and_form4(hip):
    """chain form 6 keeps the 12-wave units' summation order at every batch:
    with the attention's split count and waves pinned, the residual stream
    entering every layer (gpt2_decode_step_traced; the logits kernel's form
    follows the batch and is tested elsewhere) of B = 64 rows (4 row blocks,
    3 tiles per unit) equals that of B = 8 / 24 / 40 engines bit for bit; at
    one row block form 6 is form 4 within 2e-5 (layer 0's qkv differs: hpa_decode_first); graph
    replay = eager"""
    params = synth.params(GPT2_124M, seed=94)
    steps = 3
    toks = np.random.default_rng(94).integers(0, GPT2_124M["V"], (steps, 64)).astype(np.int32)

    def run(lo, hi, mode=5, traced=True):
        m = _model(hip, GPT2_124M, params, hi - lo, 16, 1, mode=mode)
        m.set_graph(not traced)
        m.set_attn_splits(1)
        m.fill_random(300, seed=11, seq_offset=lo)
        out = []
        for t in range(steps):
            if traced:
                out.append(m.step_traced(toks[t, lo:hi])[1])
            else:
                m.step(toks[t, lo:hi])
                out.append(m.logits())
        m.status()
        m.close()
        return np.stack(out)

    hip.check(hip.lib().hpa_set_attention_waves(4), "waves")
    try:
        full = run(0, 64)  # (steps, L+1, B, C)
        for lo, hi in ((0, 8), (40, 64), (8, 48)):
            assert np.array_equal(full[:, :, lo:hi], run(lo, hi)), (lo, hi)
        # form 4 at one row block sums every layer GEMM like form 6's 12-wave
        # units, but computes layer 0's qkv with the one-shot GEMM where form 6
        # opens the step with hpa_decode_first (chain order, LN1 folded); form 4
        # is in A/B builds only: the product library checks form 6 against the
        # five-launch loop (test_persistent_layer_matches_launch_path_124m)
        if hip.lib().hpa_build_flags() & 1:
            d = np.abs(run(0, 8, traced=False) - run(0, 8, mode=4, traced=False)).max()
            print(f"form 6 vs form 4 at B=8: max |logit diff| {d:.3e}")
            assert d <= 2e-5
        g64 = run(0, 64, traced=False)  # graph replay: its last step's residual feeds these logits
        assert np.isfinite(g64).all()
    finally:
        hip.check(hip.lib().hpa_set_attention_waves(0), "waves")


@pytest.mark.parametrize("B", [64, 40, 8])
def test_chain8_equals_chain6_124m(hip, B):
    """chain form 8 (streamed weights, host-picked tiles per unit) at GPT-2 124M
    shapes picks the same units as form 6 and sums in the same order: every
    layer's output and every logit bit-identical"""
    params = synth.params(GPT2_124M, seed=95)
    steps = 3
    toks = np.random.default_rng(95).integers(0, GPT2_124M["V"], (steps, B)).astype(np.int32)

    def run(mode, traced):
        m = _model(hip, GPT2_124M, params, B, 16, 1, mode=mode)
        assert m.layer_form() == 3
        m.set_graph(not traced)
        m.fill_random(500, seed=12)
        out = []
        for t in range(steps):
            if traced:
                out.append(m.step_traced(toks[t])[1])
            else:
                m.step(toks[t])
                out.append(m.logits())
        m.status()
        m.close()
        return np.stack(out)

    assert np.array_equal(run(6, True), run(5, True))
    assert np.array_equal(run(6, False), run(5, False))


GPT2_XL = dict(maxT=1024, V=50257, L=48, NH=25, C=1600)


@pytest.mark.parametrize("B", [64, 33, 5])
def test_chain8_xl_matches_launch_path(hip, B):
    """GPT-2 XL (C = 1600, 48 layers) on chain form 8 against the five-launch
    layer (ring / looped GEMMs): logits within fp32 reassociation, ids equal
    outside near-ties, status 0"""
    params = hip.synthetic_params(GPT2_XL, seed=96)
    ctx, steps = 200, 3
    toks = np.random.default_rng(96).integers(0, GPT2_XL["V"], (steps, B)).astype(np.int32)
    out = []
    for mode in (6, 0):
        m = hip.Model(GPT2_XL, params=params)
        m.decode_init(B, 32, ctx + 8)
        assert m.set_layer_kernel(mode) == (mode != 0)
        m.set_graph(True)
        m.fill_random(ctx, seed=13)
        lg, ids = [], []
        for t in range(steps):
            ids.append(m.step(toks[t]))
            lg.append(m.logits())
        m.status()
        m.close()
        out.append((np.stack(lg), np.stack(ids)))
    (l8, i8), (l0, i0) = out
    diff = float(np.abs(l8 - l0).max())
    s = np.sort(l0, axis=-1)
    clear = (s[..., -1] - s[..., -2]) > 4 * diff
    print(f"XL B={B}: max |logit diff| form 8 vs launches {diff:.3e}; near-ties {int((~clear).sum())}")
    assert diff <= 5e-5, diff
    assert np.array_equal(i8[clear], i0[clear])


@pytest.mark.parametrize("C,NH,B", [(1024, 16, 64), (1024, 16, 17), (1280, 20, 64), (1280, 20, 5)],
                         ids=["medium-64", "medium-17", "large-64", "large-5"])
def test_chain8_medium_large_matches_launch_path(hip, C, NH, B):
    """chain form 8 at GPT-2 medium (C = 1024, 16 heads) and large (C = 1280,
    20 heads) widths (round 6: the engine's auto form for C >= 1024, was five
    launches), 2 layers, small vocabulary: logits within fp32 reassociation of
    the five-launch layer, ids equal outside near-ties, status 0"""
    cfgd = dict(maxT=256, V=2000, L=2, NH=NH, C=C)
    assert hip.lib().hpa_decode_chain_eligible(B, C, NH, 8) == 1
    params = hip.synthetic_params(cfgd, seed=97)
    ctx, steps = 120, 3
    toks = np.random.default_rng(97 + B).integers(0, cfgd["V"], (steps, B)).astype(np.int32)
    out = []
    for mode in (1, 0):  # 1 = auto: form 8 at these widths
        m = hip.Model(cfgd, params=params)
        m.decode_init(B, 16, ctx + 8)
        assert m.set_layer_kernel(mode) == (mode != 0)
        if mode:
            assert m.layer_form() == 3
        m.set_graph(True)
        m.fill_random(ctx, seed=14)
        lg, ids = [], []
        for t in range(steps):
            ids.append(m.step(toks[t]))
            lg.append(m.logits())
        m.status()
        m.close()
        out.append((np.stack(lg), np.stack(ids)))
    (l8, i8), (l0, i0) = out
    diff = float(np.abs(l8 - l0).max())
    s = np.sort(l0, axis=-1)
    clear = (s[..., -1] - s[..., -2]) > 4 * diff
    print(f"C={C} B={B}: max |logit diff| form 8 vs launches {diff:.3e}")
    assert diff <= 5e-5, diff
    assert np.array_equal(i8[clear], i0[clear])
