"""The pipelined halves (hpa_pipe.hip, gpt2_decode_set_layer_kernel(model, 7)):
every layer of a decode step in ONE persistent launch, the batch in two
halves, the GEMM chain of one half on 64 CUs beside the paged attention of the
other on the rest.

Its units are chain form 6's (12-wave K split, fcproj's K parts in order) and
paged_attn_decode_f32<P, 4>'s (one context range, 4 waves), so a step must
equal the form-5 step (decode attention launch + chain form 6 per layer) bit
for bit when that step's attention runs one range of 4 waves -- the form-5
path is pinned to the oracle by test_gpu_configs.py / test_gpu_layer.py; one
case here also goes to the oracle directly (reference paged_infer.c:575-729,
oracle/paged_oracle.c)."""
import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _ab_build(hip):
    """measured slower than chain form 6 (profiles/r6/pipe/README.md): the
    pipelined halves are compiled into A/B builds only (-DHPA_AB)"""
    if not hip.lib().hpa_build_flags() & 1:
        pytest.skip("pipelined halves: A/B builds only (-DHPA_AB)")

GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)


def _run(hip, params, B, P, form, toks, ctx, pos=None, graph=True, g_cus=0):
    """logits and ids of len(toks) steps of a fresh engine; form 5 runs its
    attention as one range of 4 waves (the pipelined halves' attention)"""
    L = hip.lib()
    m = hip.Model(GPT2_124M, params=params)
    m.decode_init(B, P, GPT2_124M["maxT"])
    assert m.set_layer_kernel(form)
    if form == 5:
        m.set_attn_splits(1)
        hip.check(L.hpa_set_attention_waves(4), "waves")
    else:
        assert m.layer_form() == 5, "pipelined halves not picked"
        if g_cus:
            m.set_pipe_split(g_cus)
    m.set_graph(graph)
    m.fill_random(ctx, seed=21)
    if pos is not None:
        m.set_positions(pos)
    lg, ids = [], []
    try:
        for t in range(len(toks)):
            ids.append(m.step(toks[t]))
            lg.append(m.logits())
        m.status()
    finally:
        hip.check(L.hpa_set_attention_waves(0), "waves")
        m.close()
    return np.stack(lg), np.stack(ids)


@pytest.mark.parametrize("B,P", [(64, 16), (56, 16), (49, 16), (32, 16), (20, 16), (17, 16), (64, 8), (64, 32),
                                 (64, 64)])
def test_pipe_equals_chain6(hip, B, P):
    """every logit and id of 3 graph-replayed steps equal the chain-form step's
    bit for bit (halves of 2 row blocks at 49..64 rows, of 1 at 17..32)"""
    assert hip.lib().hpa_decode_pipe_eligible(B, 768, 12, hip.HPA_F32) == 1
    params = synth.params(GPT2_124M, seed=71)
    toks = np.random.default_rng(B + P).integers(0, GPT2_124M["V"], (3, B)).astype(np.int32)
    ref = _run(hip, params, B, P, 5, toks, 700)
    got = _run(hip, params, B, P, 7, toks, 700)
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0], ref[0]), float(np.abs(got[0] - ref[0]).max())


def test_pipe_ragged_positions_eager_and_splits(hip):
    """ragged contexts (1 .. 990 tokens, pages exactly full among them), eager
    launches, and the GEMM role on 64 / 96 / 128 CUs: all bit-identical to the
    chain-form step"""
    B, P = 64, 16
    params = synth.params(GPT2_124M, seed=72)
    rng = np.random.default_rng(72)
    pos = rng.integers(0, 990, B).astype(np.int32)
    pos[:6] = [0, 15, 16, 63, 64, 989]
    toks = rng.integers(0, GPT2_124M["V"], (2, B)).astype(np.int32)
    ref = _run(hip, params, B, P, 5, toks, 992, pos=pos)
    for graph, g in [(False, 0), (True, 96), (True, 128)]:
        got = _run(hip, params, B, P, 7, toks, 992, pos=pos, graph=graph, g_cus=g)
        assert np.array_equal(got[1], ref[1]), (graph, g)
        assert np.array_equal(got[0], ref[0]), (graph, g, float(np.abs(got[0] - ref[0]).max()))


def test_pipe_not_eligible_odd_row_blocks(hip):
    """three row blocks (33..48 rows) do not split into equal halves: not
    eligible, and form 7 there runs chain form 6"""
    L = hip.lib()
    assert [L.hpa_decode_pipe_eligible(b, 768, 12, hip.HPA_F32) for b in (16, 17, 32, 33, 48, 49, 64, 65)] == \
        [0, 1, 1, 0, 0, 1, 1, 0]
    assert L.hpa_decode_pipe_eligible(64, 768, 12, hip.HPA_BF16) == 0
    m = hip.Model(GPT2_124M, params=synth.params(GPT2_124M, seed=74))
    m.decode_init(40, 16, GPT2_124M["maxT"])
    assert m.set_layer_kernel(7) and m.layer_form() == 3
    m.close()


def test_pipe_matches_oracle(hip):
    """against the oracle on identical K/V (the GPU pool's, gpt2_decode_read_kv):
    56 rows at positions 600.., 4 steps, logits within the fp32 bar (2e-4) and
    ids equal outside near-ties"""
    B, P, ctx, steps = 56, 16, 600, 4
    cfgd = GPT2_124M
    params = synth.params(cfgd, seed=73)
    m = hip.Model(cfgd, params=params)
    m.decode_init(B, P, cfgd["maxT"])
    assert m.set_layer_kernel(7) and m.layer_form() == 5
    m.set_graph(True)
    m.fill_random(ctx, seed=22)
    o = oc.PagedDecoder(params, oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"]), B, P,
                        cfgd["maxT"])
    for layer in range(cfgd["L"]):
        for b in range(B):
            k, v = m.read_kv(layer, b, ctx)
            o.set_kv(layer, b, k, v)
    tok = np.random.default_rng(73).integers(0, cfgd["V"], B).astype(np.int32)
    worst, exempt = 0.0, 0
    try:
        for _ in range(steps):
            onext, ologits = o.step(tok)
            gnext = m.step(tok)
            gl = m.logits()
            d = float(np.abs(gl - ologits).max())
            worst = max(worst, d)
            s = np.sort(ologits, -1)
            clear = (s[:, -1] - s[:, -2]) > 2 * d
            exempt += int((~clear).sum())
            assert np.array_equal(gnext[clear], onext[clear])
            tok = onext
        m.status()
    finally:
        m.close()
        o.close()
    print(f"pipe vs oracle: max |logit diff| {worst:.2e}, near-tie rows {exempt}")
    assert worst <= 2e-4, worst
    assert exempt <= 0.02 * B * steps
