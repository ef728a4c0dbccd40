"""BASELINE.json's GPU configs at their workload sizes:

  config 2  GPT-2 124M fp32, B=64, ctx 1024, page 16  (the headline metric)
  config 3  GPT-2 XL fp32,   B=64, ctx 1024, page 32
  config 5  GPT-2 124M bf16, B=256, ctx 2048, page 8  (bf16 weights + bf16 KV)

Each is checked on the default engine path the bench times (fused GEMMs,
hipGraph replay, the engine's attention split count):
  * end to end at the full context: the GPU pool is filled to ctx - steps,
    the SAME K/V is handed to the oracle (gpt2_decode_read_kv ->
    oracle set_kv), then both decode the same tokens at positions up to
    ctx - 1; logits and greedy ids compared on every sequence (config 2: all
    64; configs 3/5: a full-depth small batch, the oracle's CPU cost);
  * at the full batch: the attention kernel at the workload's shape against
    the oracle on a sequence subset, and step properties (finite, graph replay
    == eager, deterministic).
Tolerances as test_gpu_decode.py (logits 2e-4 fp32; ids bit-exact outside
near-ties of 2x the measured max logit difference, exempt rows counted).
Config 4 (8 GPUs) is the driver's multi-GPU run; its per-GPU shape is config 2.
"""
import numpy as np
import pytest

import oracle_ctypes as oc
from test_gpu_decode import BF16_EXEMPT, BF16W_LOGIT_TOL, LOGIT_TOL, IdCheck

pytestmark = pytest.mark.gpu

CFG_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
CFG_XL = dict(maxT=1024, V=50257, L=48, NH=25, C=1600)
CFG_124M_2K = dict(maxT=2048, V=50257, L=12, NH=12, C=768)  # wpe of 2048 rows (config 5)


def _params(hip, cfgd, seed):
    return hip.synthetic_params(cfgd, seed=seed)


def _identical_cache_run(hip, cfgd, params, B, P, ctx0, steps, seed, kv_bf16=False, w_bf16=False,
                         tol=LOGIT_TOL, max_exempt_frac=0.02):
    """fill the GPU pool to ctx0, give the oracle the same K/V, decode `steps`
    greedy steps from the same tokens on both; returns the IdCheck"""
    model = hip.Model(cfgd, params=params)
    model.decode_init(B, P, cfgd["maxT"], kv_dtype=hip.HPA_BF16 if kv_bf16 else hip.HPA_F32,
                      w_dtype=hip.HPA_BF16 if w_bf16 else hip.HPA_F32)
    model.set_graph(True)
    model.fill_random(ctx0, seed=seed)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    orc = oc.PagedDecoder(params, c, B, P, cfgd["maxT"], page_seed=seed, kv_bf16=kv_bf16, w_bf16=w_bf16)
    for l in range(cfgd["L"]):
        for b in range(B):
            k, v = model.read_kv(l, b, ctx0)
            orc.set_kv(l, b, k, v)
    rng = np.random.default_rng(seed)
    tok = rng.integers(0, cfgd["V"], B).astype(np.int32)
    chk = IdCheck()
    for _ in range(steps):
        o_next, o_logits = orc.step(tok)
        g_next = model.step(tok)
        chk.add(model.logits(), o_logits, g_next, o_next)
        tok = o_next
    assert np.array_equal(model.positions(), np.full(B, ctx0 + steps, np.int32))
    splits = model.attn_splits()
    model.close()
    orc.close()
    print(f"B={B} page {P} positions {ctx0}..{ctx0 + steps - 1}, attention splits {splits}")
    chk.verify(tol, max_exempt_frac)
    return chk


def test_config2_headline_end_to_end_full_context(hip):
    """config 2 exactly as the bench runs it (B=64, page 16, graph, positions
    ~990-1023): all 64 sequences vs the oracle on identical K/V"""
    params = _params(hip, CFG_124M, 2)
    chk = _identical_cache_run(hip, CFG_124M, params, B=64, P=16, ctx0=1024 - 34, steps=34, seed=2)
    assert len(chk.rows) == 34


def _attention_subset(hip, NH, P, B, ctx, subset, bf16=False, seed=0):
    """the decode attention at a workload shape (the engine's split count):
    sequences in `subset` vs the oracle, relaunch bit-identical"""
    L = hip.lib()
    C = NH * 64
    maxp = (ctx + P - 1) // P
    pool = hip.Pool(1, NH, P, B * maxp, dtype=hip.HPA_BF16 if bf16 else hip.HPA_F32)
    rng = np.random.default_rng(seed)
    bt = rng.permutation(B * maxp).astype(np.int32).reshape(B, maxp)
    d_bt = hip.DeviceBuffer.from_array(bt)
    hip.check(L.hpa_pool_fill_random(pool.ref, d_bt.ptr, maxp, B, ctx, 7 + seed))
    q = rng.uniform(-2, 2, (B, C)).astype(np.float32)
    pos = np.full(B, ctx - 1, np.int32)
    d_q = hip.DeviceBuffer.from_array(q)
    d_pos = hip.DeviceBuffer.from_array(pos)
    S = L.hpa_attn_pick_splits(B, NH, ctx, 256)
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
    assert np.isfinite(outs[0]).all()
    for b in subset:
        k, v = pool.read_tokens(0, bt[b], ctx)
        kp = [k[i * P:(i + 1) * P].copy() for i in range(maxp)]
        vp = [v[i * P:(i + 1) * P].copy() for i in range(maxp)]
        ref = oc.attention_decode(q[b], kp, vp, ctx, NH)
        assert np.abs(outs[0][b] - ref).max() <= 1e-4, b
    return S


def _step_properties(hip, cfgd, B, P, ctx0, kv_bf16=False, w_bf16=False, seed=3):
    """full-batch step at the workload's context: finite, graph == eager,
    deterministic (two engines on the same weights and cache)"""
    params = _params(hip, cfgd, seed)
    runs = []
    for graph in (True, False, True):
        m = hip.Model(cfgd, params=params)
        m.decode_init(B, P, ctx0 + 8, kv_dtype=hip.HPA_BF16 if kv_bf16 else hip.HPA_F32,
                      w_dtype=hip.HPA_BF16 if w_bf16 else hip.HPA_F32)
        m.set_graph(graph)
        m.fill_random(ctx0, seed=seed)
        tok = np.random.default_rng(seed).integers(0, cfgd["V"], B).astype(np.int32)
        ids = [m.step(tok)]
        for _ in range(3):
            ids.append(m.step(None))
        lg = m.logits()
        assert np.isfinite(lg).all()
        runs.append((np.stack(ids), lg))
        m.close()
    for ids, lg in runs[1:]:
        assert np.array_equal(ids, runs[0][0]) and np.array_equal(lg, runs[0][1])


# ---------------------------------------------------------------- config 3: GPT-2 XL
def test_config3_xl_attention_full_size(hip):
    """B=64, NH=25, ctx 1024, page 32 (40 GB of K/V at L=48; one layer here)"""
    _attention_subset(hip, NH=25, P=32, B=64, ctx=1024, subset=(0, 31, 63), seed=3)


def test_config3_xl_step_properties_full_batch(hip):
    _step_properties(hip, CFG_XL, B=64, P=32, ctx0=1000)


def test_config3_xl_end_to_end_full_depth(hip):
    """all 48 layers, V=50257, at positions ~1000-1023 on identical K/V; B=2
    (the oracle's CPU time)"""
    params = _params(hip, CFG_XL, 33)
    _identical_cache_run(hip, CFG_XL, params, B=2, P=32, ctx0=1000, steps=6, seed=33)


def test_config3_xl_full_batch_end_to_end(hip):
    """the full batch of config 3 (B=64: the layer GEMMs that run at it --
    qkv / fc on the ring kernel, hpa_gemm_ring.hip) against the oracle, all
    48 layers and V=50257; a short context (the K/V the oracle is handed is
    40 GB at ctx 1000, and the GEMMs do not depend on it)"""
    params = _params(hip, CFG_XL, 35)
    _identical_cache_run(hip, CFG_XL, params, B=64, P=32, ctx0=40, steps=2, seed=35)


# ---------------------------------------------------------------- config 5: bf16, B=256, ctx 2048, page 8
def test_config5_attention_full_size(hip):
    """bf16 KV, B=256, ctx 2048, page 8 (identical stored values on both sides)"""
    _attention_subset(hip, NH=12, P=8, B=256, ctx=2048, subset=(0, 100, 255), bf16=True, seed=5)


def test_config5_step_properties_full_batch(hip):
    """B=256, maxT=2048 (a 2048-row wpe), positions ~2040, bf16 weights + KV"""
    _step_properties(hip, CFG_124M_2K, B=256, P=8, ctx0=2032, kv_bf16=True, w_bf16=True)


def test_config5_end_to_end_full_context(hip):
    """bf16 weights + bf16 KV at positions ~2000-2047 on identical K/V, all 12
    layers, maxT = 2048; B=8"""
    params = _params(hip, CFG_124M_2K, 55)
    _identical_cache_run(hip, CFG_124M_2K, params, B=8, P=8, ctx0=2048 - 12, steps=12, seed=55, kv_bf16=True,
                         w_bf16=True, tol=BF16W_LOGIT_TOL, max_exempt_frac=BF16_EXEMPT)


# ---------------------------------------------------------------- per-layer pinning
def _layer_pinned_run(hip, cfgd, params, B, P, ctx0, steps, seed, kv_bf16=False, w_bf16=False, layer_rtol=1e-5,
                      tol=LOGIT_TOL, max_exempt_frac=0.02, max_ctx=None, layer_form=None):
    """Each layer on the GPU's own input: gpt2_decode_step_traced returns the
    residual stream entering every layer (and LNf), the oracle runs layer l
    from the GPU's stream[l] (oracle_paged_step_ex) and its output is compared
    with the GPU's stream[l+1]; logits and ids from the GPU's final stream.
    Rounding differences then do not compound over the 12 layers, so the ids
    are held to the fp32 bar (<= 2 % near-tie rows) also for bf16 numerics.
    max_ctx (default maxT) bounds both sides' pools (the wpe stays maxT rows).
    Returns the per-layer max |diff| / max |x| and the IdCheck."""
    max_ctx = max_ctx or cfgd["maxT"]
    model = hip.Model(cfgd, params=params)
    model.decode_init(B, P, max_ctx, kv_dtype=hip.HPA_BF16 if kv_bf16 else hip.HPA_F32,
                      w_dtype=hip.HPA_BF16 if w_bf16 else hip.HPA_F32)
    if layer_form is not None:  # the layer loop the test is about (bench's default)
        assert model.layer_form() == layer_form
    model.fill_random(ctx0, seed=seed)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    orc = oc.PagedDecoder(params, c, B, P, max_ctx, page_seed=seed, kv_bf16=kv_bf16, w_bf16=w_bf16)
    for l in range(cfgd["L"]):
        for b in range(B):
            k, v = model.read_kv(l, b, ctx0)
            orc.set_kv(l, b, k, v)
    import ctypes
    off = (ctypes.c_size_t * 16)()
    oc.lib().oracle_param_offsets(c, off)
    C = cfgd["C"]
    wte = params[off[0]:off[0] + cfgd["V"] * C].reshape(cfgd["V"], C)
    wpe = params[off[1]:off[1] + cfgd["maxT"] * C].reshape(cfgd["maxT"], C)
    rng = np.random.default_rng(seed)
    tok = rng.integers(0, cfgd["V"], B).astype(np.int32)
    chk = IdCheck()
    worst_layer = np.zeros(cfgd["L"])
    for s in range(steps):
        g_next, xs = model.step_traced(tok)
        assert np.array_equal(xs[0], wte[tok] + wpe[ctx0 + s])  # the embedding add, exact
        o_next, o_logits, o_out = orc.step_forced(tok, xs)
        for l in range(cfgd["L"]):
            scale = float(np.abs(xs[l + 1]).max())
            worst_layer[l] = max(worst_layer[l], float(np.abs(o_out[l] - xs[l + 1]).max()) / scale)
        chk.add(model.logits(), o_logits, g_next, o_next)
        tok = o_next
    model.close()
    orc.close()
    print("per-layer max |diff| / max |x|: " + " ".join(f"{x:.1e}" for x in worst_layer))
    chk.verify(tol, max_exempt_frac)
    assert worst_layer.max() <= layer_rtol, worst_layer
    return worst_layer, chk


# one bf16 ulp is 2^-8 relative: a layer whose GEMM inputs differ from the
# oracle's in single-ulp flips (fp32 rounding inputs that differ by summation
# order) moves its output by far less than that relative to the stream's scale
# (measured: 1.9e-3 at layer 0, whose stream is the small embedding, 2.5e-4 to
# 8e-4 after; logits 2.7e-4; 2 of 320 rows near-ties -- profiles/r3/pinned_c5.txt)
BF16_LAYER_RTOL = 4e-3
BF16_PINNED_LOGIT_TOL = 2e-3


def test_config5_layer_pinned_full_context(hip):
    """config 5 numerics (bf16 weights + bf16 KV, page 8, maxT 2048) at
    positions ~2030-2047, B=32: every layer on the GPU's own input, ids at
    the 2 % near-tie bar"""
    params = _params(hip, CFG_124M_2K, 56)
    _layer_pinned_run(hip, CFG_124M_2K, params, B=32, P=8, ctx0=2048 - 10, steps=10, seed=56, kv_bf16=True,
                      w_bf16=True, layer_rtol=BF16_LAYER_RTOL, tol=BF16_PINNED_LOGIT_TOL, layer_form=4)


@pytest.mark.parametrize("chain", [True, False], ids=["bf16_chain", "five_launches"])
def test_config5_layer_pinned_full_batch(hip, chain, monkeypatch):
    """config 5's real batch, B=256 (bf16 weights + bf16 KV, page 8, the
    2048-row wpe): the layer loop the bench runs -- the bf16 chain
    (hpa_chain_b16.hip, one persistent launch per layer) -- and the five-launch
    loop (A-resident bf16 GEMMs, variant 5) on the shape they serve, each layer
    on the GPU's own input against the oracle; a short context (the GEMMs do
    not depend on it; the pools bounded to 64 positions), ids at the 2 %
    near-tie bar"""
    if not chain:
        monkeypatch.setenv("HPA_LAYER_KERNEL", "0")
    params = _params(hip, CFG_124M_2K, 58)
    _layer_pinned_run(hip, CFG_124M_2K, params, B=256, P=8, ctx0=40, steps=4, seed=58, kv_bf16=True,
                      w_bf16=True, layer_rtol=BF16_LAYER_RTOL, tol=BF16_PINNED_LOGIT_TOL, max_ctx=64,
                      layer_form=4 if chain else 0)


@pytest.mark.parametrize("B,P,kv_bf16", [(1, 16, False), (40, 8, True), (200, 8, False)])
def test_bf16_chain_ragged_batches(hip, B, P, kv_bf16):
    """the bf16 chain at batches that are not whole row groups of 32: one row
    (one row block), 40 rows (3 row blocks: the last row group has one block)
    and 200 rows (13 blocks), fp32 and bf16 pools; every layer against the oracle"""
    params = _params(hip, CFG_124M, 60 + B)
    _layer_pinned_run(hip, CFG_124M, params, B=B, P=P, ctx0=30, steps=3, seed=60 + B, kv_bf16=kv_bf16, w_bf16=True,
                      layer_rtol=BF16_LAYER_RTOL, tol=BF16_PINNED_LOGIT_TOL, max_ctx=64, layer_form=4)


@pytest.mark.parametrize("B,parts", [(40, (16, 24)), (96, (32, 64))])
def test_bf16_chain_shards_equal_unsharded(hip, B, parts):
    """the bf16 chain sums a row in an order that depends on neither
    the batch nor the row's place in it, and with gpt2_decode_set_global_batch
    a shard's attention splits and waves follow the global batch (up to the
    bf16 chain's 256 rows): every shard's logits and ids equal the unsharded
    engine's rows bit for bit (B = 40 as 16 + 24; B = 96 as 32 + 64, a global
    batch above 64)"""
    params = _params(hip, CFG_124M, 62)
    ctx, steps = 300, 2
    toks = np.random.default_rng(62).integers(0, CFG_124M["V"], (steps, B)).astype(np.int32)

    def run(rows, lo, total):
        m = hip.Model(CFG_124M, params=params)
        m.decode_init(rows, 16, 512, w_dtype=hip.HPA_BF16)
        if total:
            m.set_global_batch(total)
        assert m.layer_form() == 4  # the bf16 chain
        m.set_graph(True)
        m.fill_random(ctx, seed=9, seq_offset=lo)
        lg, ids = [], []
        for t in range(steps):
            ids.append(m.step(toks[t, lo:lo + rows]))
            lg.append(m.logits())
        m.status()
        splits, waves = m.attn_splits(), m.attn_waves()
        m.close()
        return np.stack(lg), np.stack(ids), (splits, waves)

    ref_l, ref_i, ref_shape = run(B, 0, 0)
    lo = 0
    for rows in parts:
        lg, ids, shape = run(rows, lo, B)
        assert shape == ref_shape, (rows, shape, ref_shape)
        assert np.array_equal(ids, ref_i[:, lo:lo + rows])
        assert np.array_equal(lg, ref_l[:, lo:lo + rows]), float(np.abs(lg - ref_l[:, lo:lo + rows]).max())
        lo += rows


def test_config2_layer_pinned_full_context(hip):
    """the fp32 headline path (its default layer form) layer by layer: B=64,
    page 16, positions ~1014-1023"""
    params = _params(hip, CFG_124M, 57)
    _layer_pinned_run(hip, CFG_124M, params, B=64, P=16, ctx0=1024 - 10, steps=10, seed=57, layer_rtol=1e-5)
