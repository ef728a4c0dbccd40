"""The drop-in paged_infer.c / block_manager.c API on the GPU against the
reference's own outputs (tests/golden/) and the oracle.

attention_paged / matmul_forward / matmul_cached run the reference's
arithmetic order on the GPU (hpa_ref_* kernels); expected agreement with the
reference: <= 1e-6 max-abs (expf ulps), matmuls bit-exact.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle_ctypes as oc
import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)


def fp(a):
    return a.ctypes.data_as(_F)


def test_attention_paged_dropin_matches_reference(hip):
    L = hip.lib()
    L.attention_paged.argtypes = [_F, _F, _F, _F, ctypes.POINTER(_F), ctypes.POINTER(_F)] + \
        [ctypes.c_int] * 5
    L.attention_paged.restype = None
    g = np.load(os.path.join(GOLD, "attn_paged_golden.npz"))
    for ci in range(int(g["ncases"])):
        B, T, C, NH, off, bs = [int(x) for x in g[f"c{ci}_shape"]]
        assert bs == 32  # the reference's BLOCK_SIZE
        kpool, vpool, order = g[f"c{ci}_kpool"], g[f"c{ci}_vpool"], g[f"c{ci}_order"]
        inp = np.ascontiguousarray(g[f"c{ci}_inp"])
        out = np.zeros((B, T, C), np.float32)
        pre = np.zeros((B, NH, T, T), np.float32)
        att = np.zeros((B, NH, T, T), np.float32)
        n = len(order)
        kb = (_F * n)(*[fp(kpool[p]) for p in order])  # host pages: staged through HBM
        vb = (_F * n)(*[fp(vpool[p]) for p in order])
        L.attention_paged(fp(out), fp(pre), fp(att), fp(inp), kb, vb, B, T, C, NH, off)
        assert np.abs(out - g[f"c{ci}_out"]).max() <= 1e-6, ci
        assert np.abs(att - g[f"c{ci}_att"]).max() <= 1e-6, ci
        assert np.abs(pre - g[f"c{ci}_preatt"]).max() <= 1e-6, ci


def test_matmul_dropins_match_reference(hip):
    L = hip.lib()
    for name in ("matmul_forward", "matmul_cached"):
        getattr(L, name).argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
        getattr(L, name).restype = None
    g = np.load(os.path.join(GOLD, "matmul_golden.npz"))
    B, T, C, OC = [int(x) for x in g["shape"]]
    out = np.zeros((B, T, OC), np.float32)
    L.matmul_forward(fp(out), fp(g["inp"]), fp(g["w"]), fp(g["b"]), B, T, C, OC)
    assert np.array_equal(out, g["fwd"])
    out = np.zeros((B, T, OC), np.float32)
    L.matmul_cached(fp(out), fp(g["inp"]), fp(g["w"]), fp(g["b"]), B, T, C, OC)
    assert np.array_equal(out, g["cached"])


def test_gpt2_forward_window_driver(hip):
    """the reference driver's calling convention (paged_infer.c:1028-1080):
    first call T=32 tokens at offset 0, then sliding windows offset t-32;
    gpt2_forward (on the decode engine) must give the logits of absolute
    position offset+T-1 == the oracle's full forward (all layers)."""
    L = hip.lib()
    cfgd = dict(maxT=64, V=1000, L=2, NH=2, C=128)
    params = synth.params(cfgd, seed=31)
    m = hip.Model(cfgd, params=params)
    T, total = 32, 40
    rng = np.random.default_rng(0)
    gen = rng.integers(0, cfgd["V"], total).astype(np.int32)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    full = oc.gpt2_forward(params, c, gen[None, :])[0]  # (total, V)
    for t in range(T, total + 1):
        off = t - T
        window = np.ascontiguousarray(gen[off:off + T])
        L.gpt2_forward(m.h, window.ctypes.data_as(_I), None, 1, T, total, off)
        lg = np.ctypeslib.as_array(L.gpt2_acts_logits(m.h), shape=(T * cfgd["V"],))
        row = lg[(T - 1) * cfgd["V"]:T * cfgd["V"]]
        assert np.abs(row - full[t - 1]).max() <= 2e-4, t
        pr = np.ctypeslib.as_array(L.gpt2_acts_probs(m.h), shape=(T * cfgd["V"],))
        prow = pr[(T - 1) * cfgd["V"]:]
        assert abs(float(prow.sum()) - 1.0) < 1e-4
    m.close()


def test_gpt2_forward_reference_main_fill_loop(hip):
    """the reference main's FIRST loop (paged_infer.c:1028-1050): the whole
    T-window at offset 0 is passed again and again, placeholders beyond the
    real tokens, one more real token each call, and the caller reads probs
    row t-1.  Every row of the window must be that position's logits, so the
    engine recomputes from the first changed position; then the sliding
    loop continues.  Compared with the oracle's full forward of the final
    tokens (each row t-1 depends on tokens 0..t-1 only)."""
    L = hip.lib()
    cfgd = dict(maxT=64, V=1000, L=2, NH=2, C=128)
    params = synth.params(cfgd, seed=37)
    m = hip.Model(cfgd, params=params)
    T, prompt, total, V = 16, 6, 24, cfgd["V"]
    rng = np.random.default_rng(3)
    gen = np.full(total, 999, np.int32)  # GPT2_EOT-like placeholder
    gen[:prompt] = rng.integers(0, V, prompt)
    c = oc.cfg(cfgd["maxT"], V, cfgd["L"], cfgd["NH"], cfgd["C"])
    for t in range(prompt, T):  # fill loop: offset 0, row t-1
        L.gpt2_forward(m.h, gen[:T].ctypes.data_as(_I), None, 1, T, total, 0)
        lg = np.ctypeslib.as_array(L.gpt2_acts_logits(m.h), shape=(T, V))
        ref = oc.gpt2_forward(params, c, gen[None, :T].copy())[0]
        assert np.abs(lg[:t] - ref[:t]).max() <= 2e-4, t  # every real row, not only t-1
        pr = np.ctypeslib.as_array(L.gpt2_acts_probs(m.h), shape=(T, V))
        assert abs(float(pr[t - 1].sum()) - 1.0) < 1e-4
        gen[t] = int(np.argmax(pr[t - 1]))
    for t in range(T, total):  # sliding loop: offset t-T, row T-1
        off = t - T
        L.gpt2_forward(m.h, np.ascontiguousarray(gen[off:off + T]).ctypes.data_as(_I), None, 1, T, total, off)
        lg = np.ctypeslib.as_array(L.gpt2_acts_logits(m.h), shape=(T, V))
        ref = oc.gpt2_forward(params, c, gen[None, :t].copy())[0]
        assert np.abs(lg[T - 1] - ref[t - 1]).max() <= 2e-4, t
        assert np.abs(lg - ref[off:t]).max() <= 2e-4, t  # the whole window's rows
        gen[t] = int(np.argmax(lg[T - 1]))
    m.close()


def test_gpt2_forward_config1_prompt_one_pass(hip):
    """BASELINE config 1's own API path at its shape: GPT-2 124M (all 12
    layers, V = 50257), B = 1, page 16, a 64-token prompt passed to the
    drop-in gpt2_forward at offset 0 (paged_infer.c:575-729).  The first
    window is ONE multi-row prefill pass returning every row's logits (the
    reference's T-row matmul_forward, :703-704, :727), not 64 single-row
    decode steps; every row must equal the oracle's full forward, and the
    sliding windows after it (one new position each: a decode step) too."""
    L = hip.lib()
    cfgd = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
    params = synth.params(cfgd, seed=41)
    m = hip.Model(cfgd, params=params)
    T, total, V = 64, 68, cfgd["V"]
    gen = np.random.default_rng(41).integers(0, V, total).astype(np.int32)
    c = oc.cfg(cfgd["maxT"], V, cfgd["L"], cfgd["NH"], cfgd["C"])
    full = oc.gpt2_forward(params, c, gen[None, :].copy())[0]  # (total, V): causal, so rows < T are the window's
    strict = full[:T]
    L.gpt2_forward(m.h, np.ascontiguousarray(gen[:T]).ctypes.data_as(_I), None, 1, T, total, 0)
    lg = np.ctypeslib.as_array(L.gpt2_acts_logits(m.h), shape=(T, V)).copy()
    d = np.abs(lg - strict).max()
    print(f"config-1 prompt: 64 rows through one prefill pass, max |logit diff| vs oracle {d:.2e}")
    assert d <= 2e-4
    s = np.sort(strict, -1)
    clear = (s[:, -1] - s[:, -2]) > 4 * d
    assert np.array_equal(lg.argmax(-1)[clear], strict.argmax(-1)[clear]) and clear.mean() > 0.9
    pr = np.ctypeslib.as_array(L.gpt2_acts_probs(m.h), shape=(T, V))
    assert np.abs(pr.sum(-1) - 1.0).max() < 1e-4
    for t in range(T + 1, total + 1):  # sliding windows: one new position each
        off = t - T
        L.gpt2_forward(m.h, np.ascontiguousarray(gen[off:t]).ctypes.data_as(_I), None, 1, T, total, off)
        lg = np.ctypeslib.as_array(L.gpt2_acts_logits(m.h), shape=(T, V))
        assert np.abs(lg - full[off:t]).max() <= 2e-4, t
    m.close()


def test_external_manager_survives_engine_teardown(hip):
    """a caller-owned manager (model.manager, paged_infer.c:986-987) gets its
    pages back and its default backend when the engine goes away
    (gpt2_decode_free), so later request_block / collect_kv_blocks hand out
    live host-visible memory, never pointers into the freed pool"""
    L = hip.lib()
    cfgd = dict(maxT=64, V=1000, L=2, NH=2, C=128)
    m = hip.Model(cfgd, params=synth.params(cfgd, seed=5))
    bm = hip.BlockManager(cfgd["C"], max_prompts=4, max_blocks=16, block_size=16, max_blocks_per_prompt=4)
    m.set_manager(bm)
    m.decode_init(4, 16, 64)
    m.step(np.arange(4, dtype=np.int32))
    L.gpt2_decode_free(m.h)
    assert L.bm_free_pages(bm.h) == 16
    i = bm.request_block(0)
    blk = bm.block(i)
    keys = ctypes.cast(blk.keys, ctypes.c_void_p).value
    assert keys and L.hpa_is_device_accessible(keys) == 1
    for j in range(16 * cfgd["C"]):  # host writes through the fresh page
        blk.keys[j] = float(j)
    n = ctypes.c_int()
    kv = L.collect_kv_blocks(bm.h, 0, ctypes.byref(n))
    assert kv and n.value == 1
    m.close()
    bm.close()


def test_lru_eviction_is_reported(hip):
    """pool pressure: the reference policy evicts the least recently used
    sequence whole (block_manager.c:104-113); the engine reports it through
    gpt2_decode_evicted so the caller can re-prefill that slot"""
    cfgd = dict(maxT=64, V=1000, L=2, NH=2, C=128)
    m = hip.Model(cfgd, params=synth.params(cfgd, seed=6))
    bm = hip.BlockManager(cfgd["C"], max_prompts=3, max_blocks=5, block_size=16, max_blocks_per_prompt=4)
    m.set_manager(bm)
    m.decode_init(3, 16, 64)
    m.prefill_ragged([list(range(30)), [], []])  # sequence 0: 2 pages
    m.prefill_ragged([[], list(range(30)), []])  # sequence 1: 2 pages
    assert not m.evicted().any()
    m.prefill_ragged([[], [], list(range(20))])  # sequence 2 needs 2 pages: only 1 free -> LRU (0) evicted
    ev = m.evicted()
    assert ev.tolist() == [True, False, False]
    assert m.positions().tolist() == [0, 30, 20]
    assert not m.evicted().any()  # reported once
    m.close()
    bm.close()


def test_block_manager_managed_pages_host_roundtrip(hip):
    """block_manager_test.c's scenario with pages in HIP managed memory (the
    library's default backend): host writes, host reads back."""
    bm = hip.BlockManager(2)
    i0 = bm.request_block(0)
    b0 = bm.block(i0)
    assert hip.lib().hpa_is_device_accessible(ctypes.cast(b0.keys, ctypes.c_void_p).value) == 1
    for i in range(32):
        for j in range(2):
            b0.keys[i * 2 + j] = 1.0 * i + 0.1 * j
            b0.values[i * 2 + j] = 2.0 * i + 0.2 * j
    i1 = bm.request_block(0)
    assert i1 == i0 + 1
    b0 = bm.block(i0)
    assert b0.keys[31 * 2 + 1] == np.float32(31.0 + 0.1)
    bm.close()
