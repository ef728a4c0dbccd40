"""Device multinomial sampling (hpa_sample_final) vs the reference's
softmax_forward + sample_mult with random_f32 coins (paged_infer.c:259-286,
:826-848; the oracle's C restatement), on logits built to stress the
integer-scan formulation of the ordered fp32 sums: wide ranges (denormal and
zero terms), quantised logits (repeated terms, rounding ties), one dominant
logit, all-equal logits, and vocabularies around the 4096-term chunk edges.
The single-lane sequential kernel (hpa_sample_final_serial) is checked too.

Tolerance: none. Draws are bit-equal (ids compared exactly), and each row
draws 6 coins so the cdf crossings fall at different indices.
"""
import numpy as np
import pytest

import oracle_ctypes as oc

pytestmark = pytest.mark.gpu


def _logits(kind, B, V, rng):
    if kind.startswith("randn"):
        return (rng.standard_normal((B, V)) * float(kind[5:])).astype(np.float32)
    if kind == "quant":  # repeated exps: many exact rounding ties
        return (np.round(rng.standard_normal((B, V)) * 4) / 4).astype(np.float32)
    if kind == "equal":
        return np.zeros((B, V), np.float32)
    if kind == "spike":  # sum = 1 + tiny terms
        x = (rng.standard_normal((B, V)) - 30).astype(np.float32)
        x[np.arange(B), rng.integers(0, V, B)] = 5.0
        return x
    if kind == "ramp":  # slowly growing terms, the sum crosses many binades late
        return np.tile(np.linspace(-20, 0, V, dtype=np.float32), (B, 1))
    raise ValueError(kind)


@pytest.mark.parametrize("entry", ["hpa_sample_final", "hpa_sample_final_serial"])
@pytest.mark.parametrize("kind,V", [("randn1", 50257), ("randn3", 50257), ("randn40", 50257),
                                    ("quant", 50257), ("equal", 50257), ("spike", 50257), ("ramp", 50257),
                                    ("randn2", 1), ("randn2", 2), ("randn2", 63), ("randn2", 4095),
                                    ("randn2", 4096), ("randn2", 4097), ("quant", 8193)])
def test_sample_final_matches_reference_sampler(hip, entry, kind, V):
    L = hip.lib()
    B, draws = 12, 6
    rng = np.random.default_rng(V + len(kind))
    x = _logits(kind, B, V, rng)
    d_x = hip.DeviceBuffer(x.nbytes)
    d_x.upload(x)
    seeds = np.arange(B, dtype=np.uint64) + np.uint64(1337 + V)
    d_st = hip.DeviceBuffer(B * 8)
    d_st.upload(seeds)
    d_next = hip.DeviceBuffer(B * 4)
    sampler = oc.Sampler(B, seed=1337 + V)
    for d in range(draws):
        hip.check(getattr(L, entry)(d_x.ptr, B, V, d_st.ptr, d_next.ptr, None, None, None), entry)
        got = d_next.download(B, np.int32)
        want = sampler.sample(x)
        assert np.array_equal(got, want), (d, got, want)
    assert np.array_equal(d_st.download(B, np.uint64), np.array([s.value for s in sampler.states], np.uint64))


def test_sample_final_inactive_rows_untouched(hip):
    L = hip.lib()
    B, V = 6, 5000
    x = np.random.default_rng(0).standard_normal((B, V)).astype(np.float32)
    d_x = hip.DeviceBuffer(x.nbytes)
    d_x.upload(x)
    st0 = np.arange(B, dtype=np.uint64) + np.uint64(7)
    d_st = hip.DeviceBuffer(B * 8)
    d_st.upload(st0)
    d_next = hip.DeviceBuffer(B * 4)
    d_next.upload(np.full(B, -5, np.int32))
    active = np.array([1, 0, 1, 0, 0, 1], np.int32)
    d_act = hip.DeviceBuffer(B * 4)
    d_act.upload(active)
    hip.check(L.hpa_sample_final(d_x.ptr, B, V, d_st.ptr, d_next.ptr, None, None, d_act.ptr))
    got, st = d_next.download(B, np.int32), d_st.download(B, np.uint64)
    sampler = oc.Sampler(B, seed=7)
    want = sampler.sample(x)
    for b in range(B):
        if active[b]:
            assert got[b] == want[b] and st[b] == sampler.states[b].value
        else:
            assert got[b] == -5 and st[b] == st0[b]
