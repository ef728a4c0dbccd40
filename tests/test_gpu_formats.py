"""Models built from the reference's own checkpoint files (v1 fp32 and v2
bf16, tests/golden/gen_checkpoints.py) decode on the GPU engine to the
reference PyTorch model's logits (train_gpt2.py GPT.forward), and a v2
checkpoint equals the same model built from its widened parameters."""
import os

import numpy as np
import pytest

import oracle_ctypes as oc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EXP = np.load(os.path.join(GOLD, "ckpt_expected.npz"))
LOGIT_TOL = 2e-4


def _decode(model, tokens, B=2):
    """the same token stream in B sequences; logits of sequence 0 per step"""
    out = []
    for t in tokens:
        model.step(np.full(B, t, np.int32))
        lg = model.logits()
        assert np.array_equal(lg[0], lg[1])  # sequences are independent and identical
        out.append(lg[0])
    return np.stack(out)


def test_v1_checkpoint_matches_reference_forward(hip):
    m = hip.Model(None, checkpoint=os.path.join(GOLD, "ckpt_v1.bin"))
    c, p = hip.read_checkpoint(os.path.join(GOLD, "ckpt_v1.bin"))
    m.decode_init(2, 16, c.max_seq_len)
    lg = _decode(m, EXP["tokens"])
    m.close()
    scale = max(1.0, float(np.abs(EXP["logits"]).max()))
    assert np.abs(lg - EXP["logits"]).max() <= LOGIT_TOL * scale
    # and against the oracle (the same bar as every decode test)
    dec = oc.PagedDecoder(p, oc.cfg(c.max_seq_len, c.vocab_size, c.num_layers, c.num_heads, c.channels), 1, 16,
                          c.max_seq_len)
    ref = np.stack([dec.step(np.array([t], np.int32))[1][0] for t in EXP["tokens"]])
    dec.close()
    assert np.abs(lg - ref).max() <= LOGIT_TOL * scale


def test_v2_checkpoint_equals_widened_params(hip):
    path = os.path.join(GOLD, "ckpt_v2.bin")
    c, p = hip.read_checkpoint(path)
    a = hip.Model(None, checkpoint=path)
    b = hip.Model(c, params=p)
    for m in (a, b):
        m.decode_init(2, 16, c.max_seq_len)
    la, lb = _decode(a, EXP["tokens"][:12]), _decode(b, EXP["tokens"][:12])
    assert np.array_equal(la, lb)
    scale = max(1.0, float(np.abs(EXP["logits"]).max()))
    # bf16 weights: close to the fp32 reference, not equal
    assert np.abs(la - EXP["logits"][:12]).max() <= 0.1 * scale
    a.close()
    b.close()
