"""On-disk formats, host-only: the v1 / v2 checkpoint
reader and writer and the tokenizer, against files written by the
reference's own train_gpt2.py (write_model :295-320, write_tokenizer
:350-363; tests/golden/gen_checkpoints.py made them), and the oracle's
model against the reference's PyTorch forward logits for the same
checkpoint.  No GPU: these are host functions of libpaged_hip.so.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle_ctypes as oc
import pagedattn as pa

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
V1 = os.path.join(GOLD, "ckpt_v1.bin")
V2 = os.path.join(GOLD, "ckpt_v2.bin")
TOK = os.path.join(GOLD, "tokenizer.bin")
EXP = np.load(os.path.join(GOLD, "ckpt_expected.npz"))
BF16_TENSORS = (0, 1, 4, 5, 6, 7, 10, 11, 12, 13)  # train_gpt2.py:267-285; LN tensors stay fp32


def _tensors(c, p):
    C, L, V, T = c.channels, c.num_layers, c.vocab_size, c.max_seq_len
    sizes = [V * C, T * C, L * C, L * C, L * 3 * C * C, L * 3 * C, L * C * C, L * C, L * C, L * C,
             L * 4 * C * C, L * 4 * C, L * C * 4 * C, L * C, C, C]
    out, o = [], 0
    for s in sizes:
        out.append(p[o:o + s])
        o += s
    assert o == p.size
    return out


def test_v1_reads_reference_file():
    c, p = pa.read_checkpoint(V1)
    assert [c.max_seq_len, c.vocab_size, c.num_layers, c.num_heads, c.channels] == list(EXP["config"])
    sums = [t.astype(np.float64).sum() for t in _tensors(c, p)]
    np.testing.assert_allclose(sums, EXP["psum"], rtol=1e-9, atol=1e-9)


def test_v2_is_v1_rounded_to_bf16():
    """bf16 tensors widen exactly to torch's RNE rounding of the fp32 ones;
    LayerNorm tensors are the fp32 values themselves"""
    c1, p1 = pa.read_checkpoint(V1)
    c2, p2 = pa.read_checkpoint(V2)
    assert c1.channels == c2.channels and c1.num_layers == c2.num_layers
    t1, t2 = _tensors(c1, p1), _tensors(c2, p2)
    for k in range(16):
        want = pa.round_bf16(t1[k]) if k in BF16_TENSORS else t1[k]
        assert np.array_equal(t2[k].view(np.uint32), want.view(np.uint32)), k


@pytest.mark.parametrize("version,ref", [(1, V1), (2, V2)])
def test_writer_reproduces_reference_bytes(tmp_path, version, ref):
    c, p = pa.read_checkpoint(V1)
    out = tmp_path / f"v{version}.bin"
    pa.write_checkpoint(out, c, p, version)
    assert out.read_bytes() == open(ref, "rb").read()


def test_reader_rejects_bad_files(tmp_path):
    raw = bytearray(open(V1, "rb").read())
    bad = tmp_path / "bad.bin"
    for mutate in ("magic", "version", "truncate"):
        b = bytearray(raw)
        if mutate == "magic":
            b[0] ^= 1
        elif mutate == "version":
            b[4:8] = (3).to_bytes(4, "little")
        else:
            b = b[:len(b) - 100]
        bad.write_bytes(bytes(b))
        with pytest.raises(RuntimeError):
            pa.read_checkpoint(bad)


def test_tokenizer_decodes_reference_file():
    tk = pa.Tokenizer(TOK)
    assert tk.init_ok == 1 and tk.vocab_size == len(EXP["offsets"]) - 1
    pieces = EXP["pieces"].tobytes()
    offs = EXP["offsets"]
    for i in range(tk.vocab_size):
        assert tk.decode(i) == pieces[offs[i]:offs[i + 1]], i
    assert tk.decode(tk.vocab_size) is None  # "invalid token id" (paged_infer.c:917-922)
    tk.free()
    assert tk.init_ok == 0
    missing = pa.Tokenizer(os.path.join(GOLD, "no_such_tokenizer.bin"))
    assert missing.init_ok == 0 and missing.decode(0) is None


def test_safe_printf_filters_control_bytes(capfd):
    libc = ctypes.CDLL(None)
    libc.fflush(None)  # earlier tests' C stdio output
    capfd.readouterr()
    for piece in (b"A", b"\x01", b" ", b"tok7", b"\n", b""):
        pa.lib().safe_printf(piece)
    libc.fflush(None)
    assert capfd.readouterr().out == "A tok7\n"


def test_oracle_matches_reference_forward():
    """the oracle's paged decode of the checkpoint's model, token by token,
    against the reference PyTorch model's logits at every position"""
    c, p = pa.read_checkpoint(V1)
    oc_c = oc.cfg(c.max_seq_len, c.vocab_size, c.num_layers, c.num_heads, c.channels)
    dec = oc.PagedDecoder(p, oc_c, 1, 16, c.max_seq_len)
    worst = 0.0
    for t, tok in enumerate(EXP["tokens"]):
        _, lg = dec.step(np.array([tok], np.int32))
        worst = max(worst, float(np.abs(lg[0] - EXP["logits"][t]).max()))
    dec.close()
    scale = float(np.abs(EXP["logits"]).max())
    assert worst <= 1e-5 * max(1.0, scale), (worst, scale)
