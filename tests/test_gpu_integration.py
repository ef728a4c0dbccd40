"""INTEGRATION.md is executable: its ctypes binding snippet and the C driver
(examples/decode_main.c) run on the GPU exactly as documented."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_ctypes_snippet_runs(hip):
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    code = re.search(r"## 3\. FFI binding.*?```python\n(.*?)```", text, re.S).group(1)
    cwd = os.getcwd()
    os.chdir(REPO)
    try:
        exec(compile(code, "INTEGRATION.md", "exec"), {})
    finally:
        os.chdir(cwd)


GOLD = os.path.join(REPO, "tests", "golden")


def _build_driver(tmp_path):
    libdir = os.path.join(REPO, "llm.c-paged_amd")
    exe = str(tmp_path / "decode_main")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", os.path.join(REPO, "examples", "decode_main.c"),
                    "-I" + os.path.join(REPO, "include"), "-L" + libdir, "-lpaged_hip", "-Wl,-rpath," + libdir,
                    "-o", exe], check=True)
    return exe


def _oracle_generate(params, c, prompts, new, sample):
    """the reference driver's loop on the oracle: every prompt token decoded
    in order, then `new` tokens, greedy or softmax + sample_mult with
    random_f32 coins from state 1337 + b (gpt2_decode_set_sampling)"""
    import numpy as np
    import oracle_ctypes as oc
    B, P = prompts.shape
    c = oc.cfg(c.max_seq_len, c.vocab_size, c.num_layers, c.num_heads, c.channels)
    dec = oc.PagedDecoder(params, c, B, 16, c.max_seq_len)
    sampler = oc.Sampler(B, seed=1337) if sample else None
    margins = []
    for t in range(P):
        nxt, logits = dec.step(prompts[:, t])
    out = []
    for t in range(new):
        if sampler is not None:
            nxt = sampler.sample(logits)
        s = np.sort(logits, -1)
        margins.append(s[:, -1] - s[:, -2])
        out.append(nxt)
        if t + 1 < new:
            nxt2, logits = dec.step(nxt)
            nxt = nxt2
    dec.close()
    return np.stack(out, 1), np.stack(margins, 1)


@pytest.mark.parametrize("mode", ["greedy", "sampled"])
def test_c_driver_matches_oracle(hip, tmp_path, mode):
    """examples/decode_main.c -- the reference main's flow (checkpoint,
    tokenizer, int32 prompt tokens, one-pass prefill, greedy or reference
    sampling, tokenizer printing) -- on the reference-written checkpoint and
    tokenizer (tests/golden); its ids equal the oracle driving the same loop
    token by token"""
    import numpy as np
    import pagedattn as pa
    exe = _build_driver(tmp_path)
    exp = np.load(os.path.join(GOLD, "ckpt_expected.npz"))
    B, P, N = 2, 8, 16
    prompts = exp["tokens"][:B * P].astype(np.int32).reshape(B, P)
    tok_file = tmp_path / "tokens.bin"
    prompts.tofile(tok_file)
    ids_file = tmp_path / "ids.bin"
    args = [exe, "-c", os.path.join(GOLD, "ckpt_v1.bin"), "-k", os.path.join(GOLD, "tokenizer.bin"), "-t",
            str(tok_file), "-b", str(B), "-p", str(P), "-n", str(N), "-o", str(ids_file)]
    if mode == "greedy":
        args.append("-g")
    r = subprocess.run(args, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    out = r.stdout
    assert b"tokens/s" in out and b"Finished!" in out
    ids = np.fromfile(ids_file, np.int32).reshape(B, P + N)
    assert np.array_equal(ids[:, :P], prompts)
    c, params = pa.read_checkpoint(os.path.join(GOLD, "ckpt_v1.bin"))
    want, margins = _oracle_generate(params, c, prompts, N, mode == "sampled")
    if mode == "greedy":  # every step's oracle margin is far above the fp32 logit differences
        assert margins.min() > 1e-4, margins.min()
    assert np.array_equal(ids[:, P:], want), (ids[:, P:], want)
    # the generated tokens of sequence 0 are printed through the tokenizer
    tk = pa.Tokenizer(os.path.join(GOLD, "tokenizer.bin"))
    def shown(piece):  # safe_printf (paged_infer.c:895-905): lone bytes only if printable or whitespace
        if piece is None or len(piece) == 0:
            return b""
        if len(piece) == 1 and not (0x20 <= piece[0] <= 0x7E or piece[0] in b"\t\n\v\f\r"):
            return b""
        return piece

    text = b"".join(shown(tk.decode(int(t))) for t in ids[0, P:])
    tk.free()
    assert text in out
