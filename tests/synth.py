"""Seeded synthetic GPT-2 weights and llm.c v1 checkpoint writer for tests.

Real GPT-2 weights cannot be fetched offline, so every
parity test runs on seeded synthetic weights with GPT-2 shapes.  The layout is
the llm.c checkpoint order (paged_infer.c:308-326, :436-502; writer
train_gpt2.py:300-326): 256 x int32 header [20240326, 1, maxT, V, L, NH, C]
followed by the 16 fp32 tensors.
"""
import numpy as np

MAGIC, VERSION_FP32 = 20240326, 1


def sizes(c):
    V, maxT, L, C = c["V"], c["maxT"], c["L"], c["C"]
    return [V * C, maxT * C, L * C, L * C, L * 3 * C * C, L * 3 * C, L * C * C, L * C,
            L * C, L * C, L * 4 * C * C, L * 4 * C, L * C * 4 * C, L * C, C, C]


def params(c, seed=0):
    """matrices ~U(-a,a) with std 0.02, biases small, LN weight ~1, LN bias ~0."""
    rng = np.random.default_rng(seed)
    out = []
    a = 0.02 * np.sqrt(3.0)
    for i, n in enumerate(sizes(c)):
        if i in (2, 8, 14):      # ln weights
            t = 1.0 + rng.uniform(-0.1, 0.1, n)
        elif i in (3, 9, 15):    # ln biases
            t = rng.uniform(-0.05, 0.05, n)
        elif i in (5, 7, 11, 13):  # linear biases
            t = rng.uniform(-0.02, 0.02, n)
        elif i == 1:             # wpe
            t = rng.uniform(-0.01 * np.sqrt(3.0), 0.01 * np.sqrt(3.0), n)
        else:
            t = rng.uniform(-a, a, n)
        out.append(t.astype(np.float32))
    return np.concatenate(out)


def write_checkpoint(path, c, p):
    hdr = np.zeros(256, np.int32)
    hdr[:7] = [MAGIC, VERSION_FP32, c["maxT"], c["V"], c["L"], c["NH"], c["C"]]
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(np.ascontiguousarray(p, np.float32).tobytes())


def offsets(c):
    s = sizes(c)
    o = np.concatenate([[0], np.cumsum(s)[:-1]])
    return [int(x) for x in o]
