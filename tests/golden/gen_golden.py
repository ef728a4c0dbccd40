#!/usr/bin/env python3
"""Generate the committed golden fixtures by running the REFERENCE itself.

Runs in the build container only (needs /root/reference and oracle/_ref built
by `make -C oracle ref`).  The reference sources are compiled where they lie
(oracle/refdrv/*.c include them by path); nothing of them is copied here.
Outputs (small .npz files of inputs + expected outputs, no pickles):

  attn_paged_golden.npz   reference attention_paged (paged_infer.c:163-240),
                          BLOCK_SIZE 32, randomly permuted page placement,
                          several (B,T,C,NH,offset) cases
  matmul_golden.npz       reference matmul_forward / matmul_cached (:92-160)
  bm_trace_golden.npz     reference block_manager.c op trace (alloc / fill /
                          touch / evict / free) with the state after each op
  forward_golden.npz      reference train_scratch.c full-L forward logits
                          (train_scratch.c:658-798) for a small synthetic model

Usage:  python tests/golden/gen_golden.py   (writes next to this file)
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import synth  # noqa: E402

REF_DIR = os.path.join(REPO, "oracle", "_ref")
_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)


def fp(a):
    return a.ctypes.data_as(_F)


def load_ref():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    paged = ctypes.CDLL(os.path.join(REF_DIR, "libref_paged.so"))
    scratch = ctypes.CDLL(os.path.join(REF_DIR, "libref_scratch.so"))
    paged.attention_paged.argtypes = [_F, _F, _F, _F, ctypes.POINTER(_F), ctypes.POINTER(_F)] + \
        [ctypes.c_int] * 5
    paged.matmul_forward.argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
    paged.matmul_cached.argtypes = [_F, _F, _F, _F] + [ctypes.c_int] * 4
    for n in ["ref_bm_create"]:
        getattr(paged, n).restype = ctypes.c_void_p
    paged.ref_bm_create.argtypes = [ctypes.c_int]
    paged.request_block.restype = ctypes.c_void_p
    paged.request_block.argtypes = [ctypes.c_void_p, ctypes.c_int]
    paged.get_current_block.restype = ctypes.c_void_p
    paged.get_current_block.argtypes = [ctypes.c_void_p, ctypes.c_int]
    paged.free_blocks_for_prompt.argtypes = [ctypes.c_void_p, ctypes.c_int]
    paged.find_least_recently_used_block.argtypes = [ctypes.c_void_p]
    paged.get_next_block_id.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    for n in ["ref_bm_block_prompt", "ref_bm_block_filled", "ref_bm_block_lru",
              "ref_bm_prompt_count", "ref_bm_touch"]:
        getattr(paged, n).argtypes = [ctypes.c_void_p, ctypes.c_int]
    paged.ref_bm_prompt_list.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    paged.ref_bm_set_filled.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    paged.ref_bm_block_index.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    paged.ref_bm_lru_epoch.argtypes = [ctypes.c_void_p]
    scratch.ref_full_forward.argtypes = [ctypes.c_char_p, _I, ctypes.c_int, ctypes.c_int, _F]
    return paged, scratch


class quiet_stdout:
    """The reference prints from inside the allocator; silence fd 1."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        self.null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.null, 1)

    def __exit__(self, *a):
        libc = ctypes.CDLL(None)
        libc.fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.null)
        os.close(self.saved)


def gen_attention(paged):
    bs = paged.ref_bm_block_size()
    rng = np.random.default_rng(20240326)
    cases = [  # B, T, C, NH, offset
        (1, 20, 10, 2, 0),     # test_paged_attn.c's shape (hs=5)
        (2, 33, 64, 4, 0),     # crosses one page boundary
        (1, 32, 128, 2, 17),   # hs=64, window offset like the sliding driver
        (2, 40, 64, 4, 50),    # starts in page 1, spans 3 pages
        (1, 1, 128, 2, 95),    # single-row decode-like query at the end of page 2
    ]
    out = {}
    for ci, (B, T, C, NH, off) in enumerate(cases):
        npages = (off + T + bs - 1) // bs
        inp = rng.uniform(-2, 2, size=(B, T, 3 * C)).astype(np.float32)
        kpool = rng.uniform(-2, 2, size=(npages, bs, C)).astype(np.float32)
        vpool = rng.uniform(-2, 2, size=(npages, bs, C)).astype(np.float32)
        order = rng.permutation(npages).astype(np.int32)
        o = np.zeros((B, T, C), np.float32)
        pre = np.zeros((B, NH, T, T), np.float32)
        att = np.zeros((B, NH, T, T), np.float32)
        kb = (_F * npages)(*[fp(kpool[p]) for p in order])
        vb = (_F * npages)(*[fp(vpool[p]) for p in order])
        paged.attention_paged(fp(o), fp(pre), fp(att), fp(inp), kb, vb, B, T, C, NH, off)
        for k, v in dict(shape=np.array([B, T, C, NH, off, bs], np.int32), inp=inp, kpool=kpool,
                         vpool=vpool, order=order, out=o, preatt=pre, att=att).items():
            out[f"c{ci}_{k}"] = v
    out["ncases"] = np.array(len(cases), np.int32)
    np.savez(os.path.join(HERE, "attn_paged_golden.npz"), **out)


def gen_matmul(paged):
    rng = np.random.default_rng(7)
    B, T, C = 3, 5, 64
    OC = 3 * C
    inp = rng.uniform(-1, 1, (B, T, C)).astype(np.float32)
    w = rng.uniform(-0.1, 0.1, (OC, C)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, (OC,)).astype(np.float32)
    fwd = np.zeros((B, T, OC), np.float32)
    cached = np.zeros((B, T, OC), np.float32)
    paged.matmul_forward(fp(fwd), fp(inp), fp(w), fp(b), B, T, C, OC)
    paged.matmul_cached(fp(cached), fp(inp), fp(w), fp(b), B, T, C, OC)
    np.savez(os.path.join(HERE, "matmul_golden.npz"), inp=inp, w=w, b=b, fwd=fwd, cached=cached,
             shape=np.array([B, T, C, OC], np.int32))


# op codes for the allocator trace
OP_REQUEST, OP_FILL, OP_TOUCH, OP_FREE = 0, 1, 2, 3


def gen_bm_trace(paged):
    """A deterministic op sequence that exercises first-fit allocation, the
    per-prompt page lists, LRU whole-prompt eviction (block_manager.c:92-113)
    and free/reuse; records the reference's full state after every op."""
    maxb = paged.ref_bm_max_blocks()
    maxp = paged.ref_bm_max_prompts()
    rng = np.random.default_rng(99)
    ops = []
    # fill the pool across 7 prompts, interleaved
    for i in range(maxb):
        ops.append((OP_REQUEST, int(rng.integers(0, 7)), 0))
        if i % 3 == 0:
            ops.append((OP_FILL, -1, int(rng.integers(1, 33))))  # fill last-returned page
        if i % 5 == 0:
            ops.append((OP_TOUCH, -1, 0))
    # pool is full: next requests evict whole LRU prompts
    for i in range(12):
        ops.append((OP_REQUEST, int(rng.integers(0, 9)), 0))
        if i % 4 == 1:
            ops.append((OP_FREE, int(rng.integers(0, 9)), 0))
    ops = np.array(ops, np.int32)
    res = []
    with quiet_stdout():
        m = paged.ref_bm_create(4)
        last = -1
        for op, p, arg in ops:
            ret = 0
            if op == OP_REQUEST:
                blk = paged.request_block(m, int(p))
                ret = paged.ref_bm_block_index(m, blk)
                last = ret
            elif op == OP_FILL:
                if last >= 0:
                    paged.ref_bm_set_filled(m, last, int(arg))
                ret = last
            elif op == OP_TOUCH:
                if last >= 0:
                    paged.ref_bm_touch(m, last)
                ret = last
            elif op == OP_FREE:
                paged.free_blocks_for_prompt(m, int(p))
            st = [ret, paged.ref_bm_lru_epoch(m), paged.find_least_recently_used_block(m)]
            st += [paged.ref_bm_block_prompt(m, i) for i in range(maxb)]
            st += [paged.ref_bm_block_filled(m, i) if paged.ref_bm_block_prompt(m, i) >= 0 else 0
                   for i in range(maxb)]
            st += [paged.ref_bm_block_lru(m, i) if paged.ref_bm_block_prompt(m, i) >= 0 else 0
                   for i in range(maxb)]
            st += [paged.ref_bm_prompt_count(m, q) for q in range(10)]
            for q in range(10):
                n = paged.ref_bm_prompt_count(m, q)
                st += [paged.ref_bm_prompt_list(m, q, i) if i < n else -1 for i in range(maxb)]
            res.append(st)
    np.savez_compressed(os.path.join(HERE, "bm_trace_golden.npz"), ops=ops, state=np.array(res, np.int32),
             meta=np.array([maxb, maxp, paged.ref_bm_block_size(), 10], np.int32))


def gen_forward(scratch):
    c = dict(maxT=64, V=1000, L=2, NH=4, C=64)
    params = synth.params(c, seed=1234)
    B, T = 2, 24
    rng = np.random.default_rng(5)
    tokens = rng.integers(0, c["V"], (B, T)).astype(np.int32)
    logits = np.zeros((B, T, c["V"]), np.float32)
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "synth.bin")
        synth.write_checkpoint(ck, c, params)
        with quiet_stdout():
            scratch.ref_full_forward(ck.encode(), tokens.ctypes.data_as(_I), B, T, fp(logits))
    np.savez(os.path.join(HERE, "forward_golden.npz"), params=params, tokens=tokens, logits=logits,
             cfg=np.array([c["maxT"], c["V"], c["L"], c["NH"], c["C"]], np.int32))


def main():
    paged, scratch = load_ref()
    gen_attention(paged)
    gen_matmul(paged)
    gen_bm_trace(paged)
    gen_forward(scratch)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
