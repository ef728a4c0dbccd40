"""The drop-in block manager (llm.c-paged_amd/csrc/block_manager.c), host
logic only (pages from host malloc, no GPU):

 * the reference's own block_manager_test.c compiled UNCHANGED against the
   drop-in source (build container only: it needs /root/reference);
 * an alloc / fill / touch / evict / free trace replayed against the
   reference's trace (tests/golden/bm_trace_golden.npz, recorded from the
   reference block_manager.c by gen_golden.py): state identical after every op;
 * run-time capacity at decode sizes (64 sequences x 64 pages).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
REF_TEST = "/root/reference/block_manager_test.c"


@pytest.fixture(scope="module")
def pa():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "llm.c-paged_amd"), "-j8"], check=True)
    import pagedattn
    pagedattn.lib()
    return pagedattn


@pytest.mark.skipif(not os.path.exists(REF_TEST), reason="reference checkout absent (GPU box)")
def test_reference_block_manager_test_compiles_unchanged(tmp_path):
    exe = tmp_path / "bmt"
    src = open(REF_TEST, "rb").read()  # fed on stdin: compiled where it lies, never copied
    inc = ["-I", os.path.join(REPO, "include"), "-iquote", os.path.join(REPO, "llm.c-paged_amd", "csrc")]
    r = subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", *inc, "-x", "c", "-",
                        "-o", str(exe)], input=src, capture_output=True)
    assert r.returncode == 0, r.stderr.decode()
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "All tests passed!" in r.stdout


class _BM(ctypes.Structure):
    _fields_ = [("C", ctypes.c_int), ("blocks", ctypes.c_void_p),
                ("prompt_block_list", ctypes.POINTER(ctypes.POINTER(ctypes.c_int))),
                ("prompt_block_count", ctypes.POINTER(ctypes.c_int)), ("lru_epoch", ctypes.c_int)]


def test_trace_matches_reference(pa):
    g = np.load(os.path.join(GOLD, "bm_trace_golden.npz"))
    ops, state, meta = g["ops"], g["state"], g["meta"]
    maxb, maxp, bs, nq = [int(x) for x in meta]
    L = pa.lib()
    h = L.create_block_manager(4)
    L.bm_use_host_pages(h)
    bm = ctypes.cast(h, ctypes.POINTER(_BM)).contents
    blocks = ctypes.cast(bm.blocks, ctypes.POINTER(pa.KVBlock))
    last = -1
    for k, (op, p, arg) in enumerate(ops):
        ret = 0
        if op == 0:
            blk = L.request_block(h, int(p))
            ret = L.bm_block_index(h, blk) if blk else -1
            last = ret
        elif op == 1:
            if last >= 0:
                blocks[last].filled = int(arg)
            ret = last
        elif op == 2:
            if last >= 0:
                bm.lru_epoch += 1
                blocks[last].lru_counter = bm.lru_epoch
            ret = last
        elif op == 3:
            L.free_blocks_for_prompt(h, int(p))
        st = [ret, bm.lru_epoch, L.find_least_recently_used_block(h)]
        st += [blocks[i].prompt_id for i in range(maxb)]
        st += [blocks[i].filled if blocks[i].prompt_id >= 0 else 0 for i in range(maxb)]
        st += [blocks[i].lru_counter if blocks[i].prompt_id >= 0 else 0 for i in range(maxb)]
        st += [bm.prompt_block_count[q] for q in range(nq)]
        for q in range(nq):
            n = bm.prompt_block_count[q]
            st += [bm.prompt_block_list[q][i] if i < n else -1 for i in range(maxb)]
        assert np.array_equal(np.array(st, np.int32), state[k]), f"op {k} {op, p, arg}"
    L.destroy_block_manager(h)


def test_decode_capacity_first_fit_and_lists(pa):
    L = pa.lib()
    B, pages_per_seq = 64, 64
    h = L.create_block_manager_ex(768, B, B * pages_per_seq, 16, pages_per_seq)
    L.bm_use_host_pages(h)
    bm = ctypes.cast(h, ctypes.POINTER(_BM)).contents
    # interleaved growth like a decode batch: page ids are handed out in order
    got = []
    for step in range(pages_per_seq):
        for b in range(B):
            blk = L.request_block(h, b)
            got.append(L.bm_block_index(h, blk))
    assert got == list(range(B * pages_per_seq))
    assert L.bm_free_pages(h) == 0
    for b in (0, 13, 63):
        assert [bm.prompt_block_list[b][i] for i in range(pages_per_seq)] == \
            [b + B * i for i in range(pages_per_seq)]
    # a full per-prompt list refuses (the reference would overflow its row)
    assert not L.request_block(h, 5)
    # free one sequence: its pages are reused lowest-first
    L.free_blocks_for_prompt(h, 13)
    assert L.bm_free_pages(h) == pages_per_seq
    blk = L.request_block(h, 13)
    assert L.bm_block_index(h, blk) == 13
    L.destroy_block_manager(h)


def test_invalid_prompt_and_empty_collect(pa):
    L = pa.lib()
    h = L.create_block_manager(8)
    L.bm_use_host_pages(h)
    assert not L.request_block(h, -1)
    assert not L.request_block(h, 100)
    n = ctypes.c_int(-5)
    assert L.collect_kv_blocks(h, 3, ctypes.byref(n)) is None and n.value == 0
    assert not L.get_current_block(h, 3)
    L.destroy_block_manager(h)
