"""The N>1 decode path on CPU: `gloo` process groups of 2-4 ranks running the
sequence sharding with the oracle's paged decoder as each rank's engine, and
the END-OF-STEP GATHER SCHEDULE OF THE PRODUCT LIBRARY: every rank asks
libpaged_hip.so for its operations (hpa_comm_gather_plan -- the exact list
hpa_comm_gatherv posts as ncclSend / ncclRecv plus the root's local copy,
llm.c-paged_amd/csrc/hpa_comm.hip) and runs them over gloo point-to-point
messages.  The per-rank byte counts follow gpt2_decode_gather's bookkeeping
(rows x V x 4 for the logits, rows x 4 for the ids; paged_infer.c).

Sharding must not change any sequence's result: what the root assembles
equals, bit for bit, an unsharded decode of the whole batch (SURVEY.md 8e:
sequences are independent, no exchange inside a step).  Covers uneven row
counts, a rank with zero rows and a non-zero root.
"""
import os
import socket

import numpy as np
import pytest

import oracle_ctypes as oc
import pagedattn
import shard
import synth

SMALL = dict(maxT=64, V=500, L=2, NH=2, C=128)
STEPS = 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tokens(B, steps, V):
    return np.random.default_rng(123).integers(0, V, (steps, B)).astype(np.int32)


def _post_plan(dist, plan, send, recv):
    """post the library's schedule for this rank over gloo: SEND / RECV as
    point-to-point messages (byte buffers), COPY as the root's local copy;
    returns the pending requests"""
    import torch
    reqs = []
    for op, peer, off, nb in plan:
        if op == pagedattn.HPA_COMM_SEND:
            reqs.append(dist.isend(torch.from_numpy(send[:nb]), peer))
        elif op == pagedattn.HPA_COMM_RECV:
            reqs.append(dist.irecv(torch.from_numpy(recv[off:off + nb]), peer))
        else:
            recv[off:off + nb] = send[:nb]
    return reqs


def _worker(rank, world, port, rows, root, mode, out_path, nbuf=1):
    """nbuf = 1: each step's gather completes before the next step; nbuf = 2:
    gpt2_decode_gather's double buffering -- step k's gather (send / receive
    buffers k % 2) is still in flight while step k+1 fills the other pair, and
    a pair is reused only after the gather that last used it (two steps
    earlier) has completed"""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo = sum(rows[:rank])
        hi = lo + rows[rank]
        B = sum(rows)
        per = SMALL["V"] * 4 if mode == "logits" else 4  # gpt2_decode_gather: bytes per row
        nbytes = [r * per for r in rows]
        plan = pagedattn.gather_plan(world, rank, root, nbytes)
        params = synth.params(SMALL, seed=5)
        c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
        dec = oc.PagedDecoder(params, c, rows[rank], 8, SMALL["maxT"], page_seed=17 + rank) if rows[rank] else None
        toks = _tokens(B, STEPS, SMALL["V"])
        sends = [np.zeros(max(nbytes[rank], 1), np.uint8) for _ in range(nbuf)]
        recvs = [np.zeros(sum(nbytes), np.uint8) if rank == root else None for _ in range(nbuf)]
        got, pending = [], []  # pending: (requests, step) of gathers still in flight

        def complete(k):  # wait for step k's gather; the root keeps what it assembled
            reqs, step = pending.pop(0)
            assert step == k
            for r in reqs:
                r.wait()
            if rank == root:
                got.append(recvs[k % nbuf].view(np.float32 if mode == "logits" else np.int32).reshape(B, -1).copy())

        for t in range(STEPS):
            if pending and pending[0][1] <= t - nbuf:  # buffer pair t % nbuf is free again
                complete(pending[0][1])
            send = sends[t % nbuf]
            if dec is not None:
                nxt, logits = dec.step(toks[t, lo:hi])
                out = logits if mode == "logits" else nxt.astype(np.int32)
                send[:nbytes[rank]] = np.ascontiguousarray(out).view(np.uint8).ravel()
            pending.append((_post_plan(dist, plan, send, recvs[t % nbuf]), t))
        while pending:
            complete(pending[0][1])
        if dec is not None:
            dec.close()
        if rank == root:
            np.save(out_path, np.stack(got))
    finally:
        dist.destroy_process_group()


def _unsharded(B, mode):
    params = synth.params(SMALL, seed=5)
    c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
    dec = oc.PagedDecoder(params, c, B, 8, SMALL["maxT"], page_seed=99)
    toks = _tokens(B, STEPS, SMALL["V"])
    out = []
    for t in range(STEPS):
        nxt, logits = dec.step(toks[t])
        out.append(logits if mode == "logits" else nxt.astype(np.int32)[:, None])
    dec.close()
    return np.stack(out)


def _spawn(world, target, args):
    """stdlib spawn: torch is imported by the ranks only, never in the pytest
    process (a -m gpu session must not map torch's HIP runtime beside the
    library's, and two HIP runtimes in one process abort at exit).  A rank
    still alive after the join timeout is terminated, then killed, before the
    exit codes are checked, so a hung gloo call cannot outlive
    the test."""
    import multiprocessing
    ctx = multiprocessing.get_context("spawn")
    procs = [ctx.Process(target=target, args=(r, world, *args)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    for p in procs:
        if p.is_alive():
            p.terminate()
            p.join(5)
        if p.is_alive():
            p.kill()
            p.join(5)
    return [p.exitcode for p in procs]


@pytest.mark.parametrize("rows,root,mode,nbuf", [([3, 3], 0, "logits", 1), ([3, 2], 0, "logits", 1),
                                                 ([2, 2], 1, "ids", 1), ([2, 0, 3], 0, "logits", 1),
                                                 ([1, 2, 1, 2], 2, "logits", 1),
                                                 # double-buffered, overlapped with the next step
                                                 ([3, 2], 0, "logits", 2), ([2, 0, 3], 1, "ids", 2)])
def test_sharded_decode_through_library_gather_schedule(tmp_path, rows, root, mode, nbuf):
    world = len(rows)
    out = str(tmp_path / "root.npy")
    codes = _spawn(world, _worker, (_free_port(), rows, root, mode, out, nbuf))
    assert all(c == 0 for c in codes), codes
    got = np.load(out)
    want = _unsharded(sum(rows), mode)
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def test_gather_plan_matches_layout():
    """the schedule's offsets are hpa_comm_gather_layout's, its RECV count is
    the layout's post count, and every byte of the root's buffer is written
    exactly once (the RECVs and the COPY tile it)"""
    import ctypes
    L = pagedattn.lib()
    sz = ctypes.c_size_t
    for rows, root in [([3, 3], 0), ([4, 3, 0, 5], 0), ([2, 0, 7, 1, 0, 9, 3, 3], 5), ([0, 0, 4], 2), ([1], 0)]:
        n = len(rows)
        nb = [r * 40 for r in rows]
        off = (sz * n)()
        own = sz()
        for rank in range(n):
            posts = L.hpa_comm_gather_layout(n, rank, root, (sz * n)(*nb), off, ctypes.byref(own))
            plan = pagedattn.gather_plan(n, rank, root, nb)
            if rank != root:
                assert plan == ([(pagedattn.HPA_COMM_SEND, root, 0, nb[rank])] if nb[rank] else [])
                continue
            recvs = [p for p in plan if p[0] == pagedattn.HPA_COMM_RECV]
            assert len(recvs) == posts
            assert all(o == off[q] and b == nb[q] for _, q, o, b in recvs)
            cover = np.zeros(sum(nb), np.int32)
            for _, _, o, b in plan:
                cover[o:o + b] += 1
            assert (cover == 1).all()
    assert L.hpa_comm_gather_plan(2, 0, 0, (sz * 2)(8, 8), None, 0) == 2  # count only
    assert L.hpa_comm_gather_plan(2, 0, 0, (sz * 2)(8, 8), (pagedattn.HpaCommOp * 1)(), 1) == -1  # too small
    assert L.hpa_comm_gather_plan(2, 2, 0, (sz * 2)(8, 8), None, 0) == -1


def test_batch_layout():
    assert shard.batch_layout(64, 8, 3, "weak") == (512, 192, 256)
    assert shard.batch_layout(64, 8, 7, "strong") == (64, 56, 64)
    assert [shard.shard_range(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    with pytest.raises(ValueError):
        shard.shard_range(3, 4, 0)
