"""The N>1 decode path on CPU: world_size-2 `gloo` process groups running
the sequence sharding (llm.c-paged_amd/shard.py, the same code bench.py
drives over RCCL) with the oracle's paged decoder as each rank's engine.

Sharding must not change any sequence's result: the logits and greedy ids
gathered to rank 0 equal, bit for bit, an unsharded decode of the whole
batch (sequences are independent, no exchange inside a step).
"""
import os
import socket

import numpy as np
import pytest

import oracle_ctypes as oc
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


def _worker(rank, world, port, batch, scaling, mode, out_path, nbuf=1):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, lo, hi = shard.batch_layout(batch, world, rank, scaling)
        counts = [shard.batch_layout(batch, world, r, scaling) for r in range(world)]
        counts = [h - l for _, l, h in counts]
        params = synth.params(SMALL, seed=5)
        c = oc.cfg(SMALL["maxT"], SMALL["V"], SMALL["L"], SMALL["NH"], SMALL["C"])
        dec = oc.PagedDecoder(params, c, hi - lo, 8, SMALL["maxT"], page_seed=17 + rank)
        g = shard.StepGather(dist, world, rank, counts, SMALL["V"], mode, "cpu", nbuf=nbuf)
        toks = _tokens(B, STEPS, SMALL["V"])
        got = []
        for t in range(STEPS):
            nxt, logits = dec.step(toks[t, lo:hi])
            i = t % nbuf
            if nbuf > 1 and rank == 0 and t >= nbuf:  # the gather of step t - nbuf, read before reuse
                g.wait(i)
                got.append(g.result(i).numpy().copy())
            g.wait(i)
            buf = g.buffer(i)
            if mode == "logits":
                buf[:hi - lo] = torch.from_numpy(logits)
            else:
                buf[:hi - lo, 0] = torch.from_numpy(nxt)
            g.gather(i, async_op=nbuf > 1)
            if rank == 0 and nbuf == 1:
                got.append(g.result().numpy().copy())
        if nbuf > 1:  # drain: the last nbuf steps, in order
            for t in range(STEPS - nbuf, STEPS):
                g.wait(t % nbuf)
                if rank == 0:
                    got.append(g.result(t % nbuf).numpy().copy())
        dec.close()
        if rank == 0:
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
        out.append(logits if mode == "logits" else nxt)
    dec.close()
    return np.stack(out)


@pytest.mark.parametrize("batch,scaling,mode,nbuf", [(3, "weak", "logits", 1), (5, "strong", "logits", 1),
                                                     (4, "weak", "ids", 1), (3, "weak", "logits", 2)])
def test_two_rank_sharded_decode_equals_unsharded(tmp_path, batch, scaling, mode, nbuf):
    """nbuf = 2: the double-buffered asynchronous gather bench.py overlaps
    with the next step"""
    # stdlib spawn: torch is imported by the ranks only, never in the pytest
    # process (a -m gpu session must not map torch's HIP runtime beside the
    # library's, and two HIP runtimes in one process abort at exit)
    import multiprocessing
    world = 2
    out = str(tmp_path / "rank0.npy")
    ctx = multiprocessing.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, scaling, mode, out, nbuf)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = np.load(out)
    B = batch * world if scaling == "weak" else batch
    want = _unsharded(B, mode)
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def test_batch_layout():
    assert shard.batch_layout(64, 8, 3, "weak") == (512, 192, 256)
    assert shard.batch_layout(64, 8, 7, "strong") == (64, 56, 64)
    assert [shard.shard_range(10, 4, r) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    with pytest.raises(ValueError):
        shard.shard_range(3, 4, 0)
