"""The N>1 decode path with the HIP engine, on the one GPU of
the test box.

* Two processes, each a HIP engine (libpaged_hip.so on device 0) decoding
  its shard of the batch (shard.batch_layout), exchanging through a
  world_size-2 gloo group (RCCL refuses two ranks on one device, so the
  transport here is gloo; the engines and the sharding are the product's).
  Rank 0's gathered logits and greedy ids equal an unsharded HIP decode of
  the whole batch bit for bit (same attention split count on both sides:
  GEMM rows never depend on M, so sharding changes no arithmetic).
* The C library's RCCL gather (hpa_comm_* + gpt2_decode_shard /
  gpt2_decode_gather, what bench.py runs at N > 1) on a 1-rank communicator:
  the double-buffered gather returns exactly the engine's logits and ids.
"""
import ctypes
import multiprocessing
import os
import socket

import numpy as np
import pytest
import shard
import synth

pytestmark = pytest.mark.gpu

SMALL = dict(maxT=128, V=1000, L=2, NH=2, C=128)
STEPS = 8
SPLITS = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tokens(B, V):
    return np.random.default_rng(321).integers(0, V, (STEPS, B)).astype(np.int32)


def _engine(hip, B):
    m = hip.Model(SMALL, params=synth.params(SMALL, seed=8))
    m.decode_init(B, 16, SMALL["maxT"])
    # five launches per layer: two processes share the one GPU here, and the
    # persistent layer needs every CU for itself (test_gpu_layer.py covers
    # its sharded == unsharded property in one process)
    m.set_layer_kernel(0)
    assert m.set_attn_splits(SPLITS) == SPLITS
    m.set_graph(True)
    return m


def _worker(rank, world, port, batch, scaling, out_path):
    import torch
    import torch.distributed as dist
    import pagedattn as hip
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hip.init(0)
        B, lo, hi = shard.batch_layout(batch, world, rank, scaling)
        counts = [h - l for _, l, h in (shard.batch_layout(batch, world, r, scaling) for r in range(world))]
        m = _engine(hip, hi - lo)
        toks = _tokens(B, SMALL["V"])
        logits, ids = [], []
        for t in range(STEPS):
            nxt = m.step(toks[t, lo:hi])
            lg = torch.zeros(max(counts), SMALL["V"])
            lg[:hi - lo] = torch.from_numpy(m.logits())
            nx = torch.zeros(max(counts), dtype=torch.int32)
            nx[:hi - lo] = torch.from_numpy(nxt)
            gl = [torch.zeros_like(lg) for _ in range(world)] if rank == 0 else None
            gi = [torch.zeros_like(nx) for _ in range(world)] if rank == 0 else None
            dist.gather(lg, gl, dst=0)
            dist.gather(nx, gi, dst=0)
            if rank == 0:
                logits.append(np.concatenate([g[:n].numpy() for g, n in zip(gl, counts)]))
                ids.append(np.concatenate([g[:n].numpy() for g, n in zip(gi, counts)]))
        m.close()
        if rank == 0:
            np.savez(out_path, logits=np.stack(logits), ids=np.stack(ids))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch,scaling", [(6, "strong"), (7, "strong"), (4, "weak")])
def test_two_hip_engines_sharded_equal_unsharded(hip, tmp_path, batch, scaling):
    world = 2
    out = str(tmp_path / "rank0.npz")
    # stdlib spawn: torch is imported by the ranks only, never in the pytest
    # process (its bundled HIP runtime beside the library's aborts at exit)
    ctx = multiprocessing.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, scaling, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = np.load(out)
    B = batch * world if scaling == "weak" else batch
    m = _engine(hip, B)
    toks = _tokens(B, SMALL["V"])
    want_l, want_i = [], []
    for t in range(STEPS):
        want_i.append(m.step(toks[t]))
        want_l.append(m.logits())
    m.close()
    assert np.array_equal(got["ids"], np.stack(want_i))
    assert np.array_equal(got["logits"], np.stack(want_l))


def test_rccl_gather_one_rank(hip):
    """hpa_comm (RCCL) + gpt2_decode_shard/gather on a 1-rank communicator:
    the asynchronous double-buffered gather of every step equals the engine's
    own logits / ids of that step"""
    L = hip.lib()
    n = L.hpa_comm_id_bytes()
    assert n >= 128
    uid = ctypes.create_string_buffer(n)
    hip.check(L.hpa_comm_unique_id(uid, n), "unique id")
    hip.check(L.hpa_comm_init(1, 0, uid), "comm init")
    try:
        assert L.hpa_comm_size() == 1 and L.hpa_comm_rank() == 0
        B = 5
        m = _engine(hip, B)
        m.shard([B], root=0)
        toks = _tokens(B, SMALL["V"])
        for t in range(STEPS):
            what = t % 2
            nxt = m.step(toks[t])
            lg = m.logits()
            m.gather(what)
            got = m.gathered(B, what)
            assert np.array_equal(got, lg if what == 0 else nxt), t
        m.close()
    finally:
        hip.check(L.hpa_comm_destroy(), "comm destroy")


def test_rccl_single_process_init_all_barrier_and_max(hip):
    """SURVEY.md 8e's single-process form (ncclCommInitAll over the devices
    one process drives; here the box's one device), the timing helpers
    bench.py uses at N > 1 (hpa_comm_barrier / hpa_comm_allreduce_max), and
    the engine's gather on that communicator"""
    L = hip.lib()
    devs = (ctypes.c_int * 1)(0)
    hip.check(L.hpa_comm_init_all(1, devs), "init_all")
    try:
        assert L.hpa_comm_size() == 1 and L.hpa_comm_rank() == 0
        hip.check(L.hpa_comm_use(0), "use")
        hip.check(L.hpa_comm_barrier(), "barrier")
        v = ctypes.c_double(3.25)
        hip.check(L.hpa_comm_allreduce_max(ctypes.byref(v)), "max")
        assert v.value == 3.25
        B = 3
        m = _engine(hip, B)
        m.shard([B], root=0)
        toks = _tokens(B, SMALL["V"])
        for t in range(3):
            nxt = m.step(toks[t])
            m.gather(1)
            assert np.array_equal(m.gathered(B, 1), nxt)
        m.close()
    finally:
        hip.check(L.hpa_comm_destroy(), "comm destroy")


# ---- BASELINE config 4's per-rank work at model size:
# GPT-2 124M, B = 64 split 32 / 32 over two engine processes on the one GPU,
# identical K/V (the fill hashes the global sequence index) to ~1000 tokens,
# 8 steps; every row's logits and greedy id equal the unsharded B = 64 engine
# bit for bit.  Both sides use five launches per layer with the global batch's
# attention split count and logits form (what gpt2_decode_shard picks: the
# ring logits form at a global batch of 64, HPA_LOGITS_FORM in the shard
# processes, which have no communicator to tell them), so the arithmetic is
# the same; the shards hand their rows over by file (the RCCL gather of this
# path is tested above on a 1-rank communicator).
GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
C4_CTX, C4_STEPS, C4_B = 990, 8, 64


def _c4_engine(hip, B, lo):
    m = hip.Model(GPT2_124M, params=synth.params(GPT2_124M, seed=41))
    m.decode_init(B, 16, GPT2_124M["maxT"])
    m.set_layer_kernel(0)
    m.set_attn_splits(hip.lib().hpa_attn_pick_splits(C4_B, GPT2_124M["NH"], GPT2_124M["maxT"], 0))
    m.set_graph(True)
    m.fill_random(C4_CTX, seed=7, seq_offset=lo)
    return m


def _c4_tokens():
    return np.random.default_rng(44).integers(0, GPT2_124M["V"], (C4_STEPS, C4_B)).astype(np.int32)


def _c4_worker(lo, hi, out_path):
    os.environ["HPA_LOGITS_FORM"] = "ring"  # the global batch's form (launch_logits_resident)
    import pagedattn as hip
    hip.init(0)
    m = _c4_engine(hip, hi - lo, lo)
    toks = _c4_tokens()
    ids, lg = [], []
    for t in range(C4_STEPS):
        ids.append(m.step(toks[t, lo:hi]))
        lg.append(m.logits())
    m.close()
    np.savez(out_path, ids=np.stack(ids), logits=np.stack(lg))


def test_config4_shards_at_model_size_equal_unsharded(hip, tmp_path):
    ctx = multiprocessing.get_context("spawn")
    halves = [(0, 32), (32, 64)]
    outs = [str(tmp_path / f"shard{r}.npz") for r in range(2)]
    procs = [ctx.Process(target=_c4_worker, args=(lo, hi, o)) for (lo, hi), o in zip(halves, outs)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = [np.load(o) for o in outs]
    m = _c4_engine(hip, C4_B, 0)
    toks = _c4_tokens()
    for t in range(C4_STEPS):
        want_ids = m.step(toks[t])
        want_lg = m.logits()
        assert np.array_equal(np.concatenate([g["ids"][t] for g in got]), want_ids), t
        assert np.array_equal(np.concatenate([g["logits"][t] for g in got]), want_lg), t
    m.close()
