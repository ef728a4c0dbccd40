"""The N>1 decode path with the HIP engine, on the one GPU of
the test box.

* Two processes, each a HIP engine (libpaged_hip.so on device 0) decoding
  its shard of the batch (shard.batch_layout), exchanging through a
  world_size-2 gloo group on the library's own gather schedule
  (hpa_comm_gather_plan, what hpa_comm_gatherv posts over RCCL; RCCL refuses
  two ranks on one device, so the transport here is gloo; the engines, the
  sharding and the schedule are the product's).
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
import oracle_ctypes as oc
import pytest
import shard
import synth
from test_gpu_decode import LOGIT_TOL, IdCheck

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
        from test_multi_rank import _post_plan

        def _run_plan(dist, plan, send, recv):
            for r in _post_plan(dist, plan, send, recv):
                r.wait()
        V = SMALL["V"]
        plan_l = hip.gather_plan(world, rank, 0, [n * V * 4 for n in counts])  # gpt2_decode_gather's bytes
        plan_i = hip.gather_plan(world, rank, 0, [n * 4 for n in counts])
        logits, ids = [], []
        for t in range(STEPS):
            nxt = m.step(toks[t, lo:hi])
            rl = np.zeros(B * V * 4, np.uint8) if rank == 0 else None
            ri = np.zeros(B * 4, np.uint8) if rank == 0 else None
            _run_plan(dist, plan_l, np.ascontiguousarray(m.logits(), np.float32).view(np.uint8).ravel(), rl)
            _run_plan(dist, plan_i, np.ascontiguousarray(nxt, np.int32).view(np.uint8).ravel(), ri)
            if rank == 0:
                logits.append(rl.view(np.float32).reshape(B, V))
                ids.append(ri.view(np.int32))
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
    for p in procs:  # a hung rank must not outlive the test
        if p.is_alive():
            p.terminate()
            p.join(5)
        if p.is_alive():
            p.kill()
            p.join(5)
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
        from conftest import runtime_mapped
        libs = runtime_mapped()
        print(f"runtime libraries mapped: {libs}")
        assert any("librccl" in x and x.startswith("/opt/rocm") for x in libs), libs
        assert not any("/torch/" in x for x in libs), libs
        assert L.hpa_comm_size() == 1 and L.hpa_comm_rank() == 0
        # the gather's compute -> comm hand-off is a device word on MI355X
        # (stream value ops; an event only where the device lacks them)
        assert L.hpa_stream_value_ops() == 1
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
        # the grouped form one thread uses for every device's engine
        handles = (ctypes.c_void_p * 1)(m.h)
        for t in range(3, 5):
            nxt = m.step(toks[t])
            hip.check(L.gpt2_decode_gather_all(handles, 1, 1), "gather_all")
            assert np.array_equal(m.gathered(B, 1), nxt)
        m.close()
    finally:
        hip.check(L.hpa_comm_destroy(), "comm destroy")


# ---- BASELINE config 4's per-rank work at model size, on the product's
# DEFAULT path: GPT-2 124M, ctx ~1000, page 16, the
# engine's default layer form (the persistent chain), graph replay, no HPA_*
# knob in any process (a worker refuses to run with one set).  Each rank is a
# process of its own, spawned one after another (the persistent kernel needs
# every CU), holding one shard: its own engine + page pool, K/V filled from the
# GLOBAL sequence index (identical to the unsharded engine's), a 1-rank RCCL
# communicator and the end-of-step gather every step (the N>1 bench's gather
# beside the default layer form).  Per case:
#   * picks "global" (gpt2_decode_set_global_batch(total), total <= 64): every
#     row's logits and id equal the unsharded engine of `total` rows bit for bit;
#   * picks "local" (the N>1 default): each shard equals a single-GPU engine of
#     its rows bit for bit (what the bench's --emulate-rank times), the
#     unsharded engine within the layer-form reassociation bound, and the
#     oracle on identical K/V (<= 2e-4, ids outside near-ties).
# Cases: weak 64 + 64 (config 4's per-rank batch; its global batch of 128 is
# above 64, so both pick modes are the local one), strong 32 + 32 and 8 x 8.
# Reference per-rank work: paged_infer.c:575-729.
GPT2_124M = dict(maxT=1024, V=50257, L=12, NH=12, C=768)
C4_CTX, C4_STEPS, C4_SEED = 990, 8, 41
FORM_TOL = 2e-5  # fcproj's K-part sum reassociates between layer forms (test_gpu_layer.py)


def _c4_tokens(total):
    return np.random.default_rng(44).integers(0, GPT2_124M["V"], (C4_STEPS, total)).astype(np.int32)


def _c4_engine(hip, params, lo, hi):
    m = hip.Model(GPT2_124M, params=params)
    m.decode_init(hi - lo, 16, GPT2_124M["maxT"])
    m.set_graph(True)
    m.fill_random(C4_CTX, seed=7, seq_offset=lo)
    return m


def _c4_rank(lo, hi, total, picks, out_path):
    """one rank of the sharded decode, in its own process"""
    knobs = sorted(k for k in os.environ if k.startswith("HPA_"))
    if knobs:
        raise SystemExit(f"product env knobs set in a config-4 rank: {knobs}")
    import pagedattn as hip
    hip.init(0)
    L = hip.lib()
    params = hip.synthetic_params(GPT2_124M, seed=C4_SEED)
    toks = _c4_tokens(total)
    n = L.hpa_comm_id_bytes()
    uid = ctypes.create_string_buffer(n)
    hip.check(L.hpa_comm_unique_id(uid, n), "unique id")
    hip.check(L.hpa_comm_init(1, 0, uid), "comm init")
    try:
        m = _c4_engine(hip, params, lo, hi)
        if picks == "global":
            m.set_global_batch(total)
        m.shard([hi - lo], root=0)
        ids, lg = [], []
        for t in range(C4_STEPS):
            ids.append(m.step(toks[t, lo:hi]))
            m.gather(0)  # the RCCL end-of-step gather of this step's logits
            g = m.gathered(hi - lo, 0)
            assert np.array_equal(g, m.logits()), t
            lg.append(g)
        m.status()  # no in-launch wait timed out
        # as the N>1 bench runs: steps enqueued back to back, each step's RCCL
        # gather on the comm stream beside the next step's persistent chain
        # launches (every chain workgroup must still become resident: ADVICE r3)
        for t in range(C4_STEPS):
            m.step_async(toks[t, lo:hi])
            m.gather(0)
        assert np.array_equal(m.gathered(hi - lo, 0), m.logits())
        m.status()
        info = np.array([m.layer_form(), m.attn_splits(), m.attn_waves()], np.int32)
        m.close()
    finally:
        hip.check(L.hpa_comm_destroy(), "comm destroy")
    np.savez(out_path, ids=np.stack(ids), logits=np.stack(lg), info=info)


def _run_ranks(tmp_path, shards, total, picks):
    ctx = multiprocessing.get_context("spawn")
    got = []
    for r, (lo, hi) in enumerate(shards):  # one after another: the persistent kernel needs every CU
        out = str(tmp_path / f"rank{r}.npz")
        p = ctx.Process(target=_c4_rank, args=(lo, hi, total, picks, out))
        p.start()
        p.join(240)
        if p.is_alive():  # a hung rank must not outlive the test
            p.terminate()
            p.join(5)
        if p.is_alive():
            p.kill()
            p.join(5)
        assert p.exitcode == 0, (r, p.exitcode)
        got.append(np.load(out))
        print(f"rank {r} ({lo}..{hi}, picks {picks}) done: form / splits / waves {tuple(got[-1]['info'])}",
              flush=True)
    return got


def _single(hip, params, lo, hi, total):
    """an unsharded engine of rows lo..hi (its own picks): ids, logits per step"""
    m = _c4_engine(hip, params, lo, hi)
    toks = _c4_tokens(total)
    ids, lg = [], []
    for t in range(C4_STEPS):
        ids.append(m.step(toks[t, lo:hi]))
        lg.append(m.logits())
    info = (m.layer_form(), m.attn_splits(), m.attn_waves())
    m.close()
    return np.stack(ids), np.stack(lg), info


def _oracle_check(hip, params, lo, hi, total, ids, logits):
    """the oracle decoding rows lo..hi from the same K/V and tokens"""
    m = _c4_engine(hip, params, lo, hi)
    B = hi - lo
    c = oc.cfg(GPT2_124M["maxT"], GPT2_124M["V"], GPT2_124M["L"], GPT2_124M["NH"], GPT2_124M["C"])
    orc = oc.PagedDecoder(params, c, B, 16, GPT2_124M["maxT"], page_seed=9)
    for l in range(GPT2_124M["L"]):
        for b in range(B):
            k, v = m.read_kv(l, b, C4_CTX)
            orc.set_kv(l, b, k, v)
    m.close()
    toks = _c4_tokens(total)
    chk = IdCheck()
    for t in range(C4_STEPS):
        o_next, o_logits = orc.step(toks[t, lo:hi])
        chk.add(logits[t], o_logits, ids[t], o_next)
    orc.close()
    chk.verify(LOGIT_TOL)


@pytest.fixture(scope="module")
def c4_params(hip):
    return hip.synthetic_params(GPT2_124M, seed=C4_SEED)


@pytest.fixture(scope="module")
def c4_unsharded64(hip, c4_params):
    return _single(hip, c4_params, 0, 64, 64)


def _cat(got, key):
    return np.concatenate([g[key] for g in got], axis=1)


@pytest.mark.parametrize("picks", ["global", "local"])
@pytest.mark.parametrize("nranks", [2, 8])
def test_config4_strong_shards_default_path(hip, tmp_path, c4_params, c4_unsharded64, nranks, picks):
    """B = 64 over 2 (32 + 32) or 8 (8 x 8) ranks"""
    per = 64 // nranks
    shards = [(r * per, (r + 1) * per) for r in range(nranks)]
    got = _run_ranks(tmp_path, shards, 64, picks)
    want_ids, want_lg, want_info = c4_unsharded64
    ids, lg = _cat(got, "ids"), _cat(got, "logits")
    print(f"{nranks} ranks, picks {picks}: rank forms / splits / waves {[tuple(g['info']) for g in got]}, "
          f"unsharded {want_info}")
    if picks == "global":
        assert all(tuple(g["info"]) == tuple(want_info) for g in got)
        assert np.array_equal(ids, want_ids) and np.array_equal(lg, want_lg)
        return
    # local: each rank is the single-GPU engine of its rows ...
    lo, hi = shards[-1]
    s_ids, s_lg, s_info = _single(hip, c4_params, lo, hi, 64)
    assert tuple(got[-1]["info"]) == tuple(s_info)
    assert np.array_equal(got[-1]["ids"], s_ids) and np.array_equal(got[-1]["logits"], s_lg)
    # ... within the layer forms' reassociation of the unsharded engine, and the oracle's
    diff = float(np.abs(lg - want_lg).max())
    print(f"max |sharded - unsharded| logits {diff:.2e}")
    assert diff <= FORM_TOL
    _oracle_check(hip, c4_params, lo, hi, 64, got[-1]["ids"], got[-1]["logits"])


def test_config4_weak_64_per_rank_default_path(hip, tmp_path, c4_params):
    """config 4's per-rank batch: 64 + 64 (global 128 > 64: both pick modes
    are the rank's own); each rank equals the single-GPU B = 64 engine of its
    rows bit for bit, the unsharded B = 128 engine within the layer forms'
    reassociation (that engine has no persistent form above 64), the oracle"""
    shards = [(0, 64), (64, 128)]
    got = _run_ranks(tmp_path, shards, 128, "global")
    for g, (lo, hi) in zip(got, shards):
        s_ids, s_lg, s_info = _single(hip, c4_params, lo, hi, 128)
        assert tuple(g["info"]) == tuple(s_info)
        assert np.array_equal(g["ids"], s_ids) and np.array_equal(g["logits"], s_lg)
    w_ids, w_lg, w_info = _single(hip, c4_params, 0, 128, 128)
    diff = float(np.abs(_cat(got, "logits") - w_lg).max())
    print(f"rank forms {[tuple(g['info']) for g in got]}, unsharded B=128 {w_info}; max |diff| {diff:.2e}")
    assert diff <= FORM_TOL
    _oracle_check(hip, c4_params, 64, 128, 128, got[1]["ids"], got[1]["logits"])
