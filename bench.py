#!/usr/bin/env python3
"""Decode throughput benchmark of the MI355X paged-attention decode path.

Metric (BASELINE.json): decode tokens/sec, GPT-2 124M paged attention,
B=64, ctx 1024, page 16, fp32, on 1/2/4/8 MI355X (configs[1] at N=1).  For
N>1 the decode shards by sequence: the metric's B = 64 is split
over the N ranks (strong scaling, the default: BASELINE.md section 3's 2/4/8-GPU
rows, 32/16/8 sequences per rank), each rank decoding its own rows from its
own page pool with replicated weights.  --scaling weak gives every rank 64
sequences instead (BASELINE configs[3]: B = 512 at 8 GPUs) and prints that
config's own metric string, not the headline's.  --emulate-rank N times rank
0's engine of an N-GPU run on one GPU.  The one
collective is the end-of-step gather of the logits to rank 0 (--gather ids:
the greedy ids only), run by the C library over RCCL/xGMI
(gpt2_decode_gather: double-buffered on its own stream, so step k's gather
overlaps step k+1).  No torch in the measuring processes: the RCCL id goes
through a file, and the timing barriers and the max-over-ranks time run on
the library's own communicator (hpa_comm_barrier / hpa_comm_allreduce_max).

One "step" = one decode step of the whole batch: every sequence gets one new
token at its absolute position, all layers (QKV + KV append into the HBM page
pool, paged attention over 0..pos through the block table, projections, MLP,
residuals, LayerNorms), final LN, logits (B x 50257), greedy argmax.  The KV
cache is prefilled to ctx - (warmup + steps + 1) positions with synthetic K/V
(default; --prefill real runs the one-pass prefill -- B*T-row GEMMs and the
causal multi-query attention on MFMA -- and reports its throughput too;
--prefill decode runs token-by-token decode steps instead); the timed steps
then decode at positions up to ctx - 1.  Weights are seeded synthetic GPT-2
(no checkpoints offline).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))

import numpy as np  # noqa: E402

METRIC = "decode tokens/sec GPT-2 124M paged-attn, B=64 T=1024, 1/2/4/8 MI355X"
# --scaling weak at N > 1 is BASELINE configs[3] (64 sequences per GPU), not the headline metric
METRIC_WEAK = "decode tokens/sec GPT-2 124M paged-attn, B=64 per GPU (B=512 at 8 GPUs), T=1024, N MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def pmc_traffic(kernel_prefix, batch_per_gpu, ctx, page_size, dtype):
    """HBM bytes per launch of the dominant kernel from a committed PMC
    summary (tools/pmc_traffic.sh -> profiles/rNN/pmc_traffic*.json) taken on
    this workload, newest round first; (None, None) when there is none"""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_traffic*.json")), reverse=True)
    for path in paths:
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        c = d.get("config") or {}
        # the attention kernel's bytes depend on the KV storage type, not on the weights'
        if (c.get("batch_per_gpu"), c.get("seq_len"), c.get("page_size"), "bf16 KV" in c.get("dtype", "fp32")) != \
                (batch_per_gpu, ctx, page_size, "bf16 KV" in dtype):
            continue
        for name, k in d["kernels"].items():
            if name.startswith(kernel_prefix):
                rel = os.path.relpath(path, REPO)
                return k["hbm_bytes"], f"{rel}: {name}, {k['launches']} launches"
    return None, None


def comm_id_path():
    """the RCCL id's rendezvous file: one per launch (the launcher's pid is
    every worker's parent) and master port, on the node's local disk"""
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"hpa_rccl_id_{os.getppid()}_{port}")


def comm_init(L, pagedattn, world, rank):
    """N > 1: the library's own RCCL communicator (libpaged_hip.so, built
    against /opt/rocm's RCCL), no torch in this process.  Rank 0 writes the
    ncclUniqueId to a file, the others read it; the communicator then carries
    the end-of-step gather, the timing barriers and the max-over-ranks time.
    A rank whose communicator cannot be created exits non-zero and no value
    is reported (a scaling line without the north star's collective would
    leave work out of the timed region)."""
    n = L.hpa_comm_id_bytes()
    path = comm_id_path()
    uid = ctypes.create_string_buffer(n)
    if rank == 0:
        pagedattn.check(L.hpa_comm_unique_id(uid, n), "comm_unique_id")
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid.raw)
        os.replace(tmp, path)
    else:
        t0 = time.time()
        while not (os.path.exists(path) and os.path.getsize(path) == n):
            if time.time() - t0 > 120:
                print(f"[bench] rank {rank}: no RCCL id from rank 0 in 120 s ({path})", file=sys.stderr, flush=True)
                sys.exit(3)
            time.sleep(0.01)
        with open(path, "rb") as f:
            uid = ctypes.create_string_buffer(f.read(), n)
    maps = open("/proc/self/maps").read().split("\n")
    libs = sorted({ln.split()[-1] for ln in maps if ("librccl" in ln or "libamdhip64" in ln) and "/" in ln})
    print(f"[bench] rank {rank}/{world}: process loaded {', '.join(libs)}", file=sys.stderr, flush=True)
    if L.hpa_comm_init(world, rank, uid) != 0:
        print(f"[bench] rank {rank}: RCCL communicator init failed "
              f"({L.hpa_last_error().decode(errors='replace')}); no value reported", file=sys.stderr, flush=True)
        sys.exit(4)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--spinup", type=float, default=2.0,
                    help="seconds of untimed decode steps before the warm-up (positions reset to the start "
                         "afterwards, so the timed steps decode at the same positions): a fresh box's first "
                         "seconds of load run slower")
    ap.add_argument("--batch", type=int, default=64,
                    help="sequences in total, split over the ranks (--scaling strong, the default: the metric's "
                         "B=64), or per GPU (--scaling weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default, the metric's 2/4/8-GPU points): --batch in total, split over the "
                         "ranks; weak: --batch sequences per GPU (BASELINE configs[3] at N=8: 64 x 8 = 512), "
                         "reported under configs[3]'s own metric string")
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--page-size", type=int, default=16)
    ap.add_argument("--kv-dtype", default="f32", choices=["f32", "bf16"],
                    help="KV pool storage (bf16: BASELINE config 5; arithmetic stays fp32)")
    ap.add_argument("--w-dtype", default="f32", choices=["f32", "bf16"],
                    help="GEMM weight storage (bf16: weights and GEMM inputs bf16, fp32 accumulation on "
                         "bf16 MFMA -- the 'bf16 decode' of BASELINE config 5)")
    ap.add_argument("--model", default="124M", choices=["124M", "XL"])
    ap.add_argument("--prefill", default="synthetic", choices=["synthetic", "real", "decode"])
    ap.add_argument("--prefill-chunk", type=int, default=256, help="tokens per sequence per prefill call")
    ap.add_argument("--gather", default="logits", choices=["ids", "logits", "none"],
                    help="end-of-step gather to rank 0 (N>1)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=4,
                    help="attention roofline timing: prof_steps x L back-to-back launches (0 = off)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="per CPU run (-Ofast all cores, -Ofast at OMP_NUM_THREADS, strict all cores)")
    ap.add_argument("--attn-waves", type=int, default=0,
                    help="waves per attention workgroup for every launch (0 = the engine's pick by batch)")
    ap.add_argument("--attn-splits", type=int, default=0, help="attention context ranges (0 = by shape)")
    ap.add_argument("--layer-kernel", type=int, default=-1, choices=[-1, 0, 1, 2, 3, 4, 5, 6, 7],
                    help="gpt2_decode_set_layer_kernel: 0 five launches per layer; 1 auto (the form measured "
                         "fastest for the batch: chain form 6 at C = 768, form 8 at C >= 1024, the bf16 chain "
                         "on bf16 weights); 3 the attention launch + the chain (4-wave units); 5 chain form 6 "
                         "(12-wave multi-tile units); 6 chain form 8 (streamed weights, also GPT-2 XL); 2 the "
                         "full persistent layer and 4 the wide-unit chain: A/B builds (-DHPA_AB) only; 7 the "
                         "pipelined halves (one launch for every layer, attention and GEMM chain on disjoint CUs); "
                         "-1 the engine's default (HPA_LAYER_KERNEL or 1)")
    ap.add_argument("--pipe-g", type=int, default=0,
                    help="CUs of the pipelined halves' GEMM role (form 7; multiple of 8; 0 = the default 64)")
    ap.add_argument("--picks", default="local", choices=["local", "global"],
                    help="N>1 / --emulate-rank: shape picks by the rank's own batch (default: a rank computes "
                         "what a single-GPU engine of its rows computes) or by the global batch "
                         "(gpt2_decode_set_global_batch: rows bit-identical to the unsharded engine)")
    ap.add_argument("--emulate-rank", type=int, default=0,
                    help="N: on one GPU, time rank 0's engine of an N-GPU run (B/N rows for --scaling strong, "
                         "B for weak, with --picks), and report the per-rank step and the N-GPU projection; "
                         "rank 0's gather (--gather) runs every step on a 1-rank communicator")
    ap.add_argument("--sample", action="store_true",
                    help="multinomial sampling as the reference driver (default: greedy argmax)")
    ap.add_argument("--gemm-waves", default="", help="fused GEMM waves qkv,attproj,fc,fcproj,logits (0 = auto)")
    ap.add_argument("--gemm-rows", default="", help="fused GEMM 16-row blocks per workgroup, same order")
    ap.add_argument("--gemm-cols", default="", help="fused GEMM 16-column tiles per workgroup, same order")
    return ap.parse_args()


def cpu_baseline(cfgd, B, P, start_ctx, end_ctx, budget_s, kv_bf16=False, w_bf16=False):
    """The oracle's OpenMP C restatement of the same paged decode, timed at
    the GPU's positions on EVERY core this process may use (the
    affinity mask, not the job's OMP_NUM_THREADS share), with the OMP_NUM_THREADS
    figure beside it (the box sets 16, its CPU share): the -Ofast build at all
    cores (the value), the -Ofast build at OMP_NUM_THREADS, the strict build at
    all cores; each a bounded sample.  Rank 0, N=1.  Test infrastructure only
    (never the measured product)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_ctypes as oc
    import pagedattn
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    quota = cgroup_cpu_quota()
    params = pagedattn.synthetic_params(cfgd, seed=1337)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    # thread counts: every core of the affinity mask, and the
    # cores the job's CPU quota actually grants (cgroup cpu.max; on the GPU box
    # the mask shows the whole machine while the quota is the job's share)
    usable = min(affinity, quota) if quota else affinity
    counts = [affinity] + [n for n in (usable, share) if n and n != affinity]
    counts = list(dict.fromkeys(counts))
    plan = [(True, n, budget_s if n == usable else min(budget_s, 4.0)) for n in counts] + [(False, usable, budget_s)]
    runs = []
    for fast, threads, bud in plan:
        build = "-O3 -Ofast -march=x86-64-v3 (liboracle_fast.so)" if fast else \
            "-O2 -fno-fast-math -ffp-contract=off (liboracle.so)"
        used = oc.lib(fast).oracle_set_threads(threads)
        dec = oc.PagedDecoder(params, c, B, P, cfgd["maxT"], page_seed=3, fast=fast, kv_bf16=kv_bf16,
                              w_bf16=w_bf16)
        dec.fill_random(start_ctx, seed=5)
        tok = np.random.default_rng(0).integers(0, cfgd["V"], B).astype(np.int32)
        steps, t0 = 0, time.perf_counter()
        while start_ctx + steps < end_ctx:
            tok, _ = dec.step(tok, want_logits=False)
            steps += 1
            el = time.perf_counter() - t0
            if el >= bud:
                break
        dec.close()
        runs.append({"build": build, "threads": used, "value": round(B * steps / el, 2), "steps": steps,
                     "positions": f"{start_ctx}..{start_ctx + steps - 1}", "seconds": round(el, 2)})
    best = max((r for r in runs if "Ofast" in r["build"]), key=lambda r: r["value"])
    return {"value": best["value"], "unit": "tokens/s", "cores": best["threads"], "kind": "port",
            "nproc": os.cpu_count(), "affinity_cores": affinity, "cgroup_cpu_quota": quota,
            "sample": f"oracle/ C restatement of the same paged decode (OpenMP), GPT-2 "
                      f"{'XL' if cfgd['C'] == 1600 else '124M'}"
                      f"{' bf16-rounded weights and GEMM inputs' if w_bf16 else ' fp32'}"
                      f"{' (bf16 KV)' if kv_bf16 else ''}, B={B}, page {P}, decode steps at the GPU's positions "
                      f"after a synthetic K/V fill; timed on all {affinity} cores of the affinity mask and on the "
                      f"{usable} cores the job's CPU quota grants (cgroup cpu.max: {quota or 'unlimited'}), "
                      f"value = the faster -Ofast run ({best['threads']} threads); every run in 'builds'; "
                      f"cpu: {cpu_model}",
            "builds": runs}


def cgroup_cpu_quota():
    """CPUs the cgroup's cpu.max grants (quota / period, rounded up), or 0 when unlimited / unknown"""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return 0


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        args.gpus = world
    import pagedattn
    import shard
    L = pagedattn.lib()
    pagedattn.init(int(os.environ.get("HPA_DEVICE", local_rank)))  # HPA_DEVICE: rehearse N ranks on one GPU
    if world > 1:
        comm_init(L, pagedattn, world, rank)
    pagedattn.check(L.hpa_set_attention_waves(args.attn_waves), "attention waves")

    cfgd = dict(pagedattn.GPT2_124M if args.model == "124M" else pagedattn.GPT2_XL)
    if args.ctx > cfgd["maxT"]:  # config 5: ctx 2048 -> 2048 rows of (synthetic) wpe, SURVEY.md 8d
        cfgd["maxT"] = args.ctx
    kv_bf16 = args.kv_dtype == "bf16"
    w_bf16 = args.w_dtype == "bf16"
    emulate = args.emulate_rank if world == 1 and args.emulate_rank > 1 else 0
    layout_world = emulate or world  # --emulate-rank N: rank 0's share of an N-GPU run, on this one GPU
    B, lo, hi = shard.batch_layout(args.batch, layout_world, rank, args.scaling)
    B_local = hi - lo
    counts = [shard.batch_layout(args.batch, layout_world, r, args.scaling) for r in range(layout_world)]
    counts = [h - l for _, l, h in counts]
    P = args.page_size
    ctx = min(args.ctx, cfgd["maxT"])
    need = args.warmup + args.steps + 1
    window = min(need, ctx // 2)
    start = ctx - window  # position of the first decoded token

    model = pagedattn.Model(cfgd, seed=1337)
    model.decode_init(B_local, P, ctx, kv_dtype=pagedattn.HPA_BF16 if kv_bf16 else pagedattn.HPA_F32,
                      w_dtype=pagedattn.HPA_BF16 if w_bf16 else pagedattn.HPA_F32)
    if args.attn_splits:
        model.set_attn_splits(args.attn_splits)
    if args.picks == "global" and layout_world > 1:
        model.set_global_batch(B)  # every row as the unsharded engine of B computes it
    if args.layer_kernel >= 0:
        model.set_layer_kernel(args.layer_kernel)
    if args.pipe_g:
        model.set_pipe_split(args.pipe_g)
    if args.sample:
        model.set_sampling(True, seed=1337 + lo)
    if args.gemm_waves or args.gemm_rows or args.gemm_cols:
        ints = lambda a: [int(x) for x in a.split(",")] if a else None  # noqa: E731
        model.gemm_config(ints(args.gemm_waves), ints(args.gemm_rows), ints(args.gemm_cols))
    model.reserve(ctx)
    rng = np.random.default_rng(1000 + rank)
    prefill_stats = None
    if args.prefill == "synthetic":
        model.fill_random(start, seed=77 + rank)
    elif args.prefill == "real":
        toks = rng.integers(0, cfgd["V"], (B_local, start)).astype(np.int32)
        model.prefill(toks[:, :min(start, 16)])  # warm-up (kernels, workspace)
        model.set_positions(np.zeros(B_local, np.int32))
        pagedattn.check(L.hpa_synchronize(), "sync")
        t0 = time.perf_counter()
        for c0 in range(0, start, args.prefill_chunk):
            model.prefill(toks[:, c0:c0 + args.prefill_chunk])
        pagedattn.check(L.hpa_synchronize(), "sync")
        el = time.perf_counter() - t0
        prefill_stats = {"tokens": B_local * start, "seconds": round(el, 4),
                         "tokens_per_s": round(B_local * start / el, 1), "chunk": args.prefill_chunk,
                         "note": "one-pass prefill of positions 0..start-1, rank 0, not part of value"}
    else:
        for _ in range(start):
            model.step(rng.integers(0, cfgd["V"], B_local).astype(np.int32), want_next=False)
    model.set_graph(not args.no_graph)
    gather = world > 1 and not args.gather.startswith("none")
    if gather:
        model.shard(counts, root=0)
    # --emulate-rank: rank 0's gather runs too, on a 1-rank communicator (its
    # local cost -- the compute -> comm hand-off, the send copy, RCCL's kernel
    # on the comm stream beside the next step: profiles/r6/recv_coresidency.txt)
    emul_gather = bool(emulate) and not args.gather.startswith("none")
    if emul_gather:
        n = L.hpa_comm_id_bytes()
        uid = ctypes.create_string_buffer(n)
        pagedattn.check(L.hpa_comm_unique_id(uid, n), "comm_unique_id")
        pagedattn.check(L.hpa_comm_init(1, 0, uid), "comm_init (1 rank)")
        model.shard([B_local], root=0)
        gather = True
    what = 0 if args.gather == "logits" else 1
    first = rng.integers(0, cfgd["V"], B_local).astype(np.int32)
    pos_now = [start]

    def one_step(tokens=None):
        if pos_now[0] >= ctx:  # slide back: pages kept, positions rewritten
            model.set_positions(np.full(B_local, start, np.int32))
            pos_now[0] = start
        model.step_async(tokens)
        pos_now[0] += 1
        if gather:
            model.gather(what)  # RCCL gather to rank 0 on the comm stream, overlapped with the next step

    def sync():  # every stream of the device: the decode stream and the comm stream
        pagedattn.check(L.hpa_device_synchronize(), "device sync")

    def status_gate(where):
        """a timed-out in-launch wait of the persistent layer invalidates the
        steps (their outputs are garbage and they end early): no value then"""
        try:
            model.status()
        except RuntimeError as e:
            print(f"[bench] rank {rank}: {e} after the {where}; no value reported", file=sys.stderr, flush=True)
            sys.exit(5)

    # under rocprofv3 the spin-up launches its steps eagerly: the profiler's
    # hipGraphLaunch path faults after a few hundred to a few thousand graph
    # replays (SIGSEGV inside the tool library, reproduced with no part of this
    # library loaded by tools/micro/graph_replay.hip), and
    # the 2 s spin-up replays ~1,800 step graphs.  Eager steps keep the GPU as
    # busy (the step is ~40 launches of ~1 ms of kernels); the warm-up and
    # timed steps stay graph replays.
    profiled = any(k.startswith("ROCPROF") for k in os.environ)
    spin_eager = args.spinup > 0 and profiled and not args.no_graph
    if spin_eager:
        model.set_graph(False)
    if args.spinup > 0:  # untimed, before the warm-up; the positions go back to `start` after it
        # local steps only (no gather: ranks may run different counts in the
        # same time, and a collective must be called by every rank alike)
        model.step_async(first)
        sync()
        t_spin, p = time.perf_counter() + args.spinup, start + 1
        while time.perf_counter() < t_spin:
            for _ in range(16):
                if p >= ctx:
                    model.set_positions(np.full(B_local, start, np.int32))
                    p = start
                model.step_async(None)
                p += 1
            sync()
        model.set_positions(np.full(B_local, start, np.int32))
        sync()
    if spin_eager:
        model.set_graph(True)
    one_step(first)
    for _ in range(args.warmup - 1 if args.warmup > 0 else 0):
        one_step(None)
    sync()
    status_gate("warm-up steps")
    if world > 1:
        pagedattn.check(L.hpa_comm_barrier(), "comm barrier")  # RCCL all-reduce + wait
    sync()
    bytes_before, _ = model.step_bytes()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(None)
    sync()
    if world > 1:
        pagedattn.check(L.hpa_comm_barrier(), "comm barrier")
    t1 = time.perf_counter()
    bytes_after, _ = model.step_bytes()
    status_gate("timed steps")
    elapsed = t1 - t0
    if world > 1:  # max over ranks, through the library's RCCL communicator
        el = ctypes.c_double(elapsed)
        pagedattn.check(L.hpa_comm_allreduce_max(ctypes.byref(el)), "comm max")
        elapsed = el.value
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    # whole job: every rank's sequences (--emulate-rank: this one GPU's rows)
    tokens_per_s = (B_local if emulate else B) * args.steps / elapsed

    # ---- live attention-kernel timing: HIP events on the launch stream around
    # back-to-back launches of the step's attention kernel over the layers, on
    # the engine's own pool at the last step's positions
    attn = None
    if args.prof_steps > 0:
        iters = args.prof_steps * cfgd["L"]
        avg_ms, per_launch_bytes = model.time_attention(iters)
        attn = dict(avg_ms=avg_ms, launches=iters, per_launch_bytes=per_launch_bytes,
                    achieved=per_launch_bytes / (avg_ms * 1e-3) / 1e9)

    if rank == 0:
        cpu = None
        want_cpu = args.cpu_baseline == "on" or (args.cpu_baseline == "auto" and world == 1)
        if want_cpu:
            try:
                # bounded sample: the oracle keeps an fp32 pool of B*ctx*C*L*2 floats, so
                # beyond config 2's B*ctx the sample takes a subset of the sequences
                # (GPT-2 XL: one sequence -- 0.6 GB of pool, 6 GB of weights on the host)
                cpu_B = B_local if B_local * ctx <= 65536 else max(1, 16384 // ctx)
                if args.model == "XL":
                    cpu_B = 1
                cpu = cpu_baseline(cfgd, cpu_B, P, start, ctx, args.cpu_seconds, kv_bf16, w_bf16)
                if cpu_B != B_local:
                    cpu["sample"] += f" (a {cpu_B}-sequence subset of the {B_local}-sequence batch)"
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        name, cus, mem = pagedattn.device_info()
        splits = model.attn_splits()
        roof = None
        if attn:
            kname = "paged_attn_decode_f32"
            traffic, tsrc = pmc_traffic(kname, B_local, ctx, P, "fp32 (bf16 KV storage)" if kv_bf16 else "fp32")
            roof = {"bound": "hbm", "kernel": kname + ("<bf16 KV>" if kv_bf16 else "")
                    + (f" ({splits} context ranges per sequence-head)" if splits > 1 else ""),
                    "achieved": round(attn["achieved"], 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(attn["achieved"] / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else int(traffic),
                    "traffic_source": tsrc, "avg_launch_ms": round(attn["avg_ms"], 5),
                    "bytes_per_launch": int(attn["per_launch_bytes"]), "launches_timed": attn["launches"]}
        step_bytes = 0.5 * (bytes_before + bytes_after)
        weak_n = layout_world > 1 and args.scaling == "weak"
        which = ("configs[4]" if kv_bf16 else "configs[2]" if args.model == "XL" else
                 "configs[3]: per-seq sharded pool" if weak_n else "configs[1]")
        result = {
            "metric": METRIC_WEAK if weak_n else METRIC,
            "value": round(tokens_per_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "spinup_s": args.spinup,
            "spinup_eager": spin_eager,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": ("bf16 weights and GEMM inputs, fp32 accumulate" if w_bf16 else "fp32")
                     + (" (bf16 KV storage)" if kv_bf16 else ""),
            "data": f"synthetic (seeded random GPT-2 {args.model} weights and tokens; KV prefill: "
                    + {"synthetic": "synthetic U(-1,1)", "real": "one-pass prefill of random tokens",
                       "decode": "decode steps"}[args.prefill] + ")",
            "config": {"workload": f"GPT-2 {args.model} {'bf16' if w_bf16 else 'fp32'} paged decode, B={B} "
                                   f"({B_local} on rank 0 of {world}, {args.scaling} scaling), ctx {ctx}, "
                                   f"page_size={P}{', bf16 KV' if kv_bf16 else ''}{', bf16 weights' if w_bf16 else ''}"
                                   f" (BASELINE.json {which})",
                       "global_batch": B, "batch_per_gpu": B_local, "seq_len": ctx, "page_size": P,
                       "decode_positions": f"{start}..{start + args.warmup + args.steps - 1}",
                       "parallelism": f"seq-shard x{world}" + (f" + RCCL gather({args.gather}) to rank 0 in the C "
                                                               "library, overlapped with the next step"
                                                               if gather else
                                                               f" (gather: {args.gather})" if world > 1 else ""),
                       "hip_graph": not args.no_graph, "attn_splits": splits,
                       "attn_waves": args.attn_waves or int(L.gpt2_decode_attn_waves(model.h)),
                       "layer_loop": {0: "five launches per layer",
                                      1: "one persistent launch per layer (hpa_decode_layer)",
                                      2: "attention launch + one persistent launch of the GEMM chain "
                                         "(hpa_decode_layer chain_only)",
                                      3: "attention launch + one persistent launch of the GEMM chain in "
                                         "wide / multi-tile units (hpa_decode_layer chain_only 2..6, 8: "
                                         "by default form 6 at C = 768, form 8 at C >= 1024)",
                                      4: "attention launch + one persistent launch of the bf16-weight GEMM "
                                         "chain (hpa_decode_chain_b16)",
                                      5: "one persistent launch of every layer: the batch in two halves, "
                                         "attention of one beside the GEMM chain of the other on disjoint CUs "
                                         "(hpa_decode_pipe)"}[model.layer_form()],
                       "attn_form": f"(sequence, head) x {splits} range(s)",
                       "token_choice": "multinomial (reference sample_mult)" if args.sample else "greedy",
                       "gemm_waves": [int(x) for x in model.gemm_config()[0]],
                       "gemm_row_blocks": [int(x) for x in model.gemm_config()[1]],
                       "gemm_col_tiles": [int(x) for x in model.gemm_config()[2]], "device": name},
            "step_roofline": {"bytes_per_step_rank0": int(step_bytes),
                              "achieved_GBps": round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                              "frac_of_8TBps": round(step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        result["config"]["picks"] = (f"global (gpt2_decode_set_global_batch({B}))" if args.picks == "global"
                                     and layout_world > 1 else "local (the rank's own batch)")
        # every HPA_* knob in this process's environment (none in the default run)
        result["config"]["env_knobs"] = {k: v for k, v in sorted(os.environ.items()) if k.startswith("HPA_")}
        result["status"] = 0  # gpt2_decode_status after the warm-up and after the timed steps
        if emulate:
            result["emulated_rank"] = {
                "n_gpus": emulate, "rank": 0, "rows": B_local, "global_batch": B, "scaling": args.scaling,
                "ms_per_step": round(ms_per_step, 4),
                "projected_n_gpu_tokens_per_s": round(sum(counts) * args.steps / elapsed, 1),
                "gather": (f"the library's {args.gather} gather every step on a 1-rank RCCL communicator (its "
                           f"local cost; the peers' transfer is not modelled)" if emul_gather else "none"),
                "note": "one GPU running rank 0's engine of an N-GPU decode; value = this GPU's tokens/s; "
                        "the projection assumes every rank steps as fast and the peers' share of the gather "
                        "stays hidden behind the next step (it overlaps on its own stream); not a multi-GPU "
                        "measurement"}
            result["n_gpus"] = 1
        if prefill_stats:
            result["prefill"] = prefill_stats
        print(json.dumps(result), flush=True)
    model.close()
    if emul_gather:
        L.hpa_comm_destroy()
    if world > 1:
        pagedattn.check(L.hpa_comm_barrier(), "comm barrier")
        L.hpa_comm_destroy()
        if rank == 0:
            try:
                os.unlink(comm_id_path())
            except OSError:
                pass


if __name__ == "__main__":
    main()
