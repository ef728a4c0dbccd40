#!/usr/bin/env python3
"""Decode throughput benchmark of the MI355X paged-attention decode path.

Metric (BASELINE.json): decode tokens/sec, GPT-2 124M paged attention,
B=64, ctx 1024, page 16, fp32, on 1/2/4/8 MI355X (configs[1] at N=1).  For
N>1 the decode shards by sequence (SURVEY.md 8e, configs[3]): every rank
decodes its own 64 sequences out of its own page pool with replicated
weights -> weak scaling; the one collective is the end-of-step RCCL gather
of the logits to rank 0 (--gather ids: greedy ids only), double-buffered on
its own stream so that step k's gather overlaps step k+1.  --scaling strong
splits a fixed global batch instead.

One "step" = one decode step of the whole batch: every sequence gets one new
token at its absolute position, all 12 layers (LN, QKV + KV append into the
HBM page pool, paged attention over 0..pos through the block table,
projections, MLP, residuals), final LN, logits (B x 50257), greedy argmax.
The KV cache is prefilled to ctx - (warmup + steps) positions with synthetic
K/V (default; --prefill real runs the one-pass prefill -- B*T-row GEMMs and
the causal multi-query attention on MFMA -- and reports its throughput too;
--prefill decode runs token-by-token decode steps instead); the timed
steps then decode at positions up to ctx - 1.  Weights are seeded synthetic
GPT-2 124M (no checkpoints offline).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "llm.c-paged_amd"))

import numpy as np  # noqa: E402

METRIC = "decode tokens/sec GPT-2 124M paged-attn, B=64 T=1024, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def pmc_traffic(kernel_prefix, batch_per_gpu, ctx, page_size, dtype):
    """HBM bytes per launch of the dominant kernel from a committed PMC
    summary (tools/pmc_traffic.sh -> profiles/r1/pmc_traffic*.json) taken on
    this workload; (None, None) when there is none"""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r1", "pmc_traffic*.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        c = d.get("config") or {}
        if (c.get("batch_per_gpu"), c.get("seq_len"), c.get("page_size"), c.get("dtype", "fp32")) != \
                (batch_per_gpu, ctx, page_size, dtype):
            continue
        for name, k in d["kernels"].items():
            if name.startswith(kernel_prefix):
                return k["hbm_bytes"], f"profiles/r1/{os.path.basename(path)}: {name}, {k['launches']} launches"
    return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64,
                    help="sequences per GPU (weak scaling) or in total (--scaling strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
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
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--attn-waves", type=int, default=4)
    ap.add_argument("--unfused", action="store_true", help="row-major GEMMs + separate row kernels")
    ap.add_argument("--lanes", type=int, default=1, help="micro-batch lanes (concurrent row groups)")
    ap.add_argument("--pipeline", type=int, default=0, help="1: two lanes, attention chunks beside GEMMs")
    ap.add_argument("--overlap", type=int, default=0,
                    help="overlapped step: chain workgroups beside the attention (0 = off)")
    ap.add_argument("--split", type=int, default=0,
                    help="split step: GEMM chains on this many CUs beside the attention (0 = off)")
    ap.add_argument("--sample", action="store_true",
                    help="multinomial sampling as the reference driver (default: greedy argmax)")
    ap.add_argument("--gemm-waves", default="", help="fused GEMM waves qkv,attproj,fc,fcproj,logits (0 = auto)")
    ap.add_argument("--gemm-rows", default="", help="fused GEMM 16-row blocks per workgroup, same order")
    ap.add_argument("--gemm-cols", default="", help="fused GEMM 16-column tiles per workgroup, same order")
    return ap.parse_args()


def cpu_baseline(cfgd, B, P, ctx, budget_s, kv_bf16=False, w_bf16=False):
    """The oracle's OpenMP C restatement of the same paged decode, timed on the
    host cores on a bounded sample (rank 0, N=1).  Test infrastructure only."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_ctypes as oc
    import pagedattn
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    os.environ["OMP_NUM_THREADS"] = str(threads)
    params = pagedattn.synthetic_params(cfgd, seed=1337)
    c = oc.cfg(cfgd["maxT"], cfgd["V"], cfgd["L"], cfgd["NH"], cfgd["C"])
    dec = oc.PagedDecoder(params, c, B, P, cfgd["maxT"], page_seed=3, fast=True, kv_bf16=kv_bf16, w_bf16=w_bf16)
    max_steps = min(256, ctx // 2)  # the budget normally ends the sample first (near ctx)
    start_ctx = ctx - max_steps
    dec.fill_random(start_ctx, seed=5)
    rng = np.random.default_rng(0)
    tok = rng.integers(0, cfgd["V"], B).astype(np.int32)
    steps, t0 = 0, time.perf_counter()
    while True:
        tok, _ = dec.step(tok, want_logits=False)
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s or steps >= max_steps:
            break
    dec.close()
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": B * steps / el, "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"oracle/liboracle_fast.so (-O3 -Ofast OpenMP C restatement), GPT-2 124M fp32"
                      f"{' (bf16 KV)' if kv_bf16 else ''}{' (bf16-rounded weights and GEMM inputs)' if w_bf16 else ''}, B={B}, page {P}, {steps} decode steps at ctx "
                      f"{start_ctx}..{start_ctx + steps} after a synthetic K/V fill, {el:.1f} s; cpu: {cpu_model}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        args.gpus = world
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import pagedattn
    import shard
    L = pagedattn.lib()
    pagedattn.init(local_rank)
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
        # one non-default stream shared by the library and torch: the decode
        # kernels, the id copy and the RCCL gather are ordered on it, and it
        # can be captured into a hipGraph (the legacy null stream cannot)
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        L.hpa_set_stream(stream.cuda_stream)
    pagedattn.check(L.hpa_set_attention_waves(args.attn_waves), "attention waves")

    cfgd = dict(pagedattn.GPT2_124M if args.model == "124M" else pagedattn.GPT2_XL)
    if args.ctx > cfgd["maxT"]:  # config 5: ctx 2048 -> 2048 rows of (synthetic) wpe, SURVEY.md 8d
        cfgd["maxT"] = args.ctx
    kv_bf16 = args.kv_dtype == "bf16"
    w_bf16 = args.w_dtype == "bf16"
    B, lo, hi = shard.batch_layout(args.batch, world, rank, args.scaling)
    B_local = hi - lo
    counts = [shard.batch_layout(args.batch, world, r, args.scaling) for r in range(world)]
    counts = [h - l for _, l, h in counts]
    P = args.page_size
    ctx = min(args.ctx, cfgd["maxT"])
    need = args.warmup + args.steps + 1
    window = min(need, ctx // 2)
    start = ctx - window  # positions of the first decoded token

    model = pagedattn.Model(cfgd, seed=1337)
    model.decode_init(B_local, P, ctx, kv_dtype=pagedattn.HPA_BF16 if kv_bf16 else pagedattn.HPA_F32,
                      w_dtype=pagedattn.HPA_BF16 if w_bf16 else pagedattn.HPA_F32)
    model.set_fused(not args.unfused)
    if not args.unfused:
        model.set_lanes(args.lanes)
        if args.pipeline:
            model.set_pipeline(True)
    if args.sample:
        model.set_sampling(True, seed=1337 + rank * B_local)
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
        for p in range(start):
            model.step(rng.integers(0, cfgd["V"], B_local).astype(np.int32), want_next=False)
    if args.split and not args.unfused:
        model.set_split(args.split)
    if args.overlap and not args.unfused:
        model.set_overlap(args.overlap)
    model.set_graph(not args.no_graph)
    first = rng.integers(0, cfgd["V"], B_local).astype(np.int32)
    pos_now = [start]

    gather = None
    nstep = [0]
    if world > 1 and args.gather != "none":
        # double-buffered: step k's output is copied on the compute stream,
        # then gathered on a comm stream while step k+1 computes
        gather = shard.StepGather(dist, world, rank, counts, cfgd["V"], args.gather, "cuda", nbuf=2)
        comm = torch.cuda.Stream()
        src, nbytes = ((model.logits_ptr(), B_local * cfgd["V"] * 4) if args.gather == "logits"
                       else (model.next_ptr(), B_local * 4))

    def one_step(tokens=None):
        if pos_now[0] >= ctx:  # slide back: pages kept, positions rewritten
            model.set_positions(np.full(B_local, start, np.int32))
            pos_now[0] = start
        model.step_async(tokens)
        pos_now[0] += 1
        if gather is not None:
            i = nstep[0] % 2
            gather.wait(i)  # the compute stream waits for the gather that last used buffer i
            L.hpa_memcpy_async(gather.buffer(i).data_ptr(), src, nbytes)  # compute stream
            comm.wait_stream(stream)
            with torch.cuda.stream(comm):  # RCCL gather to rank 0, overlapped with the next step
                gather.gather(i, async_op=True)
        nstep[0] += 1

    def sync():
        pagedattn.check(L.hpa_synchronize(), "sync")
        torch.cuda.synchronize()

    one_step(first)
    for _ in range(args.warmup - 1 if args.warmup > 0 else 0):
        one_step(None)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    bytes_before, _ = model.step_bytes()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step(None)
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    bytes_after, attn_after = model.step_bytes()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)
    tokens_per_s = B * args.steps / elapsed  # whole job: every rank's sequences

    # ---- live attention-kernel timing: HIP events on the launch stream around
    # back-to-back launches of the step's attention kernel over the layers, on
    # the engine's own pool at the last step's positions
    attn = None
    if args.prof_steps > 0:
        iters = args.prof_steps * cfgd["L"]
        avg_ms, per_launch_bytes = model.time_attention(iters)
        attn = dict(avg_ms=avg_ms, launches=iters, per_launch_bytes=per_launch_bytes,
                    achieved=per_launch_bytes / (avg_ms * 1e-3) / 1e9)

    result = None
    if rank == 0:
        cpu = None
        want_cpu = args.cpu_baseline == "on" or (args.cpu_baseline == "auto" and world == 1)
        if want_cpu and args.model == "124M":
            try:
                # bounded sample: the oracle keeps an fp32 pool of B*ctx*C*L*2 floats, so
                # beyond config 2's B*ctx the sample takes a subset of the sequences
                cpu_B = B_local if B_local * ctx <= 65536 else max(1, 16384 // ctx)
                cpu = cpu_baseline(cfgd, cpu_B, P, ctx, args.cpu_seconds, kv_bf16, w_bf16)
                if cpu_B != B_local:
                    cpu["sample"] += f" (a {cpu_B}-sequence subset of the {B_local}-sequence batch)"
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        name, cus, mem = pagedattn.device_info()
        roof = None
        if attn:
            traffic, tsrc = pmc_traffic("paged_attn_decode_f32", B_local, ctx, P,
                                        "fp32 (bf16 KV storage)" if kv_bf16 else "fp32")
            roof = {"bound": "hbm", "kernel": "paged_attn_decode_f32" + ("<bf16 KV>" if kv_bf16 else ""),
                    "achieved": round(attn["achieved"], 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(attn["achieved"] / HBM_PEAK_GBS, 4),
                    "traffic": None if traffic is None else int(traffic),
                    "traffic_source": tsrc, "avg_launch_ms": round(attn["avg_ms"], 5),
                    "bytes_per_launch": int(attn["per_launch_bytes"]), "launches_timed": attn["launches"]}
        step_bytes = 0.5 * (bytes_before + bytes_after)
        result = {
            "metric": METRIC,
            "value": round(tokens_per_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": ("bf16 weights and GEMM inputs, fp32 accumulate" if w_bf16 else "fp32")
                     + (" (bf16 KV storage)" if kv_bf16 else ""),
            "data": "synthetic (seeded random GPT-2 124M weights and tokens; KV prefill: "
                    + {"synthetic": "synthetic U(-1,1)", "real": "one-pass prefill of random tokens",
                       "decode": "decode steps"}[args.prefill] + ")",
            "config": {"workload": f"GPT-2 {args.model} {'bf16' if w_bf16 else 'fp32'} paged decode, batch={B_local} per GPU x {world} "
                                   f"(B={B}), ctx {ctx}, page_size={P}{', bf16 KV' if kv_bf16 else ''}"
                                   f"{', bf16 weights' if w_bf16 else ''} (BASELINE.json "
                                   + ("configs[4])" if kv_bf16 else "configs[2])" if args.model == "XL" else
                                      "configs[1])" if world == 1 else "configs[3]: per-seq sharded pool)"),
                       "global_batch": B, "batch_per_gpu": B_local, "seq_len": ctx, "page_size": P,
                       "decode_positions": f"{start}..{start + args.warmup + args.steps - 1}",
                       "parallelism": f"seq-shard x{world}" + (f" + RCCL gather({args.gather}) to rank 0, overlapped with the next step"
                                                               if world > 1 and args.gather != "none" else ""),
                       "hip_graph": not args.no_graph, "gemm_path": "unfused" if args.unfused else "fused",
                       "lanes": 1 if args.unfused else L.gpt2_decode_lanes(model.h),
                       "pipeline": bool(L.gpt2_decode_pipeline(model.h)),
                       "split_gemm_cus": 0 if args.unfused else L.gpt2_decode_split(model.h),
                       "overlap_chain_blocks": 0 if args.unfused else L.gpt2_decode_overlap(model.h),
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
        if prefill_stats:
            result["prefill"] = prefill_stats
        print(json.dumps(result), flush=True)
    model.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
