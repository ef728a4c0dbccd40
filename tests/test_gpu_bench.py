"""bench.py's contract on the GPU: one JSON line with the metric of
BASELINE.json, a positive whole-job value, the attention-kernel roofline and
the config fields the driver reads (a short run: 3 timed steps)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--cpu-baseline", "off", *args], capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_default_line():
    d = _bench()
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert abs(d["value"] - 64 * 1000.0 / d["ms_per_step"]) / d["value"] < 1e-3  # B=64 tokens per step
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1
    assert abs(r["achieved"] / r["peak"] - r["frac"]) < 1e-3
    c = d["config"]
    assert c["global_batch"] == 64 and c["seq_len"] == 1024 and c["page_size"] == 16 and c["hip_graph"]


def test_bench_small_batch_split_attention_line():
    """B=8 (the per-GPU batch of strong scaling at N=8): the split-context
    attention is in use and the line is well formed"""
    d = _bench("--batch", "8")
    assert d["config"]["global_batch"] == 8 and d["config"]["attn_splits"] >= 2
    assert d["value"] > 0 and 0 < d["roofline"]["frac"] < 1


@pytest.mark.parametrize("n", [2, 8])
def test_bench_default_multi_gpu_line_is_the_metric(n):
    """the default N>1 line (rehearsed on one GPU with --emulate-rank N) is the
    headline metric: B = 64 split over the N ranks (BASELINE.md section 3's
    2/4/8-GPU rows), so value, global_batch and the metric string agree"""
    d = _bench("--emulate-rank", str(n))
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    c, e = d["config"], d["emulated_rank"]
    assert d["metric"] == base["metric"] and d["scaling"] == "strong"
    assert c["global_batch"] == 64 and c["batch_per_gpu"] == 64 // n and "configs[1]" in c["workload"]
    assert e["rows"] == 64 // n and e["global_batch"] == 64
    # value = this GPU's rows; the projection = all N ranks' rows at this step time
    assert abs(d["value"] - (64 // n) * 1000.0 / d["ms_per_step"]) / d["value"] < 1e-3
    assert abs(e["projected_n_gpu_tokens_per_s"] * d["ms_per_step"] / 64000.0 - 1) < 1e-2
    assert "1-rank RCCL communicator" in e["gather"]  # rank 0's gather runs in the timed steps
    assert d["status"] == 0


def test_bench_weak_line_is_labelled_config4():
    """--scaling weak at N>1 (64 sequences per rank) is BASELINE configs[3],
    reported under its own metric string, never the headline's"""
    d = _bench("--emulate-rank", "2", "--scaling", "weak")
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] != base["metric"] and "per GPU" in d["metric"]
    assert d["config"]["global_batch"] == 128 and "configs[3]" in d["config"]["workload"]
