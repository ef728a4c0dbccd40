#!/usr/bin/env python3
"""Per-kernel HBM bytes per launch from the two PMC passes of
tools/pmc_traffic.sh.  Corrections (MI355X_MICROARCH.md, HBM [CDNA4]):
FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reports half the
bytes of a 16-B-per-lane streaming read -> x2; WRITE_SIZE is exact for
16-B-per-lane stores.  Writes <outdir>/traffic.json keyed by kernel name."""
import collections
import csv
import glob
import json
import os
import re
import sys

out = sys.argv[1]


def short(name):
    """kernel identifier with its template arguments, e.g.
    paged_attn_decode_f32<16, 4, true>"""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void\s+", "", n)
    depth, cut = 0, len(n)
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return n[:cut]


def load(ctr):
    files = glob.glob(os.path.join(out, ctr, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
            agg[key].append(float(r["Counter_Value"]))
    return agg


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
res = {}
for key in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
    f, w = fetch.get(key, []), write.get(key, [])
    fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
    wb = 1024.0 * sum(w) / len(w) if w else None
    name = f"{key[0]} grid={key[1]} wg={key[2]}"
    res[name] = {"launches": len(f), "fetch_bytes": fb, "write_bytes": wb,
                 "hbm_bytes": (fb or 0.0) + (wb or 0.0)}
    print(f"{name:60s} n={len(f):5d} fetch {fb / 1e6 if fb else 0:10.2f} MB  write {wb / 1e6 if wb else 0:9.2f} MB")
cfg = None
try:  # the bench line printed by the profiled run names the workload
    for line in open(os.path.join(out, "FETCH_SIZE.log")):
        if line.startswith("{"):
            j = json.loads(line)
            c = j["config"]
            cfg = {k: c.get(k) for k in ("workload", "batch_per_gpu", "seq_len", "page_size", "gemm_path")}
            cfg["dtype"] = j.get("dtype", "fp32")
except (OSError, ValueError, KeyError):
    pass
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, --kernel-trace, eager "
                     "launches; FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes",
           "config": cfg, "kernels": res},
          open(os.path.join(out, "traffic.json"), "w"), indent=1)
