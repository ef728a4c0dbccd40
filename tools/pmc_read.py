#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection.csv files: per kernel (name prefix),
average counter value per dispatch, plus kernel-trace durations."""
import collections
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"][:50]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        if "pack" in k or "rocclr" in k or "elementwise" in k:
            continue
        vals = "  ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items()))
        print(f"{os.path.basename(d):8s} {k[:28]:28s} n={len(next(iter(cs.values())))} {vals}")
