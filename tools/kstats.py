#!/usr/bin/env python3
"""Per (kernel, grid) average durations from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 0
r = list(csv.DictReader(open(path)))
agg = collections.defaultdict(list)
for x in r:
    key = (x["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:], x["Grid_Size_X"], x["Grid_Size_Y"], x["Grid_Size_Z"],
           x["Workgroup_Size_X"], x.get("VGPR_Count", ""), x.get("Accum_VGPR_Count", ""))
    agg[key].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
tot = 0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    s = sum(v) / 1000
    tot += s
    per = f"{s / steps:8.1f} us/step" if steps else ""
    print(f"{k[0]:40s} g=({k[1]},{k[2]},{k[3]}) wg={k[4]} vgpr={k[5]}/{k[6]} n={len(v):5d} "
          f"avg={s / len(v):8.2f} us {per}")
print(f"total {tot:.1f} us")
