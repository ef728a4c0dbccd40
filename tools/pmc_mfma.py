#!/usr/bin/env python3
"""Per-kernel MFMA utilisation from tools/pmc_mfma.sh's pass.

For each (kernel, grid): launches, average duration (kernel trace), MFMA
instructions per launch, matrix-pipe busy cycles per launch, the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), and
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (duration x clock x 1024 SIMDs)
the fraction of the chip's matrix-pipe cycles the kernel kept busy at the
clock it ran (the guide: the GRBM quotient reads high below ~0.3 ms), and
  mfma_busy_nominal = the same against 2.4 GHz, the clock the spec peaks
(157.3 TF fp32, 2.5 PF bf16 dense) are quoted at.  Writes <outdir>/mfma.json."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402

out = sys.argv[1]
SIMDS = 256 * 4
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "pmc", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(out, "pmc", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        gs = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        key = (short(r["Kernel_Name"]), gs, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"])
               * int(r["Workgroup_Size_Z"]))
        durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
res = {}
rows = []
for key, c in vals.items():
    n = len(c.get("SQ_INSTS_MFMA", []))
    if not n:
        continue
    avg = lambda k: sum(c[k]) / len(c[k]) if c.get(k) else 0.0  # noqa: E731
    d = durs.get(key)
    dur = sum(d) / len(d) if d else None
    clk = avg("GRBM_GUI_ACTIVE") / 8 / dur if dur else None
    busy = avg("SQ_VALU_MFMA_BUSY_CYCLES")
    util = busy / (dur * clk * SIMDS) if dur and clk else None
    nominal = busy / (dur * 2.4e9 * SIMDS) if dur else None
    name = f"{key[0]} grid={key[1]} wg={key[2]}"
    res[name] = {"launches": n, "avg_us": dur * 1e6 if dur else None, "mfma_insts": avg("SQ_INSTS_MFMA"),
                 "mfma_busy_cycles": busy, "clock_ghz": clk / 1e9 if clk else None, "mfma_busy": util,
                 "mfma_busy_nominal": nominal,
                 "cu_busy_quad_cycles": avg("SQ_BUSY_CU_CYCLES"), "wave_quad_cycles": avg("SQ_WAVE_CYCLES")}
    rows.append((dur * n if dur else 0, name, res[name]))
for _, name, r in sorted(rows, reverse=True):
    if not r["mfma_insts"]:
        continue
    print(f"{name[:78]:78s} n={r['launches']:4d} {r['avg_us'] or 0:8.2f} us  MFMA {r['mfma_insts']:10.0f}  "
          f"clk {r['clock_ghz'] or 0:4.2f} GHz  mfma_busy {100 * (r['mfma_busy'] or 0):5.1f} %  "
          f"vs 2.4 GHz {100 * (r['mfma_busy_nominal'] or 0):5.1f} %")
cfg = None
for line in open(os.path.join(out, "bench.log")):
    if line.startswith("{"):
        cfg = json.loads(line).get("config")
json.dump({"config": cfg, "kernels": res}, open(os.path.join(out, "mfma.json"), "w"), indent=1)
