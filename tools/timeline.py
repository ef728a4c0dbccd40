#!/usr/bin/env python3
"""Timeline view of a rocprofv3 kernel_trace.csv: for the last `window`
kernels, per kernel kind the average duration and the average idle gap
before it (time between the previous kernel's end and its start when no
other kernel was running), plus how much of the window the GPU had at least
one kernel in flight.  usage: timeline.py kernel_trace.csv [window]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
window = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-38:],
              r["Grid_Size_X"], r["Grid_Size_Y"]) for r in rows))
ks = ks[-window:]
t0, t1 = ks[0][0], max(k[1] for k in ks)
busy = 0
cur_s, cur_e = ks[0][0], ks[0][1]
gaps = collections.defaultdict(list)
durs = collections.defaultdict(list)
for s, e, name, gx, gy in ks:
    key = f"{name} g=({gx},{gy})"
    durs[key].append(e - s)
    if s > cur_e:
        busy += cur_e - cur_s
        gaps[key].append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        gaps[key].append(0)
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print(f"window {len(ks)} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us "
      f"({100.0 * busy / span:.1f} %), idle {(span - busy) / 1e3:.1f} us")
tot = sorted(durs, key=lambda k: -sum(durs[k]))
for k in tot:
    d, g = durs[k], gaps[k]
    print(f"{k:60s} n={len(d):5d} avg {sum(d) / len(d) / 1e3:8.2f} us  idle-before {sum(g) / len(g) / 1e3:6.2f} us"
          f"  sum {sum(d) / 1e3:9.1f} us")

# concurrency: sum of kernel durations over the union of their intervals
tot = sum(e - s for s, e, *_ in ks)
print(f"concurrency (sum of durations / busy time): {tot / busy:.2f}")
