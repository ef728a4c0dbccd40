#!/bin/bash
# kernel trace of one bench configuration: per-kernel average durations
set -u
tag=$1; shift
out=gpurun_out/kt_$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run --output-format csv -- python bench.py --cpu-baseline off --prof-steps 0 --steps 10 "$@" > $out/p.log 2>&1
echo "rocprof rc=$?"
python3 tools/timeline.py $out/prof/run_kernel_trace.csv 700 > $out/timeline.txt 2>&1; head -10 $out/timeline.txt
