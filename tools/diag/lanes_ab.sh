#!/bin/bash
# lanes A/B: graph vs eager, 1/2/4 lanes; kernel trace of eager 2 lanes
set -u
out=gpurun_out/lanes; mkdir -p $out
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 "$@" > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $out/$tag.log; exit 1; }; grep "^{" $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'])"; }
b l1g --lanes 1 && b l2g --lanes 2 && b l1e --lanes 1 --no-graph && b l2e --lanes 2 --no-graph && b l4e --lanes 4 --no-graph && b l2g_hq --lanes 2 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run --output-format csv -- python bench.py --cpu-baseline off --prof-steps 0 --steps 8 --lanes 2 --no-graph > $out/p.log 2>&1; echo "rocprof rc=$?"
python3 tools/timeline.py $out/prof/run_kernel_trace.csv 600 > $out/timeline.txt 2>&1; head -12 $out/timeline.txt; tail -1 $out/timeline.txt
