#!/bin/bash
# lanes vs hardware queues: step time of 1/2 lanes (graph and eager) at the
# default and a larger GPU_MAX_HW_QUEUES, and the kernel concurrency of one
set -u
out=gpurun_out/lhq; mkdir -p $out
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 "$@" > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $out/$tag.log; exit 1; }; grep "^{" $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'])"; }
b q4_l1 --lanes 1 && b q4_l2g --lanes 2 && b q4_l2e --lanes 2 --no-graph || exit 1
export GPU_MAX_HW_QUEUES=8
b q8_l1 --lanes 1 && b q8_l2g --lanes 2 && b q8_l2e --lanes 2 --no-graph || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run --output-format csv -- python bench.py --cpu-baseline off --prof-steps 0 --steps 8 --lanes 2 --no-graph > $out/p.log 2>&1; echo "rocprof rc=$?"
python3 tools/timeline.py $out/prof/run_kernel_trace.csv 600 | tail -1
