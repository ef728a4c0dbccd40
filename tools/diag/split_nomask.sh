#!/bin/bash
set -u
out=gpurun_out/snm; mkdir -p $out
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 "$@" > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $out/$tag.log; exit 1; }; grep "^{" $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['ms_per_step'], d['config']['split_gemm_cus'])"; }
b nm_eager --split 256 --no-graph || exit 1
timeout -k 10 100 python -X faulthandler bench.py --cpu-baseline off --prof-steps 0 --split 256 > $out/fh.log 2>&1; echo "graph rc=$?"; grep -v "^ *$" $out/fh.log | tail -12
exit 0
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run --output-format csv -- python bench.py --cpu-baseline off --prof-steps 0 --steps 8 --split 256 > $out/p.log 2>&1; echo "rocprof rc=$?"
python3 tools/timeline.py $out/prof/run_kernel_trace.csv 600 > $out/timeline.txt; head -8 $out/timeline.txt; tail -1 $out/timeline.txt
