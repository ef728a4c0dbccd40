#!/bin/bash
# Split-step sweep: tests, then bench lines for GEMM CU budgets, then a
# kernel trace of one budget (concurrency of the two streams).
# usage: tools/split_sweep.sh <tag> "<cus list>" [trace_cus] [bench args...]
set -u
tag=$1; list=$2; tr=${3:-0}; shift 3 || shift $#
out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -k split -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider -x > "$out/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$out/t.log"; [ $rc = 0 ] || exit $rc
for n in $list; do
  timeout -k 10 300 python bench.py --cpu-baseline off --prof-steps 0 --split $n "$@" > "$out/b_$n.log" 2>&1
  rc=$?; [ $rc = 0 ] || { echo "bench $n rc=$rc"; tail -5 "$out/b_$n.log"; exit $rc; }
  grep "^{" "$out/b_$n.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split', $n, 'ms/step', d['ms_per_step'], 'tok/s', d['value'])"
done
if [ "$tr" != 0 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/prof" -o run --output-format csv -- python bench.py --cpu-baseline off --prof-steps 0 --steps 8 --split $tr "$@" > "$out/p.log" 2>&1
  echo "rocprof rc=$?"
  python3 tools/timeline.py "$out/prof/run_kernel_trace.csv" > "$out/timeline.txt" 2>&1; tail -14 "$out/timeline.txt"
fi
exit 0
