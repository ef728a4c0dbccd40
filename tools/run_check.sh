#!/bin/bash
# GPU check: selected tests, then bench (1 GPU) and the kernel-stats profile.
# usage: tools/run_check.sh <tag> "<pytest selection>" [bench args...]
set -u
tag=$1; sel=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -m pytest $sel -m gpu -q -p no:cacheprovider -x > "$out/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$out/t.log"
if [ $rc != 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --cpu-baseline off "$@" > "$out/b.log" 2>&1
rc=$?; echo "bench rc=$rc"
if [ $rc != 0 ]; then tail -5 "$out/b.log"; exit $rc; fi
grep "^{" "$out/b.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'value', d['value'], 'attn', d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python bench.py --cpu-baseline off --steps 10 "$@" > "$out/p.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 tools/kstats.py "$out/prof/run_kernel_trace.csv" > "$out/kstats.txt" 2>&1; head -12 "$out/kstats.txt"
exit 0
