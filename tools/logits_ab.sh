#!/bin/bash
# GPU box: logits kernel tests, then bench A/B of the logits forms (ring
# default vs HPA_LOGITS_FORM=16), then a rocprofv3 kernel-stats pass.
# usage: tools/logits_ab.sh <tag> [bench args...]
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -k "logits" -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/t.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" "$out/t.log" | tail -12
[ $rc = 0 ] || exit $rc
for f in ring 16 ring 16; do
  HPA_LOGITS_FORM=$f timeout -k 10 300 python bench.py --cpu-baseline off --steps 30 "$@" > "$out/b_$f.log" 2>&1
  rc=$?; [ $rc = 0 ] || { tail -5 "$out/b_$f.log"; exit $rc; }
  grep "^{" "$out/b_$f.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', 'ms/step', d['ms_per_step'], 'value', d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python bench.py --cpu-baseline off --steps 10 "$@" > "$out/p.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 tools/kstats.py "$out/prof/run_kernel_trace.csv" > "$out/kstats.txt" 2>&1; head -14 "$out/kstats.txt"
exit 0
