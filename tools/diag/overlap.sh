#!/bin/bash
# overlapped step: tests, then bench lines for chain workgroup counts
set -u
out=gpurun_out/ovl; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -k overlap -m gpu -v --timeout 100 --timeout-method thread -p no:cacheprovider -x > $out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" $out/t.log | head -20; [ $rc = 0 ] || exit $rc
for n in ${1:-64 128 192 256}; do
  timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 --overlap $n > $out/b_$n.log 2>&1 || { echo "fail $n"; tail -3 $out/b_$n.log; exit 1; }
  grep "^{" $out/b_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap', $n, 'ms/step', d['ms_per_step'], d['value'])"
done
