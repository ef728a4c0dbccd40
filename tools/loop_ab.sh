#!/bin/bash
# looped-GEMM loop-exit fix: GPU tests of the GEMM users, then the XL GEMM
# sweep, the XL bench, the prefill bench and the default bench
set -u
out=gpurun_out/loop; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_prefill.py tests/test_gpu_decode.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; echo "pytest rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 240 python -u tools/gemm_tune.py 64 1600 > $out/tune_xl.log 2>&1 || exit $?
grep -E "sum best" $out/tune_xl.log
timeout -k 10 300 python -u bench.py --model XL --page-size 32 --cpu-baseline off > $out/bench_xl.log 2>&1 || exit $?
grep "^{" $out/bench_xl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('XL', d['ms_per_step'], d['value'])"
timeout -k 10 300 python -u bench.py --prefill real --cpu-baseline off > $out/bench_prefill.log 2>&1 || exit $?
grep -i "prefill" $out/bench_prefill.log | tail -3
timeout -k 10 300 python -u bench.py --cpu-baseline off > $out/bench_c2.log 2>&1 || exit $?
grep "^{" $out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['ms_per_step'], d['value'])"
