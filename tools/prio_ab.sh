#!/bin/bash
# s_setprio around the looped GEMM's MFMA clusters: GPU tests of the GEMM
# users, the XL GEMM sweep, the XL bench and the prefill bench
set -u
out=gpurun_out/prio; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_prefill.py tests/test_gpu_decode.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; echo "pytest rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 240 python -u tools/gemm_tune.py 64 1600 > $out/tune_xl.log 2>&1 || exit $?
grep -v "^\[hpa" $out/tune_xl.log | grep -A1 auto | grep " us"; grep "sum best" $out/tune_xl.log
timeout -k 10 300 python -u bench.py --model XL --page-size 32 --cpu-baseline off > $out/bench_xl.log 2>&1 || exit $?
grep "^{" $out/bench_xl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('XL', d['ms_per_step'], d['value'])"
timeout -k 10 300 python -u bench.py --prefill real --cpu-baseline off > $out/bench_prefill.log 2>&1 || exit $?
grep "^{" $out/bench_prefill.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefill', d['prefill']['tokens_per_s'], 'decode', d['value'])"
