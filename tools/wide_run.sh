# the chain's wide units: parity tests, then bench A/B (HPA_PL_WIDE=0: 4-wave units everywhere)
set -u
o=gpurun_out/wide2; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 240 --timeout-method thread > $o/pytest_layer.txt 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $o/pytest_layer.txt | tail -8; [ $rc -le 1 ] || exit $rc
for b in 64 48 32 8; do
  timeout -k 10 300 python bench.py --batch $b --cpu-baseline off > $o/bench_b${b}_wide.log 2>&1 || exit $?
  HPA_PL_WIDE=0 timeout -k 10 300 python bench.py --batch $b --cpu-baseline off > $o/bench_b${b}_slot.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_b64_wide_again.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $o/bench_b*.log
