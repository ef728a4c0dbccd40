# the chain's wide units: parity tests, then B = 8 / 16 bench A/B (HPA_PL_WIDE=0: the 4-wave units)
set -u
o=gpurun_out/wide; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 240 --timeout-method thread > $o/pytest_layer.txt 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $o/pytest_layer.txt | tail -22; [ $rc -le 1 ] || exit $rc
for b in 8 16; do
  timeout -k 10 300 python bench.py --batch $b --cpu-baseline off > $o/bench_b${b}_wide.log 2>&1 || exit $?
  HPA_PL_WIDE=0 timeout -k 10 300 python bench.py --batch $b --cpu-baseline off > $o/bench_b${b}_slot.log 2>&1 || exit $?
done
grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $o/bench_b*.log
