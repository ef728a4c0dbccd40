# the chain's wide units: parity tests, then bench A/B (HPA_PL_WIDE=0: 4-wave units; =12: wide only at <= 16 rows)
set -u
o=gpurun_out/wide; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 240 --timeout-method thread > $o/pytest_layer.txt 2>&1
rc=$?; grep -E "FAIL|ERROR|passed|failed" $o/pytest_layer.txt | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --batch 32 --cpu-baseline off > $o/bench_b32_wide6.log 2>&1 || exit $?
HPA_PL_WIDE=12 timeout -k 10 300 python bench.py --batch 32 --cpu-baseline off > $o/bench_b32_slot.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 24 --cpu-baseline off > $o/bench_b24_wide6.log 2>&1 || exit $?
HPA_PL_WIDE=12 timeout -k 10 300 python bench.py --batch 24 --cpu-baseline off > $o/bench_b24_slot.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --batch 8 --cpu-baseline off > $o/bench_b8_wide12.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench_b64.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $o/bench_b*.log
