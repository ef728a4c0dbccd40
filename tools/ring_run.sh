set -u
o=gpurun_out/ring; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k "ring" > $o/pytest.txt 2>&1; rc=$?; tail -2 $o/pytest.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/ring_tune.py > $o/tune0.txt 2>&1 || exit $?
HPA_RING_MODE=1 timeout -k 10 120 python -u tools/ring_tune.py > $o/tune1.txt 2>&1 || exit $?
HPA_RING_MODE=2 timeout -k 10 120 python -u tools/ring_tune.py > $o/tune2.txt 2>&1 || exit $?
HPA_RING_ROT=1 timeout -k 10 120 python -u tools/ring_tune.py > $o/tune3_rot.txt 2>&1 || exit $?
HPA_RING_ROT=1 HPA_RING_MODE=1 timeout -k 10 120 python -u tools/ring_tune.py > $o/tune4_rot_loads.txt 2>&1 || exit $?
cat $o/tune*.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "config3" > $o/pytest_xl.txt 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed|B=" $o/pytest_xl.txt | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 > $o/bench_xl_ring.log 2>&1 || exit $?
HPA_GEMM_RING=0 timeout -k 10 300 python bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 > $o/bench_xl_loop.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' $o/bench_xl_ring.log $o/bench_xl_loop.log
