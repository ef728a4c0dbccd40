# round-end evidence, part a: the full GPU suite, the ring GEMM scan, XL
# bench A/B, then profile_round.sh a
set -u
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.txt; grep -E "^FAILED|^ERROR" gpurun_out/final/pytest_gpu.txt | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python -u tools/ring_tune.py > gpurun_out/final/ring_tune.txt 2>&1 || exit $?
cat gpurun_out/final/ring_tune.txt
timeout -k 10 300 python bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 > gpurun_out/final/bench_xl_split.log 2>&1 || exit $?
HPA_GEMM_RING=1 timeout -k 10 300 python bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 > gpurun_out/final/bench_xl_ring1.log 2>&1 || exit $?
HPA_GEMM_RING=0 timeout -k 10 300 python bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 > gpurun_out/final/bench_xl_loop.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/final/bench_xl_*.log
bash tools/profile_round.sh gpurun_out/final a
