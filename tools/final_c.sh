# round-end evidence on the final tree: the full GPU suite, the headline bench
# (with its CPU baseline) and its rocprofv3 kernel stats, the small batches, XL
set -u
o=gpurun_out/final2; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 240 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.txt 2>&1
rc=$?; tail -3 $o/pytest_gpu.txt; grep -E "^FAILED|^ERROR" $o/pytest_gpu.txt | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py > $o/bench_c2.log 2>&1 || exit $?
grep "^{" $o/bench_c2.log > $o/bench_line.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof_c2 -o run --output-format csv -- python3 bench.py --cpu-baseline off > $o/prof_c2.log 2>&1 || exit $?
python3 tools/kstats.py $o/prof_c2/run_kernel_trace.csv 32 > $o/kstats_c2.txt
for b in 8 16 32; do timeout -k 10 300 python bench.py --batch $b --cpu-baseline off > $o/bench_b$b.log 2>&1 || exit $?; done
timeout -k 10 400 python bench.py --model XL --page-size 32 --cpu-baseline off > $o/bench_xl.log 2>&1 || exit $?
grep -ho '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $o/bench_*.log
head -6 $o/kstats_c2.txt
