#!/bin/bash
# round 5: the bf16-weight chain (hpa_chain_b16.hip): parity tests, config-5 bench A/B, kernel stats
set -u
o=gpurun_out/r5d; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "config5 or bf16_chain" > $o/pytest_b16.txt 2>&1 || exit $?
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_chain.txt 2>&1 || exit $?
HPA_LAYER_KERNEL=0 timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_five.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o c5 -- python3 bench.py $C5 --spinup 0 > $o/prof_c5.txt 2>&1 || exit $?
