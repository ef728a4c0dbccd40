#!/bin/bash
# round 5: config-5 bench, bf16 chain vs five launches, and kernel stats
set -u
o=gpurun_out/r5e2; mkdir -p $o; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_chain.txt 2>&1 || exit $?
HPA_LAYER_KERNEL=0 timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_five.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o c5 -- python3 bench.py $C5 --spinup 0 > $o/prof_c5.txt 2>&1 || exit $?
