#!/bin/bash
# round 5: GPU suite on the reverted (round-4 layer) tree + default bench + kernel stats
set -u
o=gpurun_out/r5c; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 4 > $o/bench.txt 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off > $o/bench_prof.txt 2>&1 || exit $?
