#!/bin/bash
# round 5, first GPU call: the whole GPU suite after the pruning + new tests,
# the per-CU stream microbenchmark, the default bench and the N=8 rank shape
set -u
o=gpurun_out/r5a; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 240 ./tools/micro/cu_stream > $o/cu_stream.txt 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 4 > $o/bench.txt 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --emulate-rank 8 --cpu-baseline off > $o/emul8.txt 2>&1 || exit $?
