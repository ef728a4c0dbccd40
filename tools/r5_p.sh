#!/bin/bash
# round 5: co-residency test, then the whole GPU suite on the pruned product library, default bench + kernel stats
set -u
o=gpurun_out/r5p; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_coresidency.py -v -s --timeout 200 --timeout-method thread > $o/pytest_cores.txt 2>&1 || exit $?
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 4 > $o/bench.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c2 -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --spinup 0 > $o/prof_c2.txt 2>&1 || exit $?
