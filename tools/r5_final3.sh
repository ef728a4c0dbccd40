#!/bin/bash
# round 5 final validation (after the bf16-pool attention waves change): smoke, GPU suite, default bench, kernel stats
set -u
o=gpurun_out/r5final3; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > $o/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $o/bench_default.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c2 -- python3 bench.py --cpu-baseline off --spinup 0 > $o/prof_c2.txt 2>&1 || exit $?
