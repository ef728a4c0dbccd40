#!/bin/bash
# round 5: co-residency test with 200 held CUs
set -u
o=gpurun_out/r5q; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_coresidency.py -v -s --timeout 200 --timeout-method thread > $o/pytest_cores.txt 2>&1 || exit $?
