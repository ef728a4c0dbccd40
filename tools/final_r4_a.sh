#!/bin/bash
# round-4 evidence, part a: the full GPU suite
set -u
o=gpurun_out/r4final; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.txt 2>&1
rc=$?; tail -3 $o/pytest_gpu.txt; grep -E "^FAILED|^ERROR" $o/pytest_gpu.txt | head
exit $rc
