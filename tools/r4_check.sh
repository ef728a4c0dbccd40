#!/bin/bash
# round 4: validity + config-4 default-path tests, the pinned B=256 check, a bench line
set -u
o=gpurun_out/r4a; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests/test_gpu_multi_rank.py tests/test_gpu_configs.py -x -v -s \
  --timeout 400 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > $o/bench.txt 2>&1 || exit $?
for n in 2 4 8; do
  timeout -k 10 120 python -u bench.py --emulate-rank $n --cpu-baseline off > $o/emul$n.txt 2>&1 || exit $?
done
