#!/bin/bash
# qkv epilogue with the K/V destination (pos -> page) resolved before the
# phase's wait: the parity suites of the chain / first launch, then a same-box
# A/B of the step against the previous library (ab_old/, HPA_LIB) at B = 64 and
# B = 8, alternating, plus kernel stats of the new tree at B = 64
set -u
o=gpurun_out/r5kvdst; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_configs.py tests/test_gpu_multi_rank.py \
  tests/test_gpu_coresidency.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/ab_old/libpaged_hip.so; else L=$PWD/llm.c-paged_amd/libpaged_hip.so; fi
    HPA_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline off > $o/b64_${v}_$r.txt 2>&1 || exit $?
    HPA_LIB=$L timeout -k 10 200 python -u bench.py --batch 8 --cpu-baseline off --steps 30 --warmup 3 > $o/b8_${v}_$r.txt 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c2 -- python3 bench.py --cpu-baseline off --spinup 0 > $o/prof_c2.txt 2>&1 || exit $?
