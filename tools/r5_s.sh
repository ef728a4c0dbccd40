#!/bin/bash
# round 5: chain form 6 beside its attention (no kernel boundary): parity, then bench A/B against the boundary
set -u
o=gpurun_out/r5s; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > $o/pytest_layer_decode.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "config2" > $o/pytest_c2.txt 2>&1 || exit $?
for B in 64 32 16 8; do
  timeout -k 10 200 python -u bench.py --batch $B --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b${B}.txt 2>&1 || exit $?
  HPA_LIB=$PWD/llm.c-paged_amd/libnb.so timeout -k 10 200 python -u bench.py --batch $B --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b${B}_nb.txt 2>&1 || exit $?
done
