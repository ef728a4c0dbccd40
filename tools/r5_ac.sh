#!/bin/bash
# round 5: config 5 with 8-wave attention on bf16 pools at >= 8 workgroups per CU: parity + bench (with CPU baseline)
set -u
o=gpurun_out/r5ac; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_attention.py -x -q --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --steps 25 --warmup 3 --cpu-seconds 4 > $o/bench_c5.txt 2>&1 || exit $?
