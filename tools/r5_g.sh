#!/bin/bash
# round 5: bf16 chain v2 (bf16 fch, fcproj 4x3, qkv 2x5, late poll-wave prefetch): tests, traces, config-5 A/B
set -u
o=gpurun_out/r5g; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "config5 or bf16_chain" > $o/pytest_b16.txt 2>&1 || exit $?
for B in 256 64; do
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 200 python -u tools/pl_trace.py $B 2000 1 b16 > $o/trace_b16_b$B.txt 2>&1 || exit $?
  HPA_LIB=$PWD/llm.c-paged_amd/libcb_trace_pl0.so timeout -k 10 200 python -u tools/pl_trace.py $B 2000 1 b16 > $o/trace_b16_pl0_b$B.txt 2>&1 || exit $?
done
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libcb_pl0.so timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_pl0.txt 2>&1 || exit $?
