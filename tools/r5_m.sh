#!/bin/bash
# round 5: the wave-local bf16 logits kernel: fused-GEMM tests, microbenchmark, config-5 bench A/B, kernel stats
set -u
o=gpurun_out/r5m; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread -k "bf16" > $o/pytest_fused_b16.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/b16_logits.py 256 10 > $o/b16_logits.txt 2>&1 || exit $?
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/liblw0.so timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_lw0.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c5 -- python3 bench.py $C5 --spinup 0 > $o/prof_c5.txt 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "config5 or bf16_chain" > $o/pytest_b16.txt 2>&1 || exit $?
