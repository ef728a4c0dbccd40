#!/bin/bash
# round 5: bf16 first launch (embed + qkv(0)), continuous weight stream in the A-resident bf16 kernel
set -u
o=gpurun_out/r5i; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "config5 or bf16_chain" > $o/pytest_b16.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 200 python -u tools/pl_trace.py 256 2000 1 b16 > $o/trace_b16_b256.txt 2>&1 || exit $?
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5.txt 2>&1 || exit $?
for u in 16; do
  HPA_LIB=$PWD/llm.c-paged_amd/libu$u.so timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_u$u.txt 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c5 -- python3 bench.py $C5 --spinup 0 > $o/prof_c5.txt 2>&1 || exit $?
