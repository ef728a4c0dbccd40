#!/bin/bash
# round 5: bf16 logits with 2 (product) / 4 (A/B) column tiles per wave per round: microbenchmark,
# config-5 bench, kernel stats, then the whole GPU suite
set -u
o=gpurun_out/r5k; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/b16_logits.py 256 10 > $o/b16_logits_tpw2.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libtpw4.so timeout -k 10 240 python -u tools/b16_logits.py 256 10 > $o/b16_logits_tpw4.txt 2>&1 || exit $?
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 20 --warmup 3"
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libtpw4.so timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5_tpw4.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c5 -- python3 bench.py $C5 --spinup 0 > $o/prof_c5.txt 2>&1 || exit $?
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || exit $?
