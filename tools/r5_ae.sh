#!/bin/bash
# round 5: chain form 8 with 4 weight half-tiles in flight (libah4) vs 3 (product): parity + XL bench A/B
set -u
o=gpurun_out/r5ae; mkdir -p $o; export TMPDIR=/tmp
HPA_LIB=$PWD/llm.c-paged_amd/libah4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py -x -q --timeout 300 --timeout-method thread -k "chain8" > $o/pytest_ah4.txt 2>&1 || exit $?
for rep in 1 2; do
for lib in libpaged_hip.so libah4.so; do
  HPA_LIB=$PWD/llm.c-paged_amd/$lib timeout -k 10 300 python -u bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 --warmup 2 > $o/xl.txt 2>&1 || exit $?
  tail -1 $o/xl.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib XL', d['value'], d['ms_per_step'])" >> $o/summary.txt
done
done
HPA_LIB=$PWD/llm.c-paged_amd/libah4.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o xl -- python3 bench.py --model XL --page-size 32 --cpu-baseline off --spinup 0 --steps 6 --warmup 2 > $o/prof.txt 2>&1 || exit $?
