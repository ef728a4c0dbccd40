#!/bin/bash
# round 5: XL chain form 8 with each unit's tile walk rotated by row block (librot1 consecutive, librot2 spread):
# parity, XL bench A/B, per-wave fc timeline
set -u
o=gpurun_out/r5ag; mkdir -p $o; export TMPDIR=/tmp
for r in 1 2; do
  HPA_LIB=$PWD/llm.c-paged_amd/librot$r.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py -x -q --timeout 300 --timeout-method thread -k "chain8" > $o/pytest_rot$r.txt 2>&1 || exit $?
done
for rep in 1 2; do
for lib in libpaged_hip.so librot1.so librot2.so; do
  HPA_LIB=$PWD/llm.c-paged_amd/$lib timeout -k 10 300 python -u bench.py --model XL --page-size 32 --cpu-baseline off --steps 8 --warmup 2 > $o/xl.txt 2>&1 || exit $?
  tail -1 $o/xl.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib XL', d['value'], d['ms_per_step'])" >> $o/summary.txt
done
done
for r in 1 2; do
  HPA_LIB=$PWD/llm.c-paged_amd/libtrrot$r.so timeout -k 10 300 python -u tools/cx_wave_trace.py 64 200 > $o/cx_wave_rot$r.txt 2>&1 || exit $?
done
