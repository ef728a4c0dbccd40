#!/bin/bash
# round-4 A/B on the current tree: layer parity (forms 6 / 8), 124M B=64 / 8 and XL bench lines,
# form-6 and form-8 phase traces
set -u
o=gpurun_out/r4ab; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v -s --timeout 300 --timeout-method thread -k "chain6 or chain8 or 124m" > $o/pytest_layer.txt 2>&1 || exit $?
for B in 64 8; do
  timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off --prof-steps 0 > $o/bench_b$B.txt 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py --model XL --page-size 32 --steps 8 --warmup 2 --cpu-baseline off --prof-steps 0 > $o/bench_xl.txt 2>&1 || exit $?
for f in $o/bench_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'], d['config']['layer_loop'][-28:])"; done | tee $o/summary.txt
lib=$PWD/llm.c-paged_amd/libpaged_hip_trace.so
HPA_LIB=$lib timeout -k 10 120 python -u tools/pl_trace.py 64 990 5 > $o/trace6_b64.txt 2>&1 || exit $?
HPA_LIB=$lib timeout -k 10 120 python -u tools/pl_trace.py 8 990 5 > $o/trace6_b8.txt 2>&1 || exit $?
HPA_LIB=$lib timeout -k 10 200 python -u tools/pl_trace.py 64 990 6 XL > $o/trace8_xl.txt 2>&1 || exit $?
