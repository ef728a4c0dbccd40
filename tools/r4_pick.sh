#!/bin/bash
# round 4: the in-launch greedy pick (product) vs the separate argmax launch
# (tools/ablib/libnopick.so), and the logits prologue / walk variants
# (liblg_s1/s2/c1 + trace builds; the product is s0)
set -u
o=gpurun_out/r4pk; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_decode.py -x -v --timeout 300 \
  --timeout-method thread -k "logits or pick or greedy or oracle" > $o/pytest.txt 2>&1 || exit $?
for B in 64 8; do
  for v in prod nopick prod nopick; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = nopick ] && lib=$X/libnopick.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_$v.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B $v', d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
for v in s0t s1t s2t c1t; do
  HPA_LIB=$X/liblg_$v.so timeout -k 10 120 python -u tools/rg_trace.py 64 10 > $o/trace_$v.txt 2>&1 || exit $?
  grep -E "span|prologue|iter 0 |iter 12|loop end|iteration" $o/trace_$v.txt | sed "s/^/$v /" >> $o/summary.txt
done
for v in prod s1 s2 c1; do
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = prod ] || lib=$X/liblg_$v.so
  HPA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k_$v -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k_$v.log 2>&1 || exit $?
  python3 tools/kstats.py $o/k_$v/run_kernel_trace.csv | grep -i "logits\|argmax" | sed "s/^/$v /" >> $o/summary.txt
done
cat $o/summary.txt
