#!/bin/bash
# round-4 logits A/B on one GPU box: the ring logits kernel walking a
# contiguous run of column tiles per workgroup (librgc) vs the round-3 strided
# walk (librgs, -DHPA_RG_STRIDED=1): logits tests, per-workgroup timelines
# (trace builds librgct / librgst, tools/rg_trace.py), kernel time + bench
# ms/step, and the WRITE_SIZE / FETCH_SIZE PMC passes.
# Libraries: build/*.o of the tree + hpa_logits.hip compiled with the -D flags
# above (HPA_RG_STRIDED, HPA_RG_PRO, HPA_RG_TRACE), linked into tools/ablib/.
set -u
o=gpurun_out/r4lg; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
HPA_LIB=$X/librgc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -k logits -m gpu -x -v \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest_logits.txt 2>&1 || exit $?
for v in rgct rgst; do
  HPA_LIB=$X/lib$v.so timeout -k 10 120 python -u tools/rg_trace.py 64 10 > $o/trace_$v.txt 2>&1 || exit $?
done
for v in rgs rgc rgs rgc; do
  HPA_LIB=$X/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k_$v -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k_$v.log 2>&1 || exit $?
  python3 tools/kstats.py $o/k_$v/run_kernel_trace.csv | grep -i "logits\|argmax" | sed "s/^/$v /" >> $o/summary.txt
  HPA_LIB=$X/lib$v.so timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --cpu-baseline off --prof-steps 0 \
    > $o/b_$v.log 2>&1 || exit $?
  grep "^{" $o/b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v ms/step', d['ms_per_step'])" >> $o/summary.txt
done
for v in rgs rgc; do
  for ctr in WRITE_SIZE FETCH_SIZE; do
    HPA_LIB=$X/lib$v.so timeout -k 10 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $o/p_$v/$ctr -o run -- \
      python3 bench.py --no-graph --cpu-baseline off --prof-steps 0 --steps 4 --warmup 1 > $o/p_${v}_$ctr.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py $o/p_$v > $o/traffic_$v.txt 2>&1 || exit $?
  grep -i "logits" $o/traffic_$v.txt | sed "s/^/$v /" >> $o/summary.txt
done
cat $o/summary.txt
# form 8 (XL): the scheduling barrier after the A loads (product lib) vs none (libnosb)
for v in prod nosb prod nosb; do
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = nosb ] && lib=$X/libnosb.so
  HPA_LIB=$lib timeout -k 10 200 python3 bench.py --model XL --page-size 32 --steps 8 --warmup 2 --cpu-baseline off \
    --prof-steps 0 > $o/xl_$v.log 2>&1 || exit $?
  grep "^{" $o/xl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xl $v ms/step', d['ms_per_step'])" >> $o/summary.txt
done
cat $o/summary.txt
