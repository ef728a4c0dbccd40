#!/bin/bash
# round 4: chain form 6 with per-k-group waits in fc (tools/ablib/libgw.so, -DHPA_C6_GW=1) vs the product
set -u
o=gpurun_out/r4gw; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
HPA_LIB=$X/libgw.so timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -q --maxfail=3 --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "chain6 or 124m or two_lane" > $o/pytest.txt 2>&1 || exit $?
tail -1 $o/pytest.txt > $o/summary.txt
for B in 64 32 8; do
  for v in prod gw prod gw; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = gw ] && lib=$X/libgw.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_$v.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B $v', d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
HPA_LIB=$X/libgwt.so timeout -k 10 120 python -u tools/pl_trace.py 64 990 5 > $o/trace_gw_b64.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py 64 990 5 > $o/trace_prod_b64.txt 2>&1 || exit $?
cat $o/summary.txt $o/trace_gw_b64.txt $o/trace_prod_b64.txt
