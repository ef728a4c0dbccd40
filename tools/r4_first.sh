#!/bin/bash
# round 4: the step's first launch (embed + qkv(0) + counter zeroing, hpa_decode_first) vs the
# embed kernel + one-shot qkv(0) GEMM (tools/ablib/libnofirst.so, -DDEC_FIRST_LAUNCH=0): tests, bench A/B
set -u
o=gpurun_out/r4fl; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
timeout -k 10 900 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_configs.py tests/test_gpu_decode.py -q --maxfail=4 \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1 || exit $?
tail -2 $o/pytest.txt >> $o/summary.txt
for B in 64 8; do
  for v in prod nofirst prod nofirst; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = nofirst ] && lib=$X/libnofirst.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_$v.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B $v', d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k.log 2>&1 || exit $?
python3 tools/kstats.py $o/k/run_kernel_trace.csv 13 > $o/kstats.txt
head -8 $o/kstats.txt >> $o/summary.txt
cat $o/summary.txt
