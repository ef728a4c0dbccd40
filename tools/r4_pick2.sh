#!/bin/bash
# round 4: in-launch greedy pick (all partial loads in flight) vs the separate argmax launch, + the config-4 tests
set -u
o=gpurun_out/r4pk3; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread \
  -k "pick or logits" > $o/pytest.txt 2>&1 || exit $?
for B in 64 8; do
  for v in prod nopick prod nopick; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = nopick ] && lib=$X/libnopick.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_$v.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B $v', d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k.log 2>&1 || exit $?
python3 tools/kstats.py $o/k/run_kernel_trace.csv 13 > $o/kstats.txt
grep -i "logits\|argmax" $o/kstats.txt >> $o/summary.txt
# timeout -k 10 700 python -u -m pytest tests/test_gpu_multi_rank.py -x -v -s --timeout 600 --timeout-method thread \
  > $o/pytest_mr.txt 2>&1 || exit $?
# grep -E "passed|failed" $o/pytest_mr.txt >> $o/summary.txt
cat $o/summary.txt
