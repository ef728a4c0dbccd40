#!/bin/bash
# round 4: the balanced decode attention (hpa_paged_attention_decode_flat) -- tests, the
# attention-alone scan, bench A/B at small batches (auto = balanced vs the split grid)
set -u
o=gpurun_out/r4flat2; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_attention.py -q \
  --maxfail=4 --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1 || exit $?
tail -2 $o/pytest.txt > $o/summary.txt
timeout -k 10 300 python -u tools/attn_flat_scan.py > $o/scan.txt 2>&1 || exit $?
cat $o/scan.txt >> $o/summary.txt
for B in 8 16; do
  for f in 2 1 2 1; do
    timeout -k 10 120 python -u bench.py --batch $B --attn-flat $f --steps 40 --warmup 5 --cpu-baseline off \
      > $o/bench_b${B}_f$f.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_f$f.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B flat-mode $f', d['config']['attn_form'], d['ms_per_step'], d['value'], d['roofline']['achieved'])" >> $o/summary.txt
  done
done
cat $o/summary.txt
