#!/bin/bash
# round 4: fcproj (DE=1) / qkv (DE=2) / both (DE=3) k-group waits at 3-4 row blocks vs the product (fc only there)
set -u
o=gpurun_out/r4de; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
HPA_LIB=$X/libde3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py -q --maxfail=3 --timeout 200 \
  --timeout-method thread -p no:cacheprovider -k "chain6 or 124m" > $o/pytest.txt 2>&1 || exit $?
tail -1 $o/pytest.txt > $o/summary.txt
for B in 64 48; do
  for v in prod de1 de2 de3 prod de1 de2 de3; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = prod ] || lib=$X/lib$v.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_$v.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B $v', d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
cat $o/summary.txt
