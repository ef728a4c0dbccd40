#!/bin/bash
# round 4: the two-lane step (gpt2_decode_set_lanes) -- bit-identity test and
# bench A/B at B = 64 / 48 -- and the logits prologue / tile-walk variants
# (tools/ablib/liblg_*: s = strided walk, c = contiguous runs; PRO 0 both
# prologue tiles at the start, 1 tile 1 after the first barrier, 2 both after
# it; *t = trace builds for tools/rg_trace.py)
set -u
o=gpurun_out/r4ln; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_fused.py -x -v -s --timeout 300 \
  --timeout-method thread -k "two_lane or logits" > $o/pytest.txt 2>&1 || exit $?
for B in 64 48; do
  for ln in 1 2 1 2; do
    timeout -k 10 120 python -u bench.py --batch $B --lanes $ln --steps 40 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_b${B}_l$ln.txt 2>&1 || exit $?
    grep "^{" $o/bench_b${B}_l$ln.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B lanes', d['config']['lanes'], d['ms_per_step'], d['value'])" >> $o/summary.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k_l2 -o run -- \
  python3 bench.py --lanes 2 --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k_l2.log 2>&1 || exit $?
python3 tools/kstats.py $o/k_l2/run_kernel_trace.csv 13 > $o/kstats_l2.txt
for v in s0t s1t s2t c1t; do
  HPA_LIB=$X/liblg_$v.so timeout -k 10 120 python -u tools/rg_trace.py 64 10 > $o/trace_$v.txt 2>&1 || exit $?
  grep -E "span|prologue|iter 12|end |iteration" $o/trace_$v.txt | sed "s/^/$v /" >> $o/summary.txt
done
for v in s0 s1 s2 c1; do
  HPA_LIB=$X/liblg_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k_$v -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/k_$v.log 2>&1 || exit $?
  python3 tools/kstats.py $o/k_$v/run_kernel_trace.csv | grep -i "logits\|argmax" | sed "s/^/$v /" >> $o/summary.txt
done
cat $o/summary.txt
