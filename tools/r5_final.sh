#!/bin/bash
# round 5 final measurements: PMC traffic + MFMA busy (configs 2 and 5), kernel stats and bench lines for
# B = 8 / 16, config 5, XL, and the N = 2 / 4 / 8 rank shapes (--emulate-rank)
set -u
o=gpurun_out/r5final; mkdir -p $o; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16"
bash tools/pmc_traffic.sh $o/pmc_c2 --steps 4 --warmup 1 > $o/pmc_c2.log 2>&1 || exit $?
bash tools/pmc_traffic.sh $o/pmc_c5 $C5 --steps 4 --warmup 1 > $o/pmc_c5.log 2>&1 || exit $?
bash tools/pmc_mfma.sh $o/mfma_c2 --steps 4 --warmup 1 > $o/mfma_c2.log 2>&1 || exit $?
bash tools/pmc_mfma.sh $o/mfma_c5 $C5 --steps 4 --warmup 1 > $o/mfma_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c5 -o c5 -- python3 bench.py $C5 --cpu-baseline off --spinup 0 --steps 20 --warmup 3 > $o/prof_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_b8 -o b8 -- python3 bench.py --batch 8 --cpu-baseline off --spinup 0 --steps 30 --warmup 3 > $o/prof_b8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_xl -o xl -- python3 bench.py --model XL --cpu-baseline off --spinup 0 --steps 8 --warmup 2 > $o/prof_xl.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $C5 --steps 20 --warmup 3 --cpu-seconds 4 > $o/bench_c5.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --batch 8 --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b8.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --batch 16 --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b16.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model XL --cpu-baseline off --steps 10 --warmup 2 > $o/bench_xl.log 2>&1 || exit $?
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --emulate-rank $n --cpu-baseline off > $o/emul$n.log 2>&1 || exit $?
done
