#!/bin/bash
# round-5 final numbers after the qkv K/V-destination change (f9eb95e; its
# GPU suite: profiles/r5/experiments/kvdst/pytest_full.txt): smoke, the
# default bench, kernel stats, B = 8 / the strong-scaling ranks, config 5, XL
set -u
o=gpurun_out/r5final4; mkdir -p $o; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $o/bench_default.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o c2 -- python3 bench.py --cpu-baseline off --spinup 0 > $o/prof_c2.txt 2>&1 || exit $?
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --emulate-rank $n --cpu-baseline off > $o/emul$n.txt 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py $C5 > $o/bench_c5.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model XL --cpu-baseline off --steps 10 --warmup 2 > $o/bench_xl.txt 2>&1 || exit $?
