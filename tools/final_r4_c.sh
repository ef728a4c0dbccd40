#!/bin/bash
# round-4 evidence, part c: profile_round.sh a (config 2: bench + CPU baseline,
# rocprofv3 kernel stats, PMC traffic, MFMA busy, attention scan, small
# batches), then emulated strong-scaling ranks
set -u
o=gpurun_out/r4final; mkdir -p $o; export TMPDIR=/tmp
bash tools/profile_round.sh $o a || exit $?
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --emulate-rank $n --scaling strong --cpu-baseline off > $o/emul$n.log 2>&1 || exit $?
done
grep -ho '"ms_per_step": [0-9.]*\|"projected_n_gpu_tokens_per_s": [0-9.]*' $o/emul*.log
