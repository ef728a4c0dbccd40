#!/bin/bash
# round-4 evidence, part b: profile_round.sh b (configs 5 and 3, prefill, sampling)
set -u
o=gpurun_out/r4final; mkdir -p $o; export TMPDIR=/tmp
bash tools/profile_round.sh $o b
