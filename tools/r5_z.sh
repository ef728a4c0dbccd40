#!/bin/bash
# round 5: HBM traffic of the GPT-2 XL step's kernels (chain form 8: weight re-fetch across row blocks?)
set -u
o=gpurun_out/r5z; mkdir -p $o; export TMPDIR=/tmp
bash tools/pmc_traffic.sh $o/pmc_xl --model XL --page-size 32 --steps 2 --warmup 1 > $o/pmc_xl.log 2>&1 || exit $?
