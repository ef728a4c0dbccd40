#!/bin/bash
# A/B of one engine environment switch: bench + kernel stats with VAR=a and VAR=b.
# usage: tools/diag/env_ab.sh <tag> <VAR> <a> <b> [bench args...]
set -u
tag=$1; var=$2; va=$3; vb=$4; shift 4
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for v in $va $vb; do
  env $var=$v timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $out/$v.log 2>&1 || exit $?
  grep "^{" $out/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$var=$v ms/step', d['ms_per_step'])"
done
for v in $va $vb; do
  export $var=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/p$v -o run -- python3 bench.py --cpu-baseline off --steps 10 "$@" > $out/$v.plog 2>&1 || exit $?
  python3 tools/kstats.py $out/p$v/run_kernel_trace.csv | grep -v rocclr | head -9 | sed "s/^/$var=$v /"
done
