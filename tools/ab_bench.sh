#!/bin/bash
# A/B: bench + kernel stats with the product library and an alternative build
# (HPA_LIB).  usage: tools/ab_bench.sh <tag> <alt .so> [bench args...]
set -u
tag=$1; alt=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for v in base alt; do
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = alt ] && lib=$PWD/$alt
  HPA_LIB=$lib timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $out/$v.log 2>&1 || exit $?
  grep "^{" $out/$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v ms/step', d['ms_per_step'])"
  HPA_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$v -o run -- python3 bench.py --cpu-baseline off --steps 10 "$@" > $out/$v.plog 2>&1 || exit $?
  python3 tools/kstats.py $out/$v/run_kernel_trace.csv | grep -v rocclr | head -8 | sed "s/^/$v /"
done
