#!/bin/bash
# kernel time of one kernel family under alternative builds of the library
# (HPA_LIB): rocprofv3 kernel-trace of a short bench per build.
# usage: tools/lib_ab.sh <tag> <kernel-substring> <lib.so>... [-- bench args]
set -u
tag=$1; pat=$2; shift 2
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for lib in "${libs[@]}"; do
  n=$(basename $lib .so)
  HPA_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/$n -o run -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 "$@" > $out/$n.log 2>&1 || exit $?
  python3 tools/kstats.py $out/$n/run_kernel_trace.csv | grep -- "$pat" | sed "s/^/$n /"
  HPA_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cpu-baseline off "$@" > $out/$n.bench 2>&1 || exit $?
  grep "^{" $out/$n.bench | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n ms/step', d['ms_per_step'])"
done
