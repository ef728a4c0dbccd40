#!/bin/bash
# selected GPU tests, then A/B bench lines (each argument after the selection is a bench flag set)
set -u
sel=$1; shift
out=gpurun_out/tab; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $sel -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/t.log; [ $rc = 0 ] || exit $rc
[ $# -gt 0 ] && bash tools/diag/ab.sh "$@"
exit 0
