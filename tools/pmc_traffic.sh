#!/bin/bash
# HBM traffic of every kernel of the bench command, per the MI355X guide's
# HBM/rocprofv3 recipe: FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc passes
# (kernel-trace only, no runtime/sys trace), eager launches (--no-graph) so
# every dispatch is counted.  usage: tools/pmc_traffic.sh <outdir> [bench args]
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$out/$ctr" -o run -- \
    python3 bench.py --no-graph --cpu-baseline off --prof-steps 0 "$@" > "$out/$ctr.log" 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 tools/pmc_traffic.py "$out" > "$out/traffic.txt" && cat "$out/traffic.txt"
