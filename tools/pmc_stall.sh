#!/bin/bash
# stall breakdown of ONE fused-GEMM launch shape (tools/gemm_one.py):
# lists the SQ counters gfx950 offers, then one --pmc pass (<= 8 SQ counters)
# usage: tools/pmc_stall.sh <outdir> <gemm_one args...>
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || true
want="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"
have=""
for c in $want; do grep -qw "$c" "$out/avail.txt" && have="$have $c"; done
echo "counters:$have"
[ -n "$have" ] || exit 0
timeout -s KILL 90 rocprofv3 --pmc $have --kernel-trace --output-format csv -d "$out/pmc" -o run -- \
  python3 tools/gemm_one.py "$@" > "$out/run.log" 2>&1
rc=$?; echo "pmc rc=$rc"
exit $rc
