#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over one
# fused-GEMM configuration.  usage: tools/pmc_one.sh outdir "gemm_one args" "CTR CTR ..." ["CTR ..."] ...
set -u
out=$1; cfg=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$out/p$i" -o run -- \
    python3 tools/gemm_one.py $cfg > "$out/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  python3 - "$out/p$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for x in csv.DictReader(open(sys.argv[1])):
    if 'hpa_gemm' in x['Kernel_Name']:
        agg[x['Counter_Name']].append(float(x['Counter_Value']))
print({k: round(sum(v) / len(v), 1) for k, v in agg.items()})
PY
done
