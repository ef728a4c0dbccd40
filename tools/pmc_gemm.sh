#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over
# single GEMM configurations.  usage: tools/pmc_gemm.sh outdir "shape waves row_blocks variant col_tiles" ...
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
rocprofv3 -L > "$out/counters.txt" 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="TCC_HIT_sum TCC_MISS_sum"
P4="SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES"
i=0
for cfg in "$@"; do
  i=$((i+1))
  for p in 1 2 3 4; do
    eval "ctrs=\$P$p"
    timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$out/c${i}_p$p" -o run -- \
      python3 tools/gemm_one.py $cfg > "$out/c${i}_p$p.log" 2>&1
    rc=$?; echo "cfg $i ($cfg) pass $p rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
