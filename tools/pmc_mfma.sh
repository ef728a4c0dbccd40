#!/bin/bash
# MFMA utilisation of every kernel of a bench command (SURVEY.md 8a / north
# star: "rocprof ... MFMA utilisation against gfx950 peak"): one --pmc pass
# (kernel-trace only, eager launches so every dispatch is counted) with
#   SQ_INSTS_MFMA             MFMA instructions issued
#   SQ_VALU_MFMA_BUSY_CYCLES  matrix-pipe busy cycles (summed over SIMDs)
#   SQ_BUSY_CU_CYCLES         CU-busy quad-cycles (summed over CUs)
#   SQ_WAVE_CYCLES            wave-resident quad-cycles
#   GRBM_GUI_ACTIVE           GPU-active cycles, summed over the 8 XCDs
# then tools/pmc_mfma.py.  usage: tools/pmc_mfma.sh <outdir> [bench args]
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d "$out/pmc" -o run -- \
  python3 bench.py --no-graph --cpu-baseline off --prof-steps 0 "$@" > "$out/bench.log" 2>&1
rc=$?; echo "pmc rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
python3 tools/pmc_mfma.py "$out" > "$out/mfma.txt" && cat "$out/mfma.txt"
