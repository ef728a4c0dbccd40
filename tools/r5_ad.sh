#!/bin/bash
# round 5: why does XL chain form 8 overlap its weight stream with its MFMAs so poorly? stall counters
set -u
o=gpurun_out/r5ad; mkdir -p $o; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
P2="SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $o/p1 -o p1 -- python3 bench.py --model XL --page-size 32 --no-graph --cpu-baseline off --prof-steps 0 --steps 2 --warmup 1 > $o/p1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $o/p2 -o p2 -- python3 bench.py --model XL --page-size 32 --no-graph --cpu-baseline off --prof-steps 0 --steps 2 --warmup 1 > $o/p2.log 2>&1 || exit $?
