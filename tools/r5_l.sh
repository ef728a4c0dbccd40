#!/bin/bash
# round 5: PMC passes on the bf16 logits (A-resident, 8 waves, 4 row blocks) in isolation
set -u
o=gpurun_out/r5l; mkdir -p $o; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $o/p1 -o p1 -- python3 tools/b16_logits.py 256 5 5 8 4 > $o/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $o/p2 -o p2 -- python3 tools/b16_logits.py 256 5 5 8 4 > $o/p2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d $o/p3 -o p3 -- python3 tools/b16_logits.py 256 5 5 8 4 > $o/p3.log 2>&1 || exit $?
