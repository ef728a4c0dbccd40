#!/bin/bash
# builds the one-shot GEMM timing tool once per HPA_OS_EXP experiment
# (0 baseline, 1 no LN, 2 no MFMA, 3 L2-resident operands, 4 no epilogue)
set -e
for e in 0 1 2 3 4; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNO_TS -DHPA_OS_EXP=$e -I include -I llm.c-paged_amd/csrc \
    tools/micro/os_trace.hip -o tools/micro/os_exp$e
done
