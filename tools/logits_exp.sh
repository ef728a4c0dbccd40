#!/bin/bash
# Build timing-experiment variants of the resident logits kernel (HPA_RES_EXP
# 1: no MFMA, 2: no fold/stores, 3: weights re-read from L2) as separate
# libraries under tools/micro/exp/ (build container).  On the GPU box:
#   tools/logits_exp.sh run   -> rocprofv3 kernel traces per variant
set -eu
cd "$(dirname "$0")/.."
B=llm.c-paged_amd/build
if [ "${1:-build}" = build ]; then
  for e in 1 2 3; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Illm.c-paged_amd/csrc -DHPA_RES_EXP=$e \
      -c llm.c-paged_amd/csrc/hpa_logits.hip -o tools/micro/exp/hpa_logits_$e.o
    objs=$(ls $B/*.o | grep -v hpa_logits.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/micro/exp/libexp$e.so $objs tools/micro/exp/hpa_logits_$e.o
  done
  exit 0
fi
export TMPDIR=/tmp
mkdir -p gpurun_out/lexp
for e in 0 1 2 3; do
  lib=llm.c-paged_amd/libpaged_hip.so; [ $e = 0 ] || lib=tools/micro/exp/libexp$e.so
  HPA_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lexp/e$e -o run -- \
    python3 tools/gemm_one.py logits 4 1 4 1 64 20 > gpurun_out/lexp/e$e.log 2>&1
  python3 tools/kstats.py gpurun_out/lexp/e$e/run_kernel_trace.csv | grep "wg=1024" | sed "s/^/exp$e: /"
done
