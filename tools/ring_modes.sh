# ring GEMM diagnostic modes (hpa_gemm_ring.hip MODE), one process each, on
# the diagnostic build (the product library has no such modes):
#   make -C llm.c-paged_amd BUILD=$PWD/llm.c-paged_amd/build_rd \
#        LIB=$PWD/llm.c-paged_amd/libpaged_hip_ringdiag.so XFLAGS=-DHPA_RING_DIAG
set -u
o=gpurun_out/ringm; mkdir -p $o
lib=$PWD/llm.c-paged_amd/libpaged_hip_ringdiag.so
for m in 0 2 3 4 1; do
  HPA_LIB=$lib HPA_RING_MODE=$m timeout -k 10 120 python -u tools/ring_tune.py > $o/mode$m.txt 2>&1 || exit $?
done
grep -h "HPA_RING_MODE\|^qkv\|^fc " $o/mode*.txt
