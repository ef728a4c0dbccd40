# ring GEMM diagnostic modes (hpa_gemm_ring.hip MODE), one process each
set -u
o=gpurun_out/ringm; mkdir -p $o
for m in 0 2 3 4 1; do
  HPA_RING_MODE=$m timeout -k 10 120 python -u tools/ring_tune.py > $o/mode$m.txt 2>&1 || exit $?
done
grep -h "HPA_RING_MODE\|^qkv\|^fc " $o/mode*.txt
