#!/bin/bash
# round 5: the two-launch layer (K1 = qkv | attention | attproj, K2 = fc -> fcproj):
# parity, A/B against the attention+attproj form (k0) and round 4's (ap0), traces
set -u
o=gpurun_out/r5d; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_decode.py tests/test_gpu_multi_rank.py tests/test_gpu_configs.py -x -v -s --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
ab() {  # variant batch round
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $1 != base ] && lib=$PWD/llm.c-paged_amd/libpl_$1.so
  HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $2 --steps 60 --warmup 5 --cpu-baseline off --prof-steps 0 --spinup 1 > $o/ab_$1_b$2_$3.txt 2>&1
}
for r in 1 2; do
  for B in 64 8 16 32; do for v in base k0 ap0; do ab $v $B $r || exit $?; done; done
done
for f in $o/ab_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"; done | tee $o/ab_summary.txt
for B in 8 64; do
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 5 > $o/trace_b$B.txt 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/prof_c2.log 2>&1 || exit $?
python3 tools/kstats.py $o/prof_c2/run_kernel_trace.csv > $o/kstats_c2.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_b8 -o run -- python3 bench.py --batch 8 --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/prof_b8.log 2>&1 || exit $?
python3 tools/kstats.py $o/prof_b8/run_kernel_trace.csv > $o/kstats_b8.txt 2>&1
