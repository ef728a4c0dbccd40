#!/bin/bash
# The round's evidence on one GPU box: bench lines of every single-GPU
# BASELINE config, the rocprofv3 kernel stats of the headline bench command,
# PMC traffic (configs 2 and 5), MFMA utilisation (configs 2 and 3, prefill),
# the attention batch scan, prefill and sampling lines.
# usage: tools/profile_round.sh <outdir> [a|b]   (then copy into profiles/rNN/)
#   a: config 2 (bench, kernel stats, PMC traffic, MFMA), attention scan,
#      small-batch bench lines; b: configs 5 and 3, prefill, sampling
#   (each part fits one gpurun call); no part: both
set -u
out=$1; part=${2:-ab}; mkdir -p "$out"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  case $rc in 0) ;; *) tail -5 "$out/$name.log"; exit $rc;; esac
}
if [[ $part == *a* ]]; then
step bench_c2 400 python bench.py
grep "^{" "$out/bench_c2.log" > "$out/bench_line.json"
step prof_c2 400 rocprofv3 --kernel-trace --stats -d "$out/prof_c2" -o run --output-format csv -- \
  python3 bench.py --cpu-baseline off
python3 tools/kstats.py "$out/prof_c2/run_kernel_trace.csv" 32 > "$out/kstats_c2.txt"
step pmc_c2 900 bash tools/pmc_traffic.sh "$out/pmc_c2" --steps 8 --warmup 2
step mfma_c2 400 bash tools/pmc_mfma.sh "$out/mfma_c2" --steps 6 --warmup 2
step attn_scan 300 python tools/attn_scan_r3.py
for b in 8 16 32; do
  step bench_b$b 300 python bench.py --batch $b --cpu-baseline off
done
step prof_b8 300 rocprofv3 --kernel-trace --stats -d "$out/prof_b8" -o run --output-format csv -- \
  python3 bench.py --batch 8 --cpu-baseline off
python3 tools/kstats.py "$out/prof_b8/run_kernel_trace.csv" 32 > "$out/kstats_b8.txt"
fi
if [[ $part == *b* ]]; then
step bench_c5 500 python bench.py --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16
step prof_c5w 500 rocprofv3 --kernel-trace --stats -d "$out/prof_c5w" -o run --output-format csv -- \
  python3 bench.py --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off
step pmc_c5 900 bash tools/pmc_traffic.sh "$out/pmc_c5" --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 \
  --w-dtype bf16 --steps 4 --warmup 1
step bench_c5kv 500 python bench.py --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --cpu-baseline off
step bench_xl 600 python bench.py --model XL --page-size 32 --cpu-baseline off
step prof_xl 600 rocprofv3 --kernel-trace --stats -d "$out/prof_xl" -o run --output-format csv -- \
  python3 bench.py --model XL --page-size 32 --cpu-baseline off --steps 8
step mfma_xl 600 bash tools/pmc_mfma.sh "$out/mfma_xl" --model XL --page-size 32 --steps 3 --warmup 1
step bench_prefill 400 python bench.py --prefill real --cpu-baseline off
step mfma_prefill 600 bash tools/pmc_mfma.sh "$out/mfma_prefill" --prefill real --steps 3 --warmup 1
step bench_sample 400 python bench.py --sample --cpu-baseline off
python3 tools/kstats.py "$out/prof_c5w/run_kernel_trace.csv" 32 > "$out/kstats_c5w.txt"
python3 tools/kstats.py "$out/prof_xl/run_kernel_trace.csv" 8 > "$out/kstats_xl.txt"
fi
echo done
