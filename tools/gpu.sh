#!/bin/bash
# tools/gpu.sh -- the one driver for GPU-box runs (replaces the round-4/5
# one-off r4_*/r5_*/final_* scripts).  Every step runs under its own time
# limit and the run stops at the first failing step (no retries).
#
#   usage: tools/gpu.sh <tag> <step> [<step> ...]      (output: gpurun_out/<tag>/)
#
# steps (CFG = c2 | c5 | c5kv | xl | b8 | b16 | b32 | e2 | e4 | e8 | w2 | prefill | sample):
#   smoke              __graft_entry__.smoke()
#   suite[:K]          pytest -m gpu (K: a -k expression)
#   build              make the library in-tree (normally built before the call)
#   bench:CFG          python bench.py <CFG args>            -> bench_CFG.txt (+ .json line)
#   kstats:CFG         rocprofv3 --kernel-trace --stats of the bench command (spin-up on)
#                      -> prof_CFG/ + kstats_CFG.txt (per-kernel averages)
#   pmc:CFG            FETCH_SIZE / WRITE_SIZE, separate --pmc passes -> pmc_CFG/traffic.txt
#   mfma:CFG           SQ_INSTS_MFMA / SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE -> mfma_CFG/
#   trace:B[:MODE[:X]] per-workgroup phase trace of the chain (tools/pl_trace.py B 990 MODE X on the
#                      prebuilt -DHPA_LAYER_TRACE library llm.c-paged_amd/libpl_trace.so)
#   ab:NAME:FLAGS:CFG  A/B library (make BUILD=build_NAME LIB=libpl_NAME.so XFLAGS="FLAGS"),
#                      bench CFG on it -> bench_CFG_NAME.txt
#   lib:NAME:CFG       bench CFG on a prebuilt library (NAME "prod" = libpaged_hip.so,
#                      else llm.c-paged_amd/libpl_NAME.so), no CPU baseline -> bench_CFG_NAME_<n>.txt
#   py:NAME:ARGS       python -u ARGS (a tools/ probe)         -> NAME.txt
#   exe:NAME:ARGS      a built probe binary                    -> NAME.txt
#   rocexe:NAME:ARGS   the same under rocprofv3 --kernel-trace --stats -> NAME.txt
set -u
tag=$1; shift
o=gpurun_out/$tag; mkdir -p "$o"; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16"
cfg_args() {
  case $1 in
    c2) echo "" ;;
    c5) echo "$C5" ;;
    c5kv) echo "--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16" ;;
    xl) echo "--model XL --page-size 32 --steps 10 --warmup 2" ;;
    b8|b16|b32) echo "--batch ${1#b}" ;;
    e2|e4|e8) echo "--emulate-rank ${1#e}" ;;
    w2) echo "--emulate-rank 2 --scaling weak" ;;
    prefill) echo "--prefill real" ;;
    sample) echo "--sample" ;;
    *) echo "BAD_CFG_$1" ;;
  esac
}
run() {  # name, seconds, command...
  local name=$1 lim=$2; shift 2
  echo "[gpu.sh] $(date +%T) $name: $*"
  timeout -k 10 "$lim" "$@" > "$o/$name.txt" 2>&1
  local rc=$?
  echo "[gpu.sh] $(date +%T) $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -25 "$o/$name.txt"; exit $rc; fi
}
for st in "$@"; do
  IFS=: read -r kind a b c <<< "$st"
  case $kind in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    build) run build 600 make -s -C llm.c-paged_amd -j16 ;;
    suite)
      if [ -n "${a:-}" ]; then
        run "suite_${a//[^A-Za-z0-9]/_}" 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$a"
      else
        run suite 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
      fi ;;
    bench)
      run "bench_$a" 600 python -u bench.py $(cfg_args "$a")
      grep "^{" "$o/bench_$a.txt" > "$o/bench_$a.json" || true ;;
    kstats)
      run "kstats_run_$a" 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$o/prof_$a" -o run -- \
        python3 bench.py --cpu-baseline off $(cfg_args "$a")
      python3 tools/kstats.py "$o/prof_$a/run_kernel_trace.csv" 0 > "$o/kstats_$a.txt" ;;
    pmc)  # per-dispatch csvs dropped after the summary (traffic.txt / traffic.json): gpurun_out stays small
      run "pmc_$a" 900 bash tools/pmc_traffic.sh "$o/pmc_$a" --steps 6 --warmup 2 --spinup 0 $(cfg_args "$a")
      rm -rf "$o/pmc_$a/FETCH_SIZE" "$o/pmc_$a/WRITE_SIZE" ;;
    mfma)
      run "mfma_$a" 600 bash tools/pmc_mfma.sh "$o/mfma_$a" --steps 6 --warmup 2 --spinup 0 $(cfg_args "$a")
      rm -rf "$o/mfma_$a/pmc" ;;
    trace)  # trace:B[:MODE[:XL|b16]] on llm.c-paged_amd/libpl_trace.so (make BUILD=build_trace LIB=libpl_trace.so XFLAGS=-DHPA_LAYER_TRACE)
      HPA_LIB=llm.c-paged_amd/libpl_trace.so run "trace_${a}_${b:-5}${c:-}" 600 python -u tools/pl_trace.py "$a" 990 "${b:-5}" ${c:-} ;;
    ab)
      run "build_ab_$a" 900 make -s -C llm.c-paged_amd -j16 BUILD="build_$a" LIB="libpl_$a.so" XFLAGS="$b"
      HPA_LIB="llm.c-paged_amd/libpl_$a.so" run "bench_${c}_$a" 600 python -u bench.py --cpu-baseline off $(cfg_args "$c") ;;
    lib)
      lf=llm.c-paged_amd/libpl_$a.so; [ "$a" = prod ] && lf=llm.c-paged_amd/libpaged_hip.so
      n=1; while [ -e "$o/bench_${b}_${a}_$n.txt" ]; do n=$((n+1)); done
      HPA_LIB="$lf" run "bench_${b}_${a}_$n" 600 python -u bench.py --cpu-baseline off $(cfg_args "$b")
      grep -h '"ms_per_step"' "$o/bench_${b}_${a}_$n.txt" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[gpu.sh] $a $b', d['ms_per_step'], d['value'])" ;;
    py) run "$a" 600 python -u $b ;;
    exe) run "$a" 600 $b ;;
    rocexe)  # the trace database stays on the box (/tmp): only the log comes back
      run "$a" 600 rocprofv3 --kernel-trace --stats -d "/tmp/prof_$a" -o run -- $b ;;
    *) echo "[gpu.sh] unknown step $st"; exit 2 ;;
  esac
done
echo "[gpu.sh] all steps done"
