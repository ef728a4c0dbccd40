#!/bin/bash
# GPU-box helper: tests, bench and a rocprofv3 kernel-stats profile, each step
# under its own time limit; stops at the first crash-like exit status.
# usage: tools/gpu_run.sh <tag> [tests|notests] [bench args...]
#   PYTEST_K="expr"  selects tests (-k); ATTN_SCAN=1 runs tools/attn_scan.py first
set -u
tag=${1:-run}; shift || true
mode=${1:-tests}; shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "${ATTN_SCAN:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/attn_scan.py > "$out/attn_scan.txt" 2>&1
  rc=$?; echo "attn_scan rc=$rc"; cat "$out/attn_scan.txt" | tail -20
  if crashed $rc; then exit $rc; fi
fi
if [ "$mode" = tests ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=10 -rP --timeout 240 --timeout-method thread \
    -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > "$out/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$out/pytest_gpu.log" | tail -15
  if crashed $rc; then exit $rc; fi
fi
timeout -k 10 600 python bench.py "$@" > "$out/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' "$out/bench.log" | tail -1
if crashed $rc; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python bench.py "$@" --cpu-baseline off > "$out/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit 0
