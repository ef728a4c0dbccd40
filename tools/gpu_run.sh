#!/bin/bash
# GPU-box helper: tests, bench and a rocprofv3 kernel-stats profile, each step
# under its own time limit; stops at the first crash-like exit status.
# usage: tools/gpu_run.sh <tag> [tests|notests] [bench args...]
set -u
tag=${1:-run}; shift || true
mode=${1:-tests}; shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
crashed() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "$mode" = tests ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$out/pytest_gpu.log"
  if crashed $rc; then exit $rc; fi
fi
timeout -k 10 600 python bench.py "$@" > "$out/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' "$out/bench.log" | tail -1
if crashed $rc; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python bench.py "$@" --cpu-baseline off > "$out/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit 0
