#!/bin/bash
# the driver's default bench command on the final tree (N = 1, defaults incl. the 2 s spin-up and CPU baseline)
set -u
o=gpurun_out/r4bd; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $o/bench_default.log 2>&1 || exit $?
grep "^{" $o/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['spinup_s'], d['roofline']['frac'], d['status'])"
