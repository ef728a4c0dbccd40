#!/bin/bash
# the final tree's libraries: smoke(), the layer / fused tests, the default bench
set -u
o=gpurun_out/r4fs; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.txt 2>&1 || exit $?
tail -1 $o/smoke.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_fused.py tests/test_gpu_decode.py -q --maxfail=3 \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.txt 2>&1 || exit $?
tail -1 $o/pytest.txt
timeout -k 10 300 python -u bench.py --cpu-baseline off > $o/bench.log 2>&1 || exit $?
grep "^{" $o/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['status'])"
