#!/bin/bash
# round 5: bf16 logits microbenchmark (launch shapes, warm / cold weights), then the whole GPU suite
set -u
o=gpurun_out/r5j; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/b16_logits.py 256 10 > $o/b16_logits.txt 2>&1 || exit $?
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || exit $?
