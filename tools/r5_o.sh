#!/bin/bash
# round 5: the layer tests on the product library (forms 2 / 4 skip) and on the A/B library (all forms)
set -u
o=gpurun_out/r5o; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py -q -rs --timeout 300 --timeout-method thread > $o/pytest_layer_product.txt 2>&1 || exit $?
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_ab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py -q -rs --timeout 300 --timeout-method thread > $o/pytest_layer_ab.txt 2>&1 || exit $?
