#!/bin/bash
# page-group A/B: attention time of configs 2 and 5 per library build
set -u
out=gpurun_out/abpg; mkdir -p $out
for lib in llm.c-paged_amd/libpaged_hip.so tools/micro/exp/libpg4.so tools/micro/exp/libpg16.so; do
  n=$(basename $lib .so)
  for cfg in "c2|" "c5|--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16" "c2real|--prefill real"; do
    tag=${cfg%%|*}; args=${cfg#*|}
    HPA_LIB=$PWD/$lib timeout -k 10 300 python bench.py --cpu-baseline off $args > $out/$n.$tag.log 2>&1 || exit $?
    grep "^{" $out/$n.$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n $tag', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
