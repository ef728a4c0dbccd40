#!/bin/bash
# round-4 evidence refresh on the final tree (config 2 profile + emulated ranks), then the attention A/B
set -u
bash tools/final_r4_c.sh || exit $?
bash tools/r4_attn_ab.sh
