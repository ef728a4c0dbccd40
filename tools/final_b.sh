# round-end evidence, part b: profile_round.sh b (configs 5 and 3, prefill, sampling)
set -u
mkdir -p gpurun_out/final
bash tools/profile_round.sh gpurun_out/final b
