set -u
out=gpurun_out/sp4; mkdir -p $out
for n in 112 128 144 160 176; do
  timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 --split $n > $out/b_$n.log 2>&1 || { echo "fail $n"; tail -3 $out/b_$n.log; exit 1; }
  grep "^{" $out/b_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('split', $n, 'ms/step', d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --cpu-baseline off --prof-steps 0 --no-graph > $out/b_ng.log 2>&1 && grep "^{" $out/b_ng.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nograph ms/step', d['ms_per_step'])"
