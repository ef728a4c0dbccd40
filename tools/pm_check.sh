mkdir -p gpurun_out/pm
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pm/t.log 2>&1; rc=$?; tail -3 gpurun_out/pm/t.log
case $rc in 124|134|137|139) exit $rc;; esac
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/pm/b_syn.log 2>&1 || exit $?
grep "^{" gpurun_out/pm/b_syn.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('synthetic', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 python bench.py --cpu-baseline off --prefill real > gpurun_out/pm/b_real.log 2>&1 || exit $?
grep "^{" gpurun_out/pm/b_real.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('real', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
