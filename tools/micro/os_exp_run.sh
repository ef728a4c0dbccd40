#!/bin/bash
# rocprofv3 kernel durations of the one-shot GEMM ablations (os_exp.sh)
set -u
export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/osexp; mkdir -p $out
cd /tmp
for e in 0 1 2 3 4; do
  timeout -k 5 90 rocprofv3 --kernel-trace -d $out/e$e -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/micro/os_exp$e > $out/e$e.log 2>&1 || { echo "fail $e"; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, os
names = ['qkv', 'attproj', 'fc', 'fcproj'] * 2
out = os.path.join(os.environ['GRAFT_REPO_ROOT'], 'gpurun_out/osexp')
lab = {0: 'baseline', 1: 'no LN', 2: 'no MFMA', 3: 'L2-resident operands', 4: 'no epilogue'}
for e in range(5):
    rows = list(csv.DictReader(open(f'{out}/e{e}/run_kernel_trace.csv')))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ks = [r for r in rows if 'os_kernel' in r['Kernel_Name']]
    res = []
    for i in range(8):
        d = sorted((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in ks[i * 30:(i + 1) * 30][5:])
        res.append('%s%s %.2f' % (names[i], '(c)' if i >= 4 else '', d[len(d) // 2]))
    print('%-22s' % lab[e], ' '.join(res))
PY
