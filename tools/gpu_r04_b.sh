#!/bin/bash
# round 4 measurements: config-5 phases, the default bench line (configs 3 + 2,
# 4, 5 sub-records), a kernel trace of config 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/train_phases.py > gpurun_out/r04_train_phases.txt 2>&1 || { tail -20 gpurun_out/r04_train_phases.txt; exit 1; }
grep -v Warning gpurun_out/r04_train_phases.txt | tail -8
timeout -k 10 400 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { tail -30 gpurun_out/r04_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04_bench.json'))
print('c3 value %.4g ms/step %.4f render %.4f frac %.3f parity %s' % (d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['roofline']['frac'], d['parity']['ok']))
for k in ('config2', 'config4', 'config5'):
    c = d.get(k)
    if c: print(k, 'value %.4g ms/step %.4f' % (c['value'], c['ms_per_step']), json.dumps(c.get('parity'))[:400])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_train -o run -- python3 bench.py --config train --steps 20 --warmup 5 --no-parity > gpurun_out/r04_prof_train.log 2>&1 || { tail -20 gpurun_out/r04_prof_train.log; exit 1; }
echo prof done
