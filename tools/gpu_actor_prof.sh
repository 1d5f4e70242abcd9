#!/bin/bash
# config 4 (actor in the loop) and config 5 (train): plain bench lines + kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in actor train; do
  timeout -k 10 400 python bench.py --config $cfg --steps 30 --warmup 10 --cpu-steps 0 > gpurun_out/ap_$cfg.json 2> gpurun_out/ap_$cfg.err || { tail -20 gpurun_out/ap_$cfg.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ap_$cfg.json')); print('$cfg', 'value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'actor ms %.3f' % d['roofline']['avg_kernel_ms'], 'frac %.3f' % d['roofline']['frac'])"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ap_trace_$cfg -o run -- python3 bench.py --config $cfg --steps 30 --warmup 10 --cpu-steps 0 > gpurun_out/ap_trace_$cfg.log 2>&1 || { tail -20 gpurun_out/ap_trace_$cfg.log; exit 1; }
  f=$(find gpurun_out/ap_trace_$cfg -name '*kernel_stats.csv' | head -1)
  python -c "
import csv
rows = list(csv.DictReader(open('$f')))
for r in rows[:18]: print('%-90s %6s %10.1f us' % (r['Name'][:90], r['Calls'], float(r['AverageNs'])/1e3))"
done
