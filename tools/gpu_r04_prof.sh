#!/bin/bash
# kernel statistics of config 5 (stats kept, the full trace dropped)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf /tmp/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_train -o run --output-format csv -- python3 bench.py --config train --steps 20 --warmup 5 --no-parity > gpurun_out/r04_prof_train.log 2>&1 || { tail -20 gpurun_out/r04_prof_train.log; exit 1; }
f=$(find /tmp/prof_train -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r04_train_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r04_train_kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:40]:
    print('%-70s %6s %9.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3))
PY
