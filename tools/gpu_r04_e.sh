#!/bin/bash
# update-only timing + kernel stats (tools/update_only.py), micro conv timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/upd_micro.py > gpurun_out/upd_micro.txt 2>&1 || { tail -5 gpurun_out/upd_micro.txt; exit 1; }
grep -v Warn gpurun_out/upd_micro.txt | head -4
timeout -k 10 200 python tools/update_only.py > gpurun_out/update_only.txt 2>&1 || { tail -5 gpurun_out/update_only.txt; exit 1; }
grep update gpurun_out/update_only.txt
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 200 python tools/update_only.py > gpurun_out/update_only_rocblas.txt 2>&1 && echo "rocBLAS: $(grep update gpurun_out/update_only_rocblas.txt)"
rm -rf /tmp/prof_upd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_upd -o run --output-format csv -- python3 tools/update_only.py > gpurun_out/update_only_prof.log 2>&1 || { tail -20 gpurun_out/update_only_prof.log; exit 1; }
f=$(find /tmp/prof_upd -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r04_update_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r04_update_kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
n = 55.0
tot = sum(float(r['TotalDurationNs']) for r in rows) / n / 1e3
print('sum of kernel time per update: %.1f us' % tot)
for r in rows[:45]:
    print('%-72s %5.1f %8.1f us %8.1f us/upd' % (r['Name'][:72], int(r['Calls']) / n,
          float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / n / 1e3))
PY
