#!/bin/bash
# driver-form bench with the default warm-up and with 30 warm-up decisions
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in 10 30 10 30; do
  timeout -k 10 400 python bench.py --warmup $w > gpurun_out/r04_warm_$w.log 2>&1 || exit $?
  python - "$w" <<'PY'
import json, sys
for line in open('gpurun_out/r04_warm_%s.log' % sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line); r = d['roofline']
        print('warmup %s: %.2fM render %.4f ms frac %.3f' % (sys.argv[1], d['value'] / 1e6, r['avg_kernel_ms'], r['frac']))
PY
done
