#!/bin/bash
# Diagnostic: render-kernel time per workgroup size (DTSIM_RENDER_THREADS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${THREADS:-512 640 768 896 1024}; do
  DTSIM_RENDER_THREADS=$t timeout -k 10 120 python bench.py --config render --steps 100 --warmup 10 --cpu-steps 0 > gpurun_out/thr_$t.json 2>/dev/null || exit $?
  python - "$t" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/thr_%s.json' % sys.argv[1]) if l.startswith('{')][-1])
print('threads=%s render_ms=%.4f' % (sys.argv[1], d['roofline']['avg_kernel_ms']))
PY
done
