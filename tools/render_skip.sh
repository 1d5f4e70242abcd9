#!/bin/bash
# Diagnostic: render_kernel time with phases skipped (DTSIM_RENDER_SKIP bits:
# 1 background, 2 markings, 4 uniformity+grey, 8 Sobel/NMS/hysteresis,
# 16 hysteresis, 32 masks); outputs are invalid when a bit is set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sk in ${SKIPS:-0 1 2 4 8 32 3 12 40}; do
  DTSIM_RENDER_SKIP=$sk timeout -k 10 120 python bench.py --steps 60 --warmup 5 --cpu-steps 0 --no-parity > gpurun_out/skip_$sk.json 2>/dev/null || exit $?
  python - "$sk" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/skip_%s.json' % sys.argv[1]) if l.startswith('{')][-1])
print('skip=%-3s render_ms=%.4f min %.4f' % (sys.argv[1], d['render']['avg_kernel_ms'], d['render']['min_kernel_ms']))
PY
done
