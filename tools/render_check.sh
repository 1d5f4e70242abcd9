#!/bin/bash
# Quick loop for render_kernel: parity tests, the bench's render sub-record,
# and the phase stamps (libdtsim_stamps.so built beforehand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q -m gpu --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_render.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_render.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --cpu-steps 0 > gpurun_out/bench_render.log 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open('gpurun_out/bench_render.log'):
    if l.startswith('{'):
        r = json.loads(l)['render']
        print('render avg %.4f ms min %.4f frac %.3f parity %s' % (r['avg_kernel_ms'], r['min_kernel_ms'], r['frac'], r.get('parity')))
PY
if [ -f aido1_amd/libdtsim_stamps.so ]; then
  DTSIM_DIAG_LIB=$PWD/aido1_amd/libdtsim_stamps.so timeout -k 10 120 python tools/render_stamps.py
fi
