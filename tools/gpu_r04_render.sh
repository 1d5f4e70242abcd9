#!/bin/bash
# render change: its GPU tests, then two plain config-3 bench runs (parity on)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_dropin.py tests/test_gpu_scale.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r04_render_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04_render_tests.log)"; grep -E "FAILED|Error" gpurun_out/r04_render_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config render --steps 100 --warmup 20 --cpu-steps 0 --no-lane --no-sub > gpurun_out/r04_render_bench_$i.log 2>&1 || exit $?
  python - "$i" <<'PY'
import json, sys
for line in open('gpurun_out/r04_render_bench_%s.log' % sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line)
        r = d['roofline']
        print('value %.2fM render %.4f ms frac %.3f parity %s' % (d['value'] / 1e6, r['avg_kernel_ms'], r['frac'], d['parity']['ok']))
PY
done
