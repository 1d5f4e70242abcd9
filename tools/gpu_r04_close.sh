#!/bin/bash
# round close: the full GPU suite, smoke(), then the driver-form bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_suite_repeat.sh 1 r04_close_suite || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/r04_smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r04_close_bench.log 2>&1 || exit $?
python - <<'PY'
import json
for line in open('gpurun_out/r04_close_bench.log'):
    if line.startswith('{'):
        d = json.loads(line); r = d['roofline']
        print('headline %.2fM render %.4f ms frac %.3f parity %s | c4 %.2fM | c5 %.2fM update %.2f ms' % (
            d['value'] / 1e6, r['avg_kernel_ms'], r['frac'], d['parity']['ok'],
            d['config4']['value'] / 1e6, d['config5']['value'] / 1e6,
            d['config5']['phases_ms']['update']))
PY
