#!/bin/bash
# Quick loop for the step kernels: parity tests of test_gpu_step.py, the
# config-2 bench line (driver args and default), and the fan-kernel stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -x -q -m gpu --timeout 200 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_step.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_step.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-steps 0 --no-render $BENCH_ARGS > gpurun_out/bench_fan.log 2>&1 && timeout -k 10 200 python bench.py --cpu-steps 0 --no-render --no-parity $BENCH_ARGS >> gpurun_out/bench_fan.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-steps 0 --no-render $BENCH_ARGS >> gpurun_out/bench_fan.log 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open('gpurun_out/bench_fan.log'):
    if l.startswith('{'):
        d = json.loads(l); d["parity"] = d.get("parity") or {"ok": None}
        print('value %.3fG steps %d us/decision %.3f parity %s kernel ms %.4f' % (
            d['value'] / 1e9, d['steps'], d['step_ms_per_decision'] * 1e3, d['parity']['ok'],
            d['roofline']['avg_kernel_ms']))
PY
if [ -f aido1_amd/libdtsim_stamps.so ]; then
  DTSIM_DIAG_LIB=$PWD/aido1_amd/libdtsim_stamps.so timeout -k 10 120 python tools/fan_stamps.py
fi
