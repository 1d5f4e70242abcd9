#!/bin/bash
# update tests, then tools/gpu_r04_e.sh (micro, update-only timing and kernel stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_upd_conv.py tests/test_gpu_trainer.py tests/test_gpu_train_ops.py tests/test_gpu_guard.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r04_updconv.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04_updconv.log)"; grep -E "FAILED|Error" gpurun_out/r04_updconv.log | head -5
[ $rc -eq 0 ] || exit $rc
tools/gpu_r04_e.sh
