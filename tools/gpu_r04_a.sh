#!/bin/bash
# round 4: the update-conv kernels' tests first, then the full GPU suite twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_upd_conv.py -v --timeout 120 --timeout-method thread > gpurun_out/r04_updconv.log 2>&1
rc=$?
echo "updconv rc=$rc: $(tail -1 gpurun_out/r04_updconv.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
tools/gpu_suite_repeat.sh 2 r04_suite
