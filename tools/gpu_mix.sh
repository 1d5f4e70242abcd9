#!/bin/bash
# the GPU tests touched by a change (TESTS), then tools/render_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_step.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/mix_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/mix_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/render_round.sh
