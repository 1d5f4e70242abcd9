#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_explore.py tests/test_gpu_actor.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mix_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/mix_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/render_round.sh
