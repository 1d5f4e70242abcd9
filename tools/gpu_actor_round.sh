#!/bin/bash
# the actor / explorer GPU tests, then tools/gpu_actor_prof.sh (config 4 and 5
# bench lines + kernel traces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_actor.py tests/test_gpu_explore.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/actor_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/actor_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_actor_prof.sh
