#!/bin/bash
# config-5 pieces: replay / trainer / actor GPU tests, per-phase times of a
# TrainLoop decision (tools/train_phases.py), then the config 4 / 5 bench lines
# and kernel traces (tools/gpu_actor_prof.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_replay.py tests/test_gpu_trainer.py tests/test_gpu_actor.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/train_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/train_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/train_phases.py > gpurun_out/train_phases.txt 2>&1 || { tail -20 gpurun_out/train_phases.txt; exit 1; }
cat gpurun_out/train_phases.txt
bash tools/gpu_actor_prof.sh
