#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
POISON=1 timeout -k 10 240 python -u tools/nan_hunt.py > gpurun_out/r04_hunt_p128.log 2>&1; echo "hunt128 rc=$?"; grep -v Warn gpurun_out/r04_hunt_p128.log | tail -30
POISON=1 ENVS=4096 REPS=20 timeout -k 10 240 python -u tools/nan_hunt.py > gpurun_out/r04_hunt_p4096.log 2>&1; echo "hunt4096 rc=$?"; grep -v Warn gpurun_out/r04_hunt_p4096.log | tail -30
