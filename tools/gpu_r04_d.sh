#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_upd_conv.py tests/test_gpu_trainer.py tests/test_gpu_train_ops.py tests/test_gpu_guard.py -q --timeout 120 --timeout-method thread > gpurun_out/r04_updconv.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04_updconv.log)"; grep FAILED gpurun_out/r04_updconv.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/train_phases.py > gpurun_out/r04_train_phases.txt 2>&1; grep -v "Warn\|amdgpu\|benchmark" gpurun_out/r04_train_phases.txt | tail -7
tools/gpu_r04_prof.sh 2>&1 | grep -i "wgrad\|fwd_kernel\|dgrad\|bn_\|reduce" | head -20
