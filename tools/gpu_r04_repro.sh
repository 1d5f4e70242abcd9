#!/bin/bash
# the suite's files up to test_gpu_guard in one process, three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_actor.py tests/test_gpu_distributed.py tests/test_gpu_dropin.py tests/test_gpu_env_server.py tests/test_gpu_explore.py tests/test_gpu_guard.py tests/test_gpu_trainer.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/r04_repro_$i.log 2>&1
  rc=$?
  echo "repro $i rc=$rc: $(tail -1 gpurun_out/r04_repro_$i.log)"; grep -E "NONFINITE|FAILED" gpurun_out/r04_repro_$i.log | head -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
