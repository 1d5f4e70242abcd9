#!/bin/bash
# Run the GPU test suite up to N times in fresh processes (one at a time);
# stop at once on anything but pass (0) or ordinary test failures (1).
# usage: tools/gpu_suite_repeat.sh N TAG [pytest args...]
n=$1; tag=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 "$n"); do
  timeout -k 10 420 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread "$@" \
    > "gpurun_out/${tag}_$i.log" 2>&1
  rc=$?
  echo "run $i rc=$rc: $(tail -1 gpurun_out/${tag}_$i.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
