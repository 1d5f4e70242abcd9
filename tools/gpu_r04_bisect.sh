#!/bin/bash
# which earlier test of test_gpu_guard.py makes test_train_loop_names_the_actor_output fail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
G=tests/test_gpu_guard.py
T=$G::test_train_loop_names_the_actor_output
i=0
for pre in "$G::test_scan_finds_every_position" "$G::test_scan_many_tensors_one_bit_each" "$G::test_bn_reports_nonfinite_statistics" "$G::test_bn_reports_a_lost_partial" "$G::test_adam_reports_grad_and_param" "$G::test_update_names_the_batch[False]" "$G::test_update_names_the_batch[True]"; do
  i=$((i+1))
  timeout -k 10 300 python -u -m pytest "$pre" $T -m gpu -q -s --timeout 200 --timeout-method thread > gpurun_out/r04_bisect2_$i.log 2>&1
  rc=$?
  echo "[$pre] rc=$rc: $(tail -1 gpurun_out/r04_bisect2_$i.log)"; grep -E "NONFINITE" gpurun_out/r04_bisect2_$i.log | head -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
