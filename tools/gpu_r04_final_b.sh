#!/bin/bash
# the full GPU suite twice in fresh processes, then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/gpu_suite_repeat.sh 2 r04_suite || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/r04_smoke.log)"; exit $rc
