#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "" "SKIP_FIRST=1"; do
env $v timeout -k 10 120 python -u tools/nan_repro.py > gpurun_out/r04_repro2.log 2>&1; rc=$?
echo "== [$v] rc=$rc"; grep -v "Warn\|amdgpu.ids\|benchmark_limit" gpurun_out/r04_repro2.log | grep -v "^   \|^after" | tail -20
done
