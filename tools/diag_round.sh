#!/bin/bash
# Diagnostics on the GPU box: step_fan_kernel and render_kernel shader-clock
# stamps (the -DDTSIM_STAMPS library, built beforehand by tools/step_stamps.sh)
# and render_kernel SQ counters.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
LIB=$PWD/aido1_amd/libdtsim_stamps.so
if [ -z "$NO_STAMPS" ]; then
  DTSIM_DIAG_LIB=$LIB timeout -k 10 120 python tools/render_stamps.py > gpurun_out/render_stamps.log 2>&1 || exit 1
  cat gpurun_out/render_stamps.log
  DTSIM_DIAG_LIB=$LIB timeout -k 10 120 python tools/fan_stamps.py > gpurun_out/fan_stamps.log 2>&1 || exit 1
  cat gpurun_out/fan_stamps.log
fi
if [ -n "$RPMC" ]; then
  bash tools/render_pmc.sh > gpurun_out/render_pmc.log 2>&1 || exit 1
  cat gpurun_out/render_pmc.log
fi
