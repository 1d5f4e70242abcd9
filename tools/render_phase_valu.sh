#!/bin/bash
# VALU instructions of render_kernel by phase: SQ_INSTS_VALU / SQ_INSTS_LDS /
# SQ_INSTS_SALU per dispatch of builds that stop after phase group k
# (DTSIM_RENDER_STOP_AT, dtrender.hip), config-3 bench without parity.
# Build the libraries on the CPU first: python tools/render_phase_valu.py build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1 2 3 4 full; do
  lib="$PWD/aido1_amd/libdtsim_rstop_$k.so"
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  DTSIM_DIAG_LIB="$lib" timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES \
      --output-format csv -d "$PWD/gpurun_out/rstop_$k" -o run -- python3 bench.py --config render \
      --steps 20 --warmup 5 --cpu-steps 0 --no-lane --no-parity > "gpurun_out/rstop_$k.log" 2>&1 \
      || { echo "stop $k failed"; exit 1; }
  echo "stop $k done"
done
