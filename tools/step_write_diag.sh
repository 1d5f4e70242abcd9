#!/bin/bash
# Where do step_fan_kernel's HBM writes go?  WRITE_SIZE of the config-2 bench
# (dt_step_many, 20-decision launches) with one store class removed at a time
# (DTSIM_DIAG_SKIP_STORES bits: 1 reward, 2 reward_mod, 4 done, 8 obs,
# 16 spawn-slot refill).  Diagnostic libraries: built here on the CPU first
# (python tools/step_write_diag.py build), loaded through DTSIM_DIAG_LIB; the
# outputs of a masked build are wrong, so parity is off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 0 1 2 4 8 16; do
  lib="$PWD/aido1_amd/libdtsim_diag_st$m.so"
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  DTSIM_DIAG_LIB="$lib" timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d "$PWD/gpurun_out/stw_$m" -o run -- python3 bench.py --config lane --steps 20 \
      --warmup 20 --cpu-steps 0 --no-parity > "gpurun_out/stw_$m.log" 2>&1 || { echo "mask $m failed"; exit 1; }
  echo "mask $m done"
done
