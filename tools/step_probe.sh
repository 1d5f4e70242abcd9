#!/bin/bash
# Diagnostic: config-2 step kernel -- kernel-trace stats under a few
# DTSIM_REFILL_ENVS settings, then PMC issue counters of step_kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
for re in ${REFILLS:-1 16}; do
  DTSIM_REFILL_ENVS=$re timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$ROOT/gpurun_out/step_trace_$re" -o run -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 \
    --cpu-seconds 0 > "gpurun_out/step_trace_$re.log" 2>&1 || { echo "trace fail $re"; exit 1; }
  echo "== refill_envs=$re"; tail -n 1 "gpurun_out/step_trace_$re.log" | cut -c1-400
  find "$ROOT/gpurun_out/step_trace_$re" -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200
done
CONFIG=lane KERNEL=step_kernel SETS="${SETS:-SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVES,GRBM_GUI_ACTIVE}" \
  bash tools/kernel_pmc.sh
