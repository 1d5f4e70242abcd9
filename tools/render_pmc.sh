#!/bin/bash
# Diagnostic: rocprofv3 PMC counters for the render kernel, full vs phase 2 ablated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE"; do
  for skip in 0 8; do
    i=$((i+1))
    DTSIM_RENDER_SKIP=$skip timeout -k 10 180 rocprofv3 --pmc $ctr --output-format csv -d "$ROOT/gpurun_out/pmc_$i" -o run -- \
      python3 "$ROOT/bench.py" --config render --steps 20 --warmup 3 --cpu-seconds 0 > "gpurun_out/pmc_$i.log" 2>&1 || { echo "fail $i"; exit 1; }
    echo "pass $i skip=$skip ctr=$ctr"
  done
done
