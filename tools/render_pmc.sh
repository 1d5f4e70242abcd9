#!/bin/bash
# Diagnostic: rocprofv3 PMC counters of render_kernel alone (tools/render_stamps.py
# TIME_ONLY: 30 back-to-back renders of 4096 envs; GROUP=1: the config-3 bench's grouped
# dt_render3 launches), one counter set per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
SETS=${SETS:-"SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR,SQ_INST_CYCLES_VMEM_WR,SQ_WAVES,GRBM_GUI_ACTIVE FETCH_SIZE WRITE_SIZE"}
i=0
for ctr in $SETS; do
  i=$((i+1))
  if [ -n "$GROUP" ]; then   # the bench's grouped launches (dt_step_many + dt_render3)
    timeout -k 10 -s KILL 180 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$ROOT/gpurun_out/rpmc_$i" -o run -- \
      python3 "$ROOT/bench.py" --config render --steps 40 --warmup 10 --cpu-steps 0 --no-lane --no-sub \
      --no-parity > "gpurun_out/rpmc_$i.log" 2>&1 || { echo "fail $i"; tail -5 gpurun_out/rpmc_$i.log; exit 1; }
  else
    TIME_ONLY=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$ROOT/gpurun_out/rpmc_$i" -o run -- \
      python3 "$ROOT/tools/render_stamps.py" > "gpurun_out/rpmc_$i.log" 2>&1 || { echo "fail $i"; tail -5 gpurun_out/rpmc_$i.log; exit 1; }
  fi
  python3 - "$ROOT/gpurun_out/rpmc_$i/run_counter_collection.csv" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if 'render_kernel' in r['Kernel_Name']:
        tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
print(' '.join('%s=%.4g' % (k, tot[k] / n[k]) for k in sorted(tot)))
PY
done
