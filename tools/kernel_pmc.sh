#!/bin/bash
# Diagnostic: rocprofv3 PMC counters for the kernels whose name contains
# $KERNEL, on `bench.py --config $CONFIG`; one counter set per pass
# (SETS: space-separated, counters within a set comma-separated).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
CONFIG=${CONFIG:-actor}; KERNEL=${KERNEL:-conv32}; ARGS=${ARGS:-}
SETS=${SETS:-"SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_MFMA,SQ_WAVES,GRBM_GUI_ACTIVE"}
i=0
for ctr in $SETS; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$ROOT/gpurun_out/kpmc_$i" -o run -- \
    python3 "$ROOT/bench.py" --config $CONFIG --steps 10 --warmup 3 --cpu-steps 0 $ARGS > "gpurun_out/kpmc_$i.log" 2>&1 || { echo "fail $i"; exit 1; }
  python3 - "$ROOT/gpurun_out/kpmc_$i/run_counter_collection.csv" "$KERNEL" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    if sys.argv[2] in k:
        key = k[:70]
        tot[key][r['Counter_Name']] += float(r['Counter_Value']); n[key][r['Counter_Name']] += 1
for key in sorted(tot):
    print(key, ' '.join('%s=%.4g' % (c, tot[key][c] / n[key][c]) for c in sorted(tot[key])))
PY
done
