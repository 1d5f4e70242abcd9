#!/bin/bash
# Diagnostic: rocprofv3 PMC counters of the kernels whose names hold NEEDLE,
# inside bench.py --config CONFIG (short run), one counter set a pass; prints
# the per-launch mean of each counter per matching kernel.
# usage: tools/kernel_pmc.sh CONFIG NEEDLE [NEEDLE ...]   (SETS=... overrides the passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=$1; shift
NEEDLES="$*"
SETS=${SETS:-"SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAVES,GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR,SQ_INST_CYCLES_VMEM_WR"}
i=0
for ctr in $SETS; do
  i=$((i+1))
  rm -rf "/tmp/kpmc_$i"
  timeout -k 10 -s KILL 180 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "/tmp/kpmc_$i" -o run -- \
    python3 "$ROOT/bench.py" --config "$CFG" --steps 5 --warmup 3 --cpu-steps 0 --no-parity \
    > "gpurun_out/kpmc_$i.log" 2>&1 || { echo "fail $i"; tail -5 "gpurun_out/kpmc_$i.log"; exit 1; }
  f=$(find "/tmp/kpmc_$i" -name '*counter_collection.csv' | head -1)
  python3 - "$f" $NEEDLES <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    for nd in sys.argv[2:]:
        if nd in r['Kernel_Name']:
            key = (r['Kernel_Name'][:60], r['Counter_Name'])
            tot[key] += float(r['Counter_Value']); n[key] += 1
for k in sorted(tot):
    print(k[0], k[1], '%.4g' % (tot[k] / n[k]))
PY
done
