#!/bin/bash
# Diagnostic: rocprofv3 PMC counters of the kernels whose names hold one of
# NEEDLES, inside an arbitrary short command, one counter set a pass (each its
# own run, --pmc only); prints the per-dispatch mean of each counter per
# matching kernel.
# usage: SETS="A,B C,D" tools/cmd_pmc.sh "needle1 needle2" python3 tools/x.py args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
NEEDLES="$1"; shift
SETS=${SETS:-"SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY TCP_TOTAL_CACHE_ACCESSES_sum,TCP_TCC_READ_REQ_sum,TCC_HIT_sum,TCC_MISS_sum FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE"}
i=0
for ctr in $SETS; do
  i=$((i+1))
  rm -rf "/tmp/cpmc_$i"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "/tmp/cpmc_$i" -o run -- \
    "$@" > "gpurun_out/cpmc_$i.log" 2>&1 || { echo "fail $i ($ctr)"; tail -5 "gpurun_out/cpmc_$i.log"; exit 1; }
  f=$(find "/tmp/cpmc_$i" -name '*counter_collection.csv' | head -1)
  python3 - "$f" $NEEDLES <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    for nd in sys.argv[2:]:
        if nd in r['Kernel_Name']:
            key = (r['Kernel_Name'][:70], r['Counter_Name'])
            tot[key] += float(r['Counter_Value'])
            disp[key].add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
for k in sorted(tot):
    print(k[0], k[1], '%.4g' % (tot[k] / max(1, len(disp[k]))))
PY
done
