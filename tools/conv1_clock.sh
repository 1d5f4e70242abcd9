#!/bin/bash
# Diagnostic: is conv1s cycle-bound or clock-bound?  GRBM_GUI_ACTIVE (GPU
# cycles while busy) and SQ_BUSY_CYCLES of the full kernel on random, zero and
# piecewise-constant operands (tools/conv1_micro.py variants in diag_so/, TAGS / DATAS select).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
for tag in ${TAGS:-""}; do for data in ${DATAS:-random zero frames}; do
  CONV1_DATA=$data CONV1_TAG=$tag CONV1_ONLY=full timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
      --kernel-trace --output-format csv -d "$ROOT/gpurun_out/clk_$tag$data" -o run -- python3 "$ROOT/tools/conv1_micro.py" > gpurun_out/clk_$tag$data.log 2>&1 || { echo "fail $data"; exit 1; }
  python3 - "$ROOT/gpurun_out/clk_$tag$data" "$tag $data" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
c = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(d + '/**/run_counter_collection.csv', recursive=True)[0])):
    if 'conv1' in r['Kernel_Name']:
        c[r['Counter_Name']].append(float(r['Counter_Value']))
t = [ (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) for r in csv.DictReader(open(glob.glob(d + '/**/run_kernel_trace.csv', recursive=True)[0])) if 'conv1' in r['Kernel_Name']]
import statistics as st
print(sys.argv[2], 'kernel us %.1f' % (st.median(t) / 1e3), ' '.join('%s %.4g' % (k, st.median(v)) for k, v in c.items()))
PY
done; done
