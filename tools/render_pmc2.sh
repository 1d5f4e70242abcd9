#!/bin/bash
# render_kernel instruction mix and LDS pressure (one --pmc pass per set, the
# standalone render loop of tools/render_stamps.py TIME_ONLY=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  TIME_ONLY=1 timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/rp2_$i -o run -- python3 tools/render_stamps.py > gpurun_out/rp2_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/rp2_$i.log; }
done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/rp2_*/**/*counter_collection.csv', recursive=True)):
    acc = {}
    n = {}
    for r in csv.DictReader(open(f)):
        if 'render_kernel' not in r['Kernel_Name']:
            continue
        k = r['Counter_Name']
        d = r.get('Dispatch_Id')
        acc.setdefault(k, {}).setdefault(d, 0.0)
        acc[k][d] += float(r['Counter_Value'])
    for k, v in acc.items():
        vals = list(v.values())
        print('%-24s per dispatch %.4g (dispatches %d)' % (k, sum(vals) / len(vals), len(vals)))
PY
