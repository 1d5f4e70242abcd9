#!/bin/bash
# Where a step_pair_kernel wave's cycles go: SQ wave-cycle buckets and
# instruction counts (one --pmc pass), plus the fp64 latency microbenchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=${ARGS:---steps 20 --warmup 5 --cpu-steps 0 --no-parity --no-render}
timeout -k 10 60 ./tools/fp64_lat > gpurun_out/fp64_lat.log 2>&1 || exit 1
cat gpurun_out/fp64_lat.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH --output-format csv \
    -d "$ROOT/gpurun_out/pmc_step_sq" -o run -- python3 "$ROOT/bench.py" $ARGS \
    > gpurun_out/pmc_step_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$ROOT/gpurun_out/pmc_step_sq2" -o run -- python3 "$ROOT/bench.py" $ARGS \
    > gpurun_out/pmc_step_sq2.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for d in ('pmc_step_sq', 'pmc_step_sq2'):
    for f in glob.glob('gpurun_out/%s/**/*counter_collection.csv' % d, recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if 'step_pair_kernel' in r['Kernel_Name']:
                acc[(r['Dispatch_Id'], r['Counter_Name'])].append(float(r['Counter_Value']))
        per = collections.defaultdict(list)
        for (di, c), v in acc.items():
            per[c].append(sum(v))
        for c, v in sorted(per.items()):
            print(d, c, 'dispatches', len(v), 'mean', sum(v) / len(v))
PY
