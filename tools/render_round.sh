#!/bin/bash
# render rewrite check: parity tests, tools/render_bench.py, stamps, the config-3 bench
# in both stream arrangements, WRITE_SIZE of render_kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rr_pytest.log 2>&1 || { tail -30 gpurun_out/rr_pytest.log; exit 1; }
tail -1 gpurun_out/rr_pytest.log
timeout -k 10 120 python tools/render_bench.py || exit 1
DTSIM_DIAG_LIB=$PWD/aido1_amd/libdtsim_stamps.so timeout -k 10 120 python tools/render_stamps.py || exit 1
for m in many serial pipe; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 --no-lane --obs-mode $m > gpurun_out/rr_$m.json 2> gpurun_out/rr_$m.err || { tail -30 gpurun_out/rr_$m.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/rr_$m.json'))
print('$m', 'value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'render ms %.4f' % d['roofline']['avg_kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'step ms/launch %.4f' % d['step_launch_ms'], 'host %.4f' % d['host_enqueue_ms_per_step'], 'parity', d['parity']['ok'])"
done
TIME_ONLY=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/rr_w -o run -- python3 tools/render_stamps.py > /dev/null 2>&1 || exit 1
python3 -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('gpurun_out/rr_w/run_counter_collection.csv')) if 'render_kernel' in r['Kernel_Name']]
print('WRITE_SIZE MB per render', sum(v)/len(v)*1024/1e6, 'vs algorithmic', 153624*4096/1e6)"
