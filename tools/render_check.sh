#!/bin/bash
# render change check: render parity tests, standalone render time, stamps,
# the config-3 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_scale.py tests/test_gpu_hough.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rc_pytest.log 2>&1 || { tail -30 gpurun_out/rc_pytest.log; exit 1; }
tail -1 gpurun_out/rc_pytest.log
TIME_ONLY=1 timeout -k 10 120 python tools/render_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
DTSIM_DIAG_LIB=$PWD/aido1_amd/libdtsim_stamps.so timeout -k 10 120 python tools/render_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-steps 0 --no-lane > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err || { tail -30 gpurun_out/rc_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/rc_bench.json'))
print('config3', 'value %.4g' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'render ms %.4f' % d['roofline']['avg_kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'parity', d['parity']['ok'], d['parity']['gray_mismatches'], d['parity']['mask_mismatches'])"
