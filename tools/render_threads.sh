#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_render.py tests/test_gpu_step.py -x -q -m gpu > gpurun_out/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/pytest.log; case $rc in 0|1) ;; *) exit $rc;; esac
for t in 256 512 768 1024; do
  DTSIM_RENDER_THREADS=$t timeout -k 10 120 python bench.py --config render --steps 200 --warmup 20 --cpu-seconds 0 2>/dev/null | grep '^{' > gpurun_out/thr_$t.json || exit $?
  python -c "import json;d=json.load(open('gpurun_out/thr_$t.json'));print('threads=$t render_ms=%.4f value=%.4g step_ms=%.4f'%(d['roofline']['avg_kernel_ms'],d['value'],d['step_kernel_ms']))"
done
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 2>/dev/null | grep '^{' > gpurun_out/lane.json || exit $?
python -c "import json;d=json.load(open('gpurun_out/lane.json'));print('lane value=%.4g ms=%.4f'%(d['value'],d['roofline']['avg_kernel_ms']))"
