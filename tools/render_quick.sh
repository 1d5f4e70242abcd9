#!/bin/bash
# render parity tests + render bench (+ optional ablation)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_render.py -x -q -m gpu > gpurun_out/pytest_render.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_render.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --config render --steps 200 --warmup 20 --cpu-seconds 0 > gpurun_out/bench_render.log 2>&1 || exit $?
python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_render.log') if l.startswith('{')][-1]);print('value %.4g render_ms %.4f frac %.4f'%(d['value'],d['roofline']['avg_kernel_ms'],d['roofline']['frac']))"
if [ -n "$ABLATE" ]; then bash tools/render_ablate.sh; fi
