#!/bin/bash
# Diagnostic: render-kernel time with phases ablated (DTSIM_RENDER_SKIP bits:
# 1 background, 2 markings, 4 uniform/grey, 8 sobel/NMS, 16 hysteresis, 32 masks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in 0 1 2 4 8 16 32 63; do
  DTSIM_RENDER_SKIP=$s timeout -k 10 120 python bench.py --config render --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/abl_$s.json 2>/dev/null || exit $?
  python -c "import json;d=json.loads([l for l in open("gpurun_out/abl_$s.json") if l.startswith("{")][-1]);print('skip=$s render_ms=%.4f'%d['roofline']['avg_kernel_ms'])"
done
