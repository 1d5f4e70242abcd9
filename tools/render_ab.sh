#!/bin/bash
# A/B of a render-kernel build switch: the config-3 bench (render only) with the
# product library and a diagnostic build (DTSIM_DIAG_LIB=$1), alternated R times.
# usage: tools/render_ab.sh <diag .so> [R]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib=$1; R=${2:-3}
for i in $(seq 1 "$R"); do
  for v in product diag; do
    if [ $v = diag ]; then export DTSIM_DIAG_LIB=$PWD/$lib; else unset DTSIM_DIAG_LIB; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 20 --cpu-steps 0 --no-lane --no-sub \
      --no-parity --event-stride 1 > gpurun_out/ab_${v}_${i}.json 2> gpurun_out/ab_err.log || {
      tail -20 gpurun_out/ab_err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_${v}_${i}.json'))
print('$v', 'value %.4gM' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'render ms %.4f' % d['roofline']['avg_kernel_ms'], 'frac %.3f' % d['roofline']['frac'])"
  done
done
