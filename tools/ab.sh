#!/bin/bash
# A/B of a build switch: bench.py with the product library and a diagnostic
# build (DTSIM_DIAG_LIB=<lib>), alternated R times; one summary line a run.
# usage: tools/ab.sh <diag .so> <R> [bench args...]  (default: the render bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
lib=$1; R=${2:-3}; shift 2
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 100 --warmup 20 --cpu-steps 0 --no-lane --no-sub --no-parity \
                               --event-stride 1)
for i in $(seq 1 "$R"); do
  for v in product diag; do
    if [ $v = diag ]; then export DTSIM_DIAG_LIB=$PWD/$lib; else unset DTSIM_DIAG_LIB; fi
    timeout -k 10 300 python bench.py "${args[@]}" > gpurun_out/ab_${v}_${i}.json \
      2> gpurun_out/ab_err.log || { tail -20 gpurun_out/ab_err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_${v}_${i}.json'))
r=d['roofline']
ph=d.get('phases_ms') or {}
print('$v', 'value %.4gM' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'kernel ms %.4f' % r['avg_kernel_ms'], 'frac %.3f' % r['frac'], ('update ms %.4f' % ph['update']) if 'update' in ph else '')"
  done
done
