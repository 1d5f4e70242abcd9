#!/bin/bash
# Diagnostic: the bench's render sub-record (time + 64-env parity) for the
# default library and diagnostic builds given in LIBS (paths, built beforehand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for lib in default $LIBS; do
  i=$((i+1))
  if [ "$lib" = default ]; then unset DTSIM_DIAG_LIB; else export DTSIM_DIAG_LIB=$PWD/$lib; fi
  timeout -k 10 120 python bench.py --steps 60 --warmup 5 --cpu-steps 0 > gpurun_out/var_$i.json 2>/dev/null || exit $?
  python - "$i" "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open('gpurun_out/var_%s.json' % sys.argv[1]) if l.startswith('{')][-1])
r = d['render']
print('%-34s render_ms=%.4f min %.4f parity %s step_us %.3f' % (sys.argv[2], r['avg_kernel_ms'], r['min_kernel_ms'], r.get('parity'), d['step_ms_per_decision'] * 1e3))
PY
done
