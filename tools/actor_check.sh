#!/bin/bash
# Quick loop for the actor kernels: GPU actor tests, then the config-4 bench
# line with the fused conv12 kernel and with the unfused chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_actor.py -x -q -m gpu --timeout 200 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_actor.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_actor.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  for m in reference eval; do
    DTCONV_FUSED12=$f timeout -k 10 300 python bench.py --config actor --actor-mode $m --steps 30 --warmup 5 --cpu-steps 0 > gpurun_out/bench_actor_${f}_$m.log 2>&1 || exit 1
    python3 - "$f" "$m" <<'PY'
import json, sys
for l in open('gpurun_out/bench_actor_%s_%s.log' % (sys.argv[1], sys.argv[2])):
    if l.startswith('{'):
        d = json.loads(l)
        print('fused12=%s %-9s value %.3fM actor %.3f ms frac %.3f' % (sys.argv[1], sys.argv[2], d['value'] / 1e6, d['roofline']['avg_kernel_ms'], d['roofline']['frac']))
PY
  done
done
