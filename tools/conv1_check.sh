#!/bin/bash
# conv1 forms: GPU actor tests under the streaming (default) and banded conv1,
# then the config-4 bench line with each (reference and eval mode).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in 0 1; do
  DTCONV1_BANDED=$b timeout -k 10 400 python -u -m pytest tests/test_gpu_actor.py -x -q -m gpu --timeout 200 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_actor_$b.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_actor_$b.log; [ $rc -eq 0 ] || exit $rc
done
for b in 0 1; do
  for m in reference eval; do
    DTCONV1_BANDED=$b timeout -k 10 300 python bench.py --config actor --actor-mode $m --steps 30 --warmup 5 --cpu-steps 0 > gpurun_out/bench_actor_b${b}_$m.log 2>&1 || exit 1
    python3 - "$b" "$m" <<'PY'
import json, sys
for l in open('gpurun_out/bench_actor_b%s_%s.log' % (sys.argv[1], sys.argv[2])):
    if l.startswith('{'):
        d = json.loads(l)
        print('banded=%s %-9s value %.3fM actor %.3f ms frac %.3f' % (sys.argv[1], sys.argv[2], d['value'] / 1e6, d['roofline']['avg_kernel_ms'], d['roofline']['frac']))
PY
  done
done
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/gpurun_out/trace_conv1s" -o run -- python3 "$(pwd)/bench.py" --config actor --steps 30 --warmup 5 --cpu-steps 0 > gpurun_out/trace_conv1s.log 2>&1 || exit 1
  python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/trace_conv1s/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print('%-60s %8s calls avg %.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
PY
fi
