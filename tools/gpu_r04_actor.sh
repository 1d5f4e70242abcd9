#!/bin/bash
# actor change: its GPU tests, then config-4 bench runs (reference and eval)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_actor.py tests/test_gpu_explore.py tests/test_gpu_scale.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r04_actor_tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r04_actor_tests.log)"; grep -E "FAILED|Error" gpurun_out/r04_actor_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
for mode in reference eval; do
  timeout -k 10 300 python bench.py --config actor --actor-mode $mode --steps 30 --warmup 5 --cpu-steps 0 > gpurun_out/r04_actor_bench_$mode.log 2>&1 || exit $?
  python - "$mode" <<'PY'
import json, sys
for line in open('gpurun_out/r04_actor_bench_%s.log' % sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line)
        r = d['roofline']
        print('%s value %.3fM actor %.4f ms frac %.3f parity %s max %.2e' % (sys.argv[1], d['value'] / 1e6, r['avg_kernel_ms'], r['frac'], d['parity']['ok'], d['parity']['max_abs_err']))
PY
done
rm -rf /tmp/prof_actor
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_actor -o run --output-format csv -- python3 bench.py --config actor --steps 20 --warmup 5 --cpu-steps 0 --no-parity > gpurun_out/r04_actor_prof.log 2>&1 || exit $?
f=$(find /tmp/prof_actor -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/r04_actor_kernel_stats_new.csv
grep conv gpurun_out/r04_actor_kernel_stats_new.csv | cut -d, -f1-4 | cut -c1-40,100-200
