#!/bin/bash
# One parameterised GPU-box script (replaces the per-round lease wrappers).
# usage: tools/gpu.sh TAG STEP [STEP ...]
#   suite [pytest args]   the whole GPU suite, one process (TESTS=... narrows it)
#   smoke                 __graft_entry__.smoke()
#   driver                bench.py exactly as the driver runs it (--gpus 1 --steps 20 --warmup 5)
#   bench:<args>          bench.py with <args> (commas become spaces)
#   prof:<config>         rocprofv3 --kernel-trace --stats of bench.py --config <config>
#   py:<script>[,args]    a tools/ python script
#   profpy:<script>[,args]  the same under rocprofv3 --kernel-trace --stats (stats + trace kept)
#   ab:<diag .so>,R[,bench args]  tools/ab.sh: bench.py, product vs a diagnostic build
# Each step has its own time limit; the first failure ends the call (no retries).
# Logs: gpurun_out/<TAG>_<n>_<step>.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  local log="gpurun_out/${TAG}_${i}_${name}.log"
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 8 "$log"
  [ $rc -eq 0 ] || { echo "stopping after $name"; exit $rc; }
}
summ() {  # one-line summary of a bench JSON line
  python3 - "$1" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if not line.startswith('{'):
        continue
    d = json.loads(line)
    r = d.get('roofline') or {}
    s = '%s %.4gM ms/step %.4f frac %s' % (d['config'].get('workload'), d['value'] / 1e6,
                                          d['ms_per_step'], r.get('frac'))
    for k in ('config4', 'config4_fp16', 'config5', 'config5_fp16'):
        if isinstance(d.get(k), dict) and d[k].get('value'):
            s += ' | %s %.3gM' % (k, d[k]['value'] / 1e6)
    print(s, 'parity', (d.get('parity') or {}).get('ok'))
PY
}
for st in "$@"; do
  i=$((i + 1))
  kind=${st%%:*}; arg=${st#*:}; [ "$arg" = "$st" ] && arg=""
  args=${arg//,/ }
  case $kind in
    suite) run suite 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -x --timeout 200 \
             --timeout-method thread $args ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) run driver 600 python bench.py --gpus 1 --steps 20 --warmup 5
            summ "gpurun_out/${TAG}_${i}_driver.log" ;;
    bench) run bench 600 python bench.py $args; summ "gpurun_out/${TAG}_${i}_bench.log" ;;
    prof) rm -rf "/tmp/prof_$arg"
          run "prof_$arg" 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "/tmp/prof_$arg" -o run -- python3 "$ROOT/bench.py" --config "$arg" \
            --steps 20 --warmup 5 --cpu-steps 0 --no-parity
          f=$(find "/tmp/prof_$arg" -name '*kernel_stats.csv' | head -1)
          cp "$f" "gpurun_out/${TAG}_${arg}_kernel_stats.csv"
          cp "${f%_kernel_stats.csv}_kernel_trace.csv" "gpurun_out/${TAG}_${arg}_kernel_trace.csv"
          python3 tools/kstats.py "gpurun_out/${TAG}_${arg}_kernel_stats.csv" 25 ;;
    profpy) set -- $args; s=$1; shift; rm -rf "/tmp/prof_py"
          run "profpy_$(basename "$s" .py)" 600 rocprofv3 --kernel-trace --stats \
            --output-format csv -d /tmp/prof_py -o run -- python3 "$ROOT/tools/$s" "$@"
          f=$(find /tmp/prof_py -name '*kernel_stats.csv' | head -1)
          cp "$f" "gpurun_out/${TAG}_$(basename "$s" .py)_kernel_stats.csv"
          cp "${f%_kernel_stats.csv}_kernel_trace.csv" "gpurun_out/${TAG}_$(basename "$s" .py)_kernel_trace.csv"
          python3 tools/kstats.py "gpurun_out/${TAG}_$(basename "$s" .py)_kernel_stats.csv" 40 ;;
    ab) run ab 900 bash tools/ab.sh $args ;;
    py) set -- $args; s=$1; shift
        run "py_$(basename "$s" .py)" 600 python -u "tools/$s" "$@" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "all steps ok"
