#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout/abort stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
STEPS=${STEPS:-300}
run() {  # run <name> <timeout> cmd...; stop on fault-like exit codes
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0;; *) echo "fatal rc=$rc, stopping"; exit $rc;; esac
}
run smi 60 rocm-smi --showproductname
run pytest_gpu 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 180 --timeout-method thread
run bench 600 python bench.py --steps $STEPS --warmup 30 ${BENCH_ARGS}
if [ -n "$RENDER" ]; then
  run bench_render 600 python bench.py --config render --steps $STEPS --warmup 30 --cpu-steps 0
fi
if [ -n "$ACTOR" ]; then
  run bench_actor 600 python bench.py --config actor --steps 100 --warmup 10 --cpu-steps 0
  run bench_actor_eval 600 python bench.py --config actor --actor-mode eval --steps 100 --warmup 10 --cpu-steps 0
fi
if [ -n "$TRAIN" ]; then
  run bench_train 600 python bench.py --config train --steps 50 --warmup 5 --cpu-steps 0
fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run \
      --output-format csv -- python3 "$ROOT/bench.py" --steps $STEPS --warmup 30 --cpu-steps 0 ${BENCH_ARGS}
  if [ -n "$RENDER" ]; then
    run rocprof_render 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_render" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" --config render --steps $STEPS --warmup 30 --cpu-steps 0
  fi
fi
echo done
