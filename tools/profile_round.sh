#!/bin/bash
# Round profiles: rocprofv3 --kernel-trace --stats of every bench config, then
# PMC HBM traffic of the configs 2-3 kernels (FETCH_SIZE and WRITE_SIZE in
# separate passes: they do not fit one TCC pass).  Each GPU step has its own
# time limit; a fault/timeout stops the script.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=${STEPS:-100}
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping"; exit $rc; }
}
declare -A ARGS=(
  [lane]="--steps $STEPS --warmup 20 --cpu-seconds 0"
  [render]="--config render --steps $STEPS --warmup 20 --cpu-seconds 0"
  [actor]="--config actor --steps 30 --warmup 5 --cpu-seconds 0"
  [train]="--config train --steps 30 --warmup 5 --cpu-seconds 0")
for cfg in ${CONFIGS:-lane render actor train}; do
  step "trace_$cfg" 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/gpurun_out/trace_$cfg" -o run -- python3 "$ROOT/bench.py" ${ARGS[$cfg]}
done
for cfg in ${PMC_CONFIGS:-lane render}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step "pmc_${cfg}_$ctr" 600 rocprofv3 --pmc $ctr --output-format csv \
        -d "$ROOT/gpurun_out/pmc_${cfg}_$ctr" -o run -- python3 "$ROOT/bench.py" ${ARGS[$cfg]}
  done
done
echo done
