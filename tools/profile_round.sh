#!/bin/bash
# Round profiles: rocprofv3 --kernel-trace --stats of every bench config, then
# PMC passes of the headline line's kernels (FETCH_SIZE, WRITE_SIZE and the
# fp64 instruction counters in separate passes: they do not fit one pass).
# Each GPU step has its own time limit; a fault/timeout stops the script.
# Outputs under gpurun_out/; tools/pmc_summarize.py <round> turns them into
# profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=${STEPS:-20}; WARM=${WARM:-5}
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping"; exit $rc; }
}
declare -A ARGS=(
  [lane]="--config lane --steps $STEPS --warmup 20 --cpu-steps 0 --no-sub"
  [render]="--config render --steps 100 --warmup 20 --cpu-steps 0 --no-lane --no-sub"
  [actor]="--config actor --steps 30 --warmup 5 --cpu-steps 0"
  [train]="--config train --steps 30 --warmup 10 --cpu-steps 0")
# plain runs first (no profiler): the bench lines DESIGN quotes
if [ -z "$NO_PLAIN" ]; then
  step bench_driver 400 python3 "$ROOT/bench.py"
  step bench_lane_320 300 python3 "$ROOT/bench.py" --config lane --steps 320 --warmup 20 --cpu-steps 0
  for cfg in render actor train; do step "bench_$cfg" 600 python3 "$ROOT/bench.py" ${ARGS[$cfg]}; done
  step bench_actor_eval 600 python3 "$ROOT/bench.py" ${ARGS[actor]} --actor-mode eval
fi
# traces to /tmp (a full kernel trace outgrows gpurun_out's cap); only the
# stats and counter tables are kept
keep() {  # keep <dir name> <file glob>
  mkdir -p "gpurun_out/$1"
  find "/tmp/prof_$1" -name "$2" -exec cp {} "gpurun_out/$1/" \;
}
for cfg in ${CONFIGS:-lane render actor train}; do
  rm -rf "/tmp/prof_trace_$cfg"
  step "trace_$cfg" 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "/tmp/prof_trace_$cfg" -o run -- python3 "$ROOT/bench.py" ${ARGS[$cfg]}
  keep "trace_$cfg" '*kernel_stats.csv'
done
declare -A PMC=(
  [FETCH_SIZE]="FETCH_SIZE" [WRITE_SIZE]="WRITE_SIZE"
  [FP64]="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64")
for cfg in ${PMC_CONFIGS:-lane render}; do
  for tag in ${PMC_SETS:-FETCH_SIZE WRITE_SIZE FP64}; do
    rm -rf "/tmp/prof_pmc_${cfg}_$tag"
    step "pmc_${cfg}_$tag" 300 rocprofv3 --pmc ${PMC[$tag]} --output-format csv \
        -d "/tmp/prof_pmc_${cfg}_$tag" -o run -- python3 "$ROOT/bench.py" ${ARGS[$cfg]} --no-parity
    keep "pmc_${cfg}_$tag" '*counter_collection.csv'
  done
done
echo done
