#!/bin/bash
# config-2 step kernel check at HEAD: bench line, WRITE_SIZE / FETCH_SIZE
# passes and a kernel trace of the lane workload (no CPU baseline under the
# profiler), then the headline bench without the CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 180 python bench.py --config lane --steps 320 --warmup 20 --cpu-steps 0 > gpurun_out/lane.json 2> gpurun_out/lane.err || exit 1
timeout -k 10 240 python bench.py --cpu-steps 0 > gpurun_out/render.json 2> gpurun_out/render.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $PWD/gpurun_out/stw -o run -- python3 bench.py --config lane --steps 20 --warmup 20 --cpu-steps 0 --no-parity > gpurun_out/stw.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $PWD/gpurun_out/stf -o run -- python3 bench.py --config lane --steps 20 --warmup 20 --cpu-steps 0 --no-parity > gpurun_out/stf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stk -o run -- python3 bench.py --config lane --steps 320 --warmup 20 --cpu-steps 0 --no-parity > gpurun_out/stk.log 2>&1 || exit 1
echo ALLOK
