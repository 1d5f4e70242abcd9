#!/bin/bash
# Diagnostic: the DDPG update alone (tools/update_only.py, back to back) under
# HIP-runtime graph-execution settings, one process a setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" UPDATES=50 timeout -k 10 120 python -u tools/update_only.py > gpurun_out/genv_$tag.txt 2>&1 \
    || { echo "$tag failed"; tail -5 gpurun_out/genv_$tag.txt; return 1; }
  echo "$tag $(grep 'back to back, 5' gpurun_out/genv_$tag.txt)"
  echo "$tag $(grep 'host time' gpurun_out/genv_$tag.txt)"
}
if [ $# -gt 0 ]; then
  for kv in "$@"; do run "${kv%%=*}" "$kv"; done
  exit 0
fi
run default X=1
run batch256 DEBUG_HIP_GRAPH_BATCH_SIZE=256
run batch8 DEBUG_HIP_GRAPH_BATCH_SIZE=8
run queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run queues4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
run queues8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run default2 X=2
