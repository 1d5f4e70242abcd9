#!/bin/bash
# render variants side by side on one box: stamps of the stamps libs, times of the others
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${STAMPS:-libdtsim_stamps}; do
  echo "== stamps $v"; DTSIM_DIAG_LIB=$PWD/aido1_amd/$v.so timeout -k 10 120 python tools/render_stamps.py || exit 1
done
for v in ${TIMES:-libdtsim}; do
  echo "== time $v"; DTSIM_DIAG_LIB=$PWD/aido1_amd/$v.so timeout -k 10 120 python tools/render_bench.py 2>&1 | head -4 || exit 1
done
