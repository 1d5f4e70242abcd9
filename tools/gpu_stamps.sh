#!/bin/bash
# render_kernel: standalone time (production lib) + phase stamps (stamps lib,
# built beforehand by tools/step_stamps.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TIME_ONLY=1 timeout -k 10 120 python tools/render_stamps.py || exit 1
DTSIM_DIAG_LIB=$PWD/aido1_amd/libdtsim_stamps.so timeout -k 10 120 python tools/render_stamps.py || exit 1
