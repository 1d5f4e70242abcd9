#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_suite_repeat.sh 2 r04_suite_b || exit $?
tools/gpu_r04_b.sh
