#!/bin/bash
# conv1 check: actor GPU tests, then dt_conv1 alone (tools/conv1_micro.py
# variants built beforehand into diag_so/conv1_variants$TAG, TAGS selects) on
# random and frame-like operands, then the config-4 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_actor.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c1_pytest.log 2>&1 || { tail -40 gpurun_out/c1_pytest.log; exit 1; }
tail -1 gpurun_out/c1_pytest.log
for tag in ${TAGS:-""}; do
  for data in random frames; do
    echo "== $tag $data"
    CONV1_ONLY=full CONV1_TAG=$tag CONV1_DATA=$data timeout -k 10 120 python tools/conv1_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 400 python bench.py --config actor --steps 30 --warmup 10 --cpu-steps 0 > gpurun_out/c1_actor.json 2> gpurun_out/c1_actor.err || { tail -20 gpurun_out/c1_actor.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/c1_actor.json')); print('actor', 'value %.4g' % d['value'], 'ms/step %.3f' % d['ms_per_step'], 'actor ms %.3f' % d['roofline']['avg_kernel_ms'])"
