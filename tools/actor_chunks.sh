#!/bin/bash
# Diagnostic: config-4 actor time per conv chunk size (DTCONV_CHUNK) and path
# (DTCONV_FUSED12).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${FUSED:-0}; do
  for c in ${CHUNKS:-4096 1024 512 256}; do
    DTCONV_FUSED12=$f DTCONV_CHUNK=$c timeout -k 10 300 python bench.py --config actor --steps 30 --warmup 5 --cpu-steps 0 > gpurun_out/chunk_${f}_$c.log 2>&1 || exit 1
    python3 - "$f" "$c" <<'PY'
import json, sys
for l in open('gpurun_out/chunk_%s_%s.log' % (sys.argv[1], sys.argv[2])):
    if l.startswith('{'):
        d = json.loads(l)
        print('fused12=%s chunk=%-5s value %.3fM actor %.3f ms' % (sys.argv[1], sys.argv[2], d['value'] / 1e6, d['roofline']['avg_kernel_ms']))
PY
  done
done
