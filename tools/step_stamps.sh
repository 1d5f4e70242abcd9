#!/bin/bash
# Build the -DDTSIM_STAMPS diagnostic library (on the CPU host, before gpurun):
# the product flags and sources (_lib.build) plus the stamp define.
cd "$(dirname "$0")/.."
python3 -c "
from aido1_amd import _lib
import os
_lib.build(force=True, path=os.path.join(_lib.PKG_DIR, 'libdtsim_stamps.so'), defines=['DTSIM_STAMPS'])"
