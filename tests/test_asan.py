"""SURVEY.md §5 "Race detection / sanitizers": the host side of the C ABI and
the oracle's C restatement built with AddressSanitizer + UBSan (`make asan`,
host code only: the gfx950 device code is built uninstrumented) and
driven by tests/asan_driver.py in a process with clang's ASan runtime
preloaded: every entry point's argument checks, every map through
dt_create's validation, and the oracle tests on the sanitized oracle.  Any
sanitizer report fails the run."""
import os
import subprocess
import sys

import pytest

from conftest import REPO


def test_host_code_clean_under_asan_and_ubsan():
    if not os.path.exists('/opt/rocm/bin/hipcc'):
        pytest.skip('no hipcc')
    r = subprocess.run(['make', '-s', '-j8', 'asan'], cwd=REPO, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rt = subprocess.run(['make', '-s', 'asan-rt'], cwd=REPO, capture_output=True, text=True,
                        check=True).stdout.strip()
    assert os.path.exists(rt), rt
    env = dict(os.environ)
    pre = env.get('LD_PRELOAD', '')
    env['LD_PRELOAD'] = rt + (':' + pre if pre else '')   # the runtime first, anything else kept
    env['ASAN_OPTIONS'] = 'detect_leaks=0:halt_on_error=1:exitcode=99'
    env['UBSAN_OPTIONS'] = 'halt_on_error=1:print_stacktrace=1'
    env['DTSIM_ASAN_LIB'] = os.path.join(REPO, 'build', 'asan', 'libdtsim_asan.so')
    env['DTSIM_ORACLE_LIB'] = os.path.join(REPO, 'build', 'asan', 'liboracle_asan.so')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'tests', 'asan_driver.py')], env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert 'clean under ASan/UBSan' in r.stdout
    assert 'ERROR: AddressSanitizer' not in r.stderr and 'runtime error' not in r.stderr
