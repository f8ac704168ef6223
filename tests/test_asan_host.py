"""Host-side AddressSanitizer run of the C ABI's argument validation (SURVEY.md §5 aux:
"ASan host build").  forwardtacotron_amd.build.build_asan() compiles every csrc/*.hip with
the host code instrumented (-Xarch_host -fsanitize=address: the gfx950 device code is
untouched) into libftmi_asan.so and links tests/asan/abi_args.cpp against it; the driver
calls each entry point with invalid arguments (null / misaligned pointers, bad shapes,
unsupported options, host pointer arrays of the fused highway stack) and checks the
FTMI_E_* codes.  CPU only: no GPU is touched (the paths return before any launch)."""
import os
import shutil
import subprocess

import pytest


def _asan_env(extra=None):
    env = dict(os.environ)
    env['ASAN_OPTIONS'] = 'detect_leaks=0:halt_on_error=1'
    env.update(extra or {})
    return env


@pytest.fixture(scope='module')
def driver():
    if not (shutil.which('hipcc') or os.path.exists('/opt/rocm/bin/hipcc')):
        pytest.skip('hipcc not available')
    from forwardtacotron_amd.build import build_asan
    return str(build_asan())


def test_argument_validation_under_asan(driver):
    r = subprocess.run([driver], capture_output=True, text=True, env=_asan_env(), timeout=300)
    assert 'AddressSanitizer' not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and 'OK (0 failures)' in r.stdout, (r.stdout, r.stderr[-4000:])


def test_asan_is_live(driver):
    r = subprocess.run([driver], capture_output=True, text=True, timeout=300,
                       env=_asan_env({'FTMI_ASAN_SELFTEST': '1'}))
    assert r.returncode != 0 and 'heap-buffer-overflow' in r.stderr
