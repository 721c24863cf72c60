"""CPU AddressSanitizer run of the C-ABI host code (SURVEY §5 sanitizers): tools/asan/build_asan.sh
builds the error plumbing and the planners / argument validation of thin3, tconv, skinny and
pwsmall with -fsanitize=address on the host side, and a driver exercises them without a GPU."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_host_code_under_asan():
    b = subprocess.run(["bash", os.path.join(REPO, "tools", "asan", "build_asan.sh")], capture_output=True,
                       text=True, timeout=600)
    assert b.returncode == 0, b.stderr[-2000:]
    drv = b.stdout.strip().splitlines()[-1]
    r = subprocess.run([drv], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0"))
    assert "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0 and "ASAN OK" in r.stdout, (r.stdout, r.stderr[-2000:])
