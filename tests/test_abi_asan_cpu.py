"""Host-side AddressSanitizer check of the C-ABI (no GPU): tests/native/abi_host_check.c drives
every entry point's descriptor validation, error codes, thread-local messages and the
workspace / band queries against libthzdoe_asan.so (host code built with -fsanitize=address,
`make -C quantizationawarethzdoe_amd/csrc asan`).  An out-of-bounds access or leak on these host
paths aborts the checker; no kernel is launched."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quantizationawarethzdoe_amd", "csrc")
CHECK = os.path.join(ROOT, "tests", "native", "abi_host_check")


def test_abi_host_paths_under_asan():
    if shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("needs hipcc to build the ASan library")
    subprocess.run(["make", "-s", "-C", CSRC, "asan"], check=True, timeout=900)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    r = subprocess.run([CHECK], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi host checks passed" in r.stdout
