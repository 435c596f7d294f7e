"""Host runtime under AddressSanitizer + UndefinedBehaviorSanitizer.

``csrc/host/dataio.cpp`` is compiled with the edge-case driver ``csrc/host/check/
sanitize_dataio.cpp`` into one sanitized executable and run; the driver checks every result
itself, so a pass means no sanitizer report and correct values.  CPU only."""
import os
import shutil
import subprocess

import pytest

from dinunet_implementations_amd.csrc import build as b

pytestmark = pytest.mark.skipif(shutil.which(b.CXX) is None and not os.path.exists(b.CXX),
                                reason="no host C++ compiler")


@pytest.mark.parametrize("sanitizers", ["address,undefined"])
def test_host_runtime_under_sanitizers(tmp_path, sanitizers):
    exe = str(tmp_path / "dinunet_host_sanitized")
    try:
        b.build_host_sanitized(exe, sanitizers)
    except RuntimeError as e:
        if "cannot find" in str(e) and "asan" in str(e):
            pytest.skip("sanitizer runtime not installed")
        raise
    scratch = tmp_path / "files"
    scratch.mkdir()
    env = dict(os.environ, OMP_NUM_THREADS="4",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(scratch)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "host sanitizer checks passed" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
