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


def test_sanitizer_toolchain_reports_heap_overflow(tmp_path):
    """Negative control: the same flags do catch an out-of-bounds write, so a clean run of the
    driver above means something."""
    src = tmp_path / "oob.cpp"
    # the overflowed slot is written through a volatile pointer and read back into the exit
    # code, so no optimisation level can drop the store before ASan instruments it
    src.write_text("#include <vector>\nint main(int c, char**) { std::vector<int> v(4);"
                   " volatile int* p = v.data(); p[c + 3] = 1; return p[c + 3] + p[0]; }\n")
    exe = str(tmp_path / "oob")
    r = subprocess.run([b.CXX, "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                        str(src), "-o", exe], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-200:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, r.stderr[-2000:]
