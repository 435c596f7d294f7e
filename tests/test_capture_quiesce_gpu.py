"""RCCL collectives captured right after eager ones: no hipErrorCapturedEvent
abort of the process group's watchdog, with the deterministic quiesce (``_wait_for_pending_works``)
in place of round 5's fixed sleeps.  In a subprocess: a regression aborts that process only."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capture_right_after_eager_collectives():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag", "capture_after_eager.py"),
                        "20"], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stderr[-3000:])
    res = json.loads(lines[-1])
    assert res["ok"] and res["rounds"] == 20, res
