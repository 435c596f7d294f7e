"""The peer exchange (``parallel.peer``, ``csrc/kernels/peer.hip``) with real cross-process device
traffic: 2 / 4 site processes share one MI355X, map each other's uncached arenas through IPC
handles and run the site-mean (every wire type) and the factor all-gather eagerly and inside a
captured HIP graph replayed with fresh data, against an fp64 reference; every replica must hold
the bit-identical mean (``tools/peer_check.py``)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,wire,wait", [(2, "all", "launch"), (4, "fp16", "launch"),
                                             (4, "all", "inline")])
def test_peer_exchange_multiprocess(world, wire, wait):
    """``wait``: the waits as one-workgroup launches of their own (what sites sharing a GPU use)
    or inside the data launches (one site per GPU, production; safe here: no other kernels)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from mp_util import free_port
    env = dict(os.environ, DINUNET_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
               DINUNET_PEER_TIMEOUT_MS="20000", DINUNET_PEER_WAIT=wait)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(world), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tools", "peer_check.py"), "--wire", wire, "--reps", "3"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(lines[-1])
    log = os.environ.get("DINUNET_ERR_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": "peer", **res}) + "\n")
    assert res["ok"], res
    assert r.returncode == 0, r.stderr[-3000:]
