"""Multi-site correctness on the GPU: 2 and 4 ranks share one MI355X over gloo
(``DINUNET_BACKEND=gloo``), train through the production HIP-graph TrainStep with every engine,
both payload precisions, a ragged batch on one rank (eager step beside graph replays: the dSGD
bucket launch order must still agree) and local_iterations = 2; all replicas must end
bit-identical (``tools/multirank_check.py``).  Each case is a fresh ``torch.distributed.run``
started before any GPU use in this process's children."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    (2, ["--engine", "dSGD", "--precision", "32"]),
    (2, ["--engine", "dSGD", "--precision", "16", "--ragged"]),
    (2, ["--engine", "dSGD", "--precision", "32", "--accum", "2", "--ragged"]),
    (2, ["--engine", "rankDAD", "--precision", "32", "--ragged"]),
    (2, ["--engine", "powerSGD", "--precision", "16", "--accum", "2"]),
    (4, ["--engine", "dSGD", "--precision", "16", "--accum", "2", "--ragged"]),
    (4, ["--engine", "rankDAD", "--precision", "16"]),
    # against the fp64 oracle of each engine (tools/multirank_check.py --oracle: every site's own
    # gradient, the engine's reduction replayed in fp64).  --grad-tol bounds the FIRST step's
    # reduced gradient (the engine / payload error itself); --oracle-tol bounds the 8-step
    # parameter update, which Adam amplifies (a near-zero mean gradient's sign becomes a full lr
    # step).  Tolerances are ~2-4x the values observed on MI355X (profiles/r4_oracle_obs.jsonl):
    # dSGD fp32 grad 2.2e-8 / update 5.5e-8; fp16 3.0e-4 / 0.12; bf16 2.3e-3 / 0.11;
    # rank-dAD fp32 2.7e-7 (w2) 3.2e-7 (w3) / 0.11-0.18, fp16 2.7e-4 / 0.25;
    # PowerSGD fp32 2.1e-7 / 0.10, fp16 3.7e-4 / 0.17
    (2, ["--engine", "dSGD", "--precision", "32", "--oracle"]),
    (3, ["--engine", "dSGD", "--precision", "16", "--oracle", "--ragged", "--oracle-tol", "0.3",
         "--grad-tol", "1e-3"]),
    (2, ["--engine", "dSGD", "--precision", "16", "--payload", "bf16", "--oracle",
         "--oracle-tol", "0.3", "--grad-tol", "6e-3"]),
    (2, ["--engine", "dSGD", "--precision", "16", "--collective", "allreduce", "--oracle",
         "--oracle-tol", "0.3", "--grad-tol", "6e-3"]),
    (2, ["--engine", "rankDAD", "--precision", "32", "--dad-tol", "0", "--oracle",
         "--grad-tol", "1e-6", "--oracle-tol", "0.4"]),
    (3, ["--engine", "rankDAD", "--precision", "32", "--dad-tol", "0", "--oracle",
         "--grad-tol", "1e-6", "--oracle-tol", "0.45"]),
    (2, ["--engine", "rankDAD", "--precision", "16", "--dad-tol", "0", "--oracle",
         "--grad-tol", "8e-4", "--oracle-tol", "0.5"]),
    (2, ["--engine", "powerSGD", "--precision", "32", "--oracle", "--grad-tol", "1e-6",
         "--oracle-tol", "0.25"]),
    (3, ["--engine", "powerSGD", "--precision", "32", "--oracle", "--grad-tol", "1e-6",
         "--oracle-tol", "0.25"]),
    (2, ["--engine", "powerSGD", "--precision", "16", "--oracle", "--grad-tol", "1e-3",
         "--oracle-tol", "0.35"]),
    (2, ["--engine", "powerSGD", "--precision", "32", "--accum", "2", "--oracle",
         "--grad-tol", "1e-6", "--oracle-tol", "0.25"]),
    # the bench path across sites: HBM-resident batches, split capture, the fused Adam emitting
    # the next step's operands after the all-reduce
    (2, ["--engine", "dSGD", "--precision", "32", "--feed", "device", "--oracle"]),
    (3, ["--engine", "dSGD", "--precision", "16", "--feed", "device", "--oracle",
         "--oracle-tol", "0.3"]),
    # device-fed low-rank engines across sites (host-issued collectives: each replay's local
    # factorisation must run in the engine's reduction -- it once did not)
    (2, ["--engine", "rankDAD", "--precision", "32", "--dad-tol", "0", "--feed", "device",
         "--oracle", "--grad-tol", "1e-6", "--oracle-tol", "0.4"]),
    (2, ["--engine", "powerSGD", "--precision", "32", "--feed", "device", "--oracle",
         "--grad-tol", "1e-6", "--oracle-tol", "0.25"]),
    # the peer exchange (parallel/peer.py): real cross-process device traffic through IPC-mapped
    # HBM INSIDE the captured step (comm_graph on the gloo group too: kernels only), every engine
    # and wire against the fp64 oracle; 16-bit wires take it by default (auto)
    (2, ["--engine", "dSGD", "--precision", "32", "--collective", "peer", "--oracle"]),
    (2, ["--engine", "dSGD", "--precision", "32", "--collective", "peer", "--feed", "device",
         "--oracle"]),
    # (4 sites, fp32: the first-step gradient matches the fp64 mean to 3.4e-8 -- peer and gloo
    # all-reduce alike -- and Adam amplifies the fp32 sum-order difference to a 5.0-5.4e-2
    # update error after 8 steps for both, profiles/r6_peer_oracle_w4.jsonl)
    (4, ["--engine", "dSGD", "--precision", "32", "--collective", "peer", "--oracle",
         "--oracle-tol", "0.15", "--grad-tol", "1e-7"]),
    (4, ["--engine", "dSGD", "--precision", "32", "--collective", "peer", "--feed", "device",
         "--oracle", "--oracle-tol", "0.15"]),
    (2, ["--engine", "dSGD", "--precision", "16", "--collective", "peer", "--payload", "bf16",
         "--oracle", "--oracle-tol", "0.3", "--grad-tol", "6e-3"]),
    (2, ["--engine", "rankDAD", "--precision", "32", "--collective", "peer", "--dad-tol", "0",
         "--oracle", "--grad-tol", "1e-6", "--oracle-tol", "0.4"]),
    (2, ["--engine", "rankDAD", "--precision", "16", "--dad-tol", "0", "--feed", "device",
         "--oracle", "--oracle-tol", "0.5"]),
    (2, ["--engine", "powerSGD", "--precision", "32", "--collective", "peer", "--oracle",
         "--grad-tol", "1e-6", "--oracle-tol", "0.25"]),
    (2, ["--engine", "powerSGD", "--precision", "16", "--feed", "device", "--oracle",
         "--oracle-tol", "0.35"]),
    # device-fed accumulation (local_iterations = 2): host collectives after the replay (gloo
    # all-reduce: the captured micro-batches keep them off) and the captured peer exchange
    (2, ["--engine", "dSGD", "--precision", "32", "--feed", "device", "--accum", "2",
         "--oracle"]),
    (2, ["--engine", "dSGD", "--precision", "16", "--feed", "device", "--accum", "2",
         "--oracle", "--oracle-tol", "0.3"]),
]


@pytest.mark.parametrize("world,args", CASES, ids=[f"w{w}-" + "-".join(x for x in a if not x.startswith("--")) +
                                                   ("-ragged" if "--ragged" in a else "") + ("-oracle" if "--oracle" in a else "")
                                                   for w, a in CASES])
def test_replicas_bit_identical(world, args):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from mp_util import free_port
    env = dict(os.environ, DINUNET_BACKEND="gloo", PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(world), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "tools", "multirank_check.py")] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(lines[-1])
    log = os.environ.get("DINUNET_ERR_LOG")
    if log:
        with open(log, "a") as f:
            f.write(json.dumps({"test": "multirank", "args": args, **res}) + "\n")
    assert res["ok"], res
    if "--oracle" in args:  # the oracle ran and judged the update (and, host-fed, the gradient)
        assert res.get("oracle_ok") is True, res
        if "device" not in args:  # (device-fed: the fused Adam zeroes the gradient it consumes)
            assert "grad_rel_err" in res, res
    assert res["graph"] and res["world"] == world
    if "device" in args and "dSGD" in args and "--accum" not in args:  # the bench path: the
        assert res["adam_pack"], res  # update emits the next step's operands
        # split backward with the all-reduce; the peer exchange runs the whole step unsplit
        assert res["split"] == (not res["peer"]), res
    if "peer" in args or ("16" in args and "allreduce" not in args):  # the peer exchange, captured
        assert res["peer"] and (res["comm_graph"] or "--accum" in args), res
        if "--accum" not in args or "device" in args:  # (host-fed accumulation: eager update)
            assert res["captured_update"], res
    assert r.returncode == 0, r.stderr[-3000:]
