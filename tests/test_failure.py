"""Failure path: a site that dies mid-epoch makes the surviving sites stop with a
non-zero exit and a failure report, within the configured collective timeout, instead of hanging.

Two independent site processes (no torchrun agent, which would kill the survivors itself) train
FS-Classification over gloo on the CPU; ``DINUNET_FAULT=1:25`` SIGKILLs site 1 before its 25th
training step.
"""
import os
import signal
import subprocess
import sys
import time

from mp_util import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dead_site_makes_survivor_exit_nonzero(fs_data_root, tmp_path):
    port = free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="1", DINUNET_FAULT="1:25", DINUNET_PG_TIMEOUT="30")
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "dinunet_implementations_amd.run", "--data-path", fs_data_root,
             "--out", str(tmp_path / "out"), "--device", "cpu", "--set", "epochs=50",
             "--set", "patience=100"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    try:
        outs = [p.communicate(timeout=120) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    assert procs[1].returncode == -signal.SIGKILL, (procs[1].returncode, outs[1][1][-2000:])
    assert procs[0].returncode == 3, (procs[0].returncode, outs[0][1][-3000:])
    assert "site failure" in outs[0][1]
    assert elapsed < 90


import pytest  # noqa: E402


@pytest.mark.parametrize("store_wait", [True, False])
def test_pretrain_longer_than_collective_timeout(fs_data_root, tmp_path, store_wait):
    """The sites that do not pretrain wait for the pretraining site on the process group's store
    (its own deadline), not inside the weight broadcast: a pretraining phase much longer than
    ``collective_timeout_s`` (2 s here, pretraining held 8 s) must not make them time out."""
    port = free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="1", DINUNET_PRETRAIN_DELAY_S="8",
                   DINUNET_PRETRAIN_STORE_WAIT="1" if store_wait else "0")
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "dinunet_implementations_amd.run", "--data-path", fs_data_root,
             "--out", str(tmp_path / "out"), "--device", "cpu", "--set", "epochs=2",
             "--set", "pretrain=true", "--set", 'pretrain_args={"epochs": 1}',
             "--set", "collective_timeout_s=2"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        outs = [p.communicate(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    if not store_wait:  # negative control: the idle site's broadcast times out
        assert procs[1].returncode == 3, (procs[1].returncode, outs[1][1][-3000:])
        return
    for r, p in enumerate(procs):
        assert p.returncode == 0, (r, p.returncode, outs[r][1][-3000:])


@pytest.mark.parametrize("how", ["kill", "raise"])
def test_pretraining_site_failure_ends_the_wait(tmp_path, how):
    """The pretraining site is rank 1 (the larger site), NOT the store host: when it is killed
    mid-pretraining its heartbeat stops and the waiting site raises after collective_timeout_s of
    silence; when pretraining raises, it publishes the failure and the waiter raises at once.
    Either way the waiter exits non-zero long before pretrain_timeout_s (7 days)."""
    from dinunet_implementations_amd.data.synthetic import make_fs_sites
    root = make_fs_sites(str(tmp_path / "fs"), sites=2, subjects=(24, 48), seed=1)
    port = free_port()
    procs = []
    fault = "1:3" + (":raise" if how == "raise" else "")
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="1", DINUNET_FAULT=fault)
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "dinunet_implementations_amd.run", "--data-path", root,
             "--out", str(tmp_path / "out"), "--device", "cpu", "--set", "epochs=2",
             "--set", "pretrain=true", "--set", 'pretrain_args={"epochs": 50}',
             "--set", "collective_timeout_s=4", "--set", "pretrain_heartbeat_s=0.5"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    try:
        outs = [p.communicate(timeout=120) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.time() - t0
    if how == "kill":
        assert procs[1].returncode == -signal.SIGKILL, (procs[1].returncode, outs[1][1][-2000:])
        assert "stopped signalling" in outs[0][1], outs[0][1][-3000:]
    else:
        assert procs[1].returncode == 3, (procs[1].returncode, outs[1][1][-2000:])
        assert "injected site failure" in outs[0][1], outs[0][1][-3000:]
    assert procs[0].returncode == 3, (procs[0].returncode, outs[0][1][-3000:])
    assert elapsed < 90
