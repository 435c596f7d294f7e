"""BASELINE config 1 on the reference's own shipped data: FS-Classification, 2 sites, dSGD, CPU/gloo.

The reference publishes a dSGD test AUC of 0.814 for its 2-site ``fs-lstm_2S`` run
(``/root/reference/nnlogs.ipynb:56``; the data behind that run is unstated).  This runs
``datasets/test_fsl`` sites 0 and 1 through the launcher exactly as ``tools/fs_parity.py`` does
(10-fold, compspec defaults: epochs 101, patience 35, batch 16, lr 1e-3) and asserts that the
global test AUC, averaged over the folds, clears 0.75.  Full matrix: ``profiles/fs_parity.md``.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = "/root/reference/datasets/test_fsl"


@pytest.mark.slow
@pytest.mark.skipif(not os.path.isdir(DATA), reason="reference FS data not present")
def test_fs_two_site_dsgd_auc(tmp_path):
    sys.path.insert(0, ROOT)
    from mp_util import free_port
    from dinunet_implementations_amd.utils import analysis
    out = str(tmp_path / "out")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           "-m", "dinunet_implementations_amd.run", "--data-path", DATA, "--out", out,
           "--device", "cpu", "--set", "agg_engine=dSGD", "--set", "num_folds=10"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rep = analysis.fold_report(out)
    assert len(rep["folds"]) == 10
    auc = rep["summary"]["AUC"]["mean"]
    assert auc > 0.75, rep["summary"]
    # early stopping engaged: every fold stopped before the 101-epoch cap
    assert rep["summary"]["best_val_epoch"]["max"] < 101
