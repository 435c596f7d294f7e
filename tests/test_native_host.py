"""C++ host runtime (csrc/host/dataio.cpp) against the Python reference implementations."""
import os

import numpy as np
import pytest
import torch

from dinunet_implementations_amd.data import native

pytestmark = pytest.mark.skipif(not native.available(), reason="host library not built")


def test_fs_load_matches_python_parse(fs_data_root):
    from dinunet_implementations_amd.tasks.fs import read_stats_file
    d = os.path.join(fs_data_root, "input", "local0", "simulatorRun")
    files = sorted(f for f in os.listdir(d) if f.endswith("_aseg_stats.txt"))[:40]
    paths = [os.path.join(d, f) for f in files]
    got = native.fs_load(paths, 66)
    ref = []
    for p in paths:
        _, v = read_stats_file(p)
        v = np.asarray(v, dtype=np.float64)
        ref.append((v / v.max()).astype(np.float32))
    assert np.array_equal(got, np.stack(ref))


def test_fs_load_reports_bad_file(tmp_path):
    good = tmp_path / "a.txt"
    good.write_text("Measure:volume\tA\nx\t1.0\ny\t2.0\n")
    short = tmp_path / "b.txt"
    short.write_text("Measure:volume\tB\nx\t1.0\n")
    with pytest.raises(ValueError, match="fewer than 2"):
        native.fs_load([str(good), str(short)], 2)
    with pytest.raises(ValueError, match="cannot be read"):
        native.fs_load([str(tmp_path / "missing.txt")], 2)


@pytest.mark.parametrize("W,stride,T,temporal", [(10, 10, 980, 980), (20, 10, 980, 980),
                                                 (5, 3, 61, 60)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_ica_windows_match_reference(W, stride, T, temporal, dtype):
    from dinunet_implementations_amd.ops.reference import ica_windows
    rng = np.random.default_rng(0)
    src = rng.standard_normal((7, 6, T)).astype(dtype)
    ref = ica_windows(torch.from_numpy(src.astype(np.float32)), W, stride, temporal).numpy()
    assert np.array_equal(native.ica_windows(src, W, stride, temporal), ref)
    rows = np.array([5, 0, 3])
    assert np.array_equal(native.ica_windows(src, W, stride, temporal, rows), ref[rows])


def test_roc_auc_and_confusion_match_python():
    from dinunet_implementations_amd.utils.metrics import roc_auc_py
    rng = np.random.default_rng(1)
    for n in (1, 7, 500):
        s = np.round(rng.random(n), 2)  # ties
        y = rng.integers(0, 2, n)
        assert abs(native.roc_auc(s, y) - roc_auc_py(s, y)) < 1e-12
    p, y = rng.integers(0, 2, 300), rng.integers(0, 2, 300)
    tn, fp, fn, tp = native.confusion2(p, y)
    assert (tn, fp, fn, tp) == (((p == 0) & (y == 0)).sum(), ((p == 1) & (y == 0)).sum(),
                                ((p == 0) & (y == 1)).sum(), ((p == 1) & (y == 1)).sum())
