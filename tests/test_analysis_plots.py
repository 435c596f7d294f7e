"""utils.analysis.plot_boxes: the reference notebook's perf_box / pretrain_box figures
(NB.ipynb:131-189) from per-fold tables."""
import os

from dinunet_implementations_amd.utils.analysis import plot_boxes


def test_plot_boxes_writes_both_figures(tmp_path):
    folds = {m: [{"fold": k, "Accuracy": 0.8 + 0.01 * k, "F1": 0.75 + 0.01 * k,
                  "best_val_epoch": e + k} for k in range(10)]
             for m, e in (("scratch", 40), ("pretrain", 25))}
    perf, ep = str(tmp_path / "perf_box.png"), str(tmp_path / "pretrain_box.png")
    plot_boxes(folds, perf, ep)
    for p in (perf, ep):
        assert os.path.getsize(p) > 5000
        with open(p, "rb") as f:
            assert f.read(8) == b"\x89PNG\r\n\x1a\n"
