"""Run-analysis library (the reference notebooks' numbers) over a synthetic output tree."""
import json
import os

from dinunet_implementations_amd.utils import analysis
from dinunet_implementations_amd.utils import logs as L


def _tree(tmp_path, epochs, accs, engine="dSGD"):
    out = str(tmp_path)
    for fold, (ep, acc) in enumerate(zip(epochs, accs)):
        for site in ("local0", "local1", "remote"):
            d = L.fold_dir(out, site, "FS-Classification", fold)
            logs = {"agg_engine": engine, "best_val_epoch": ep, "cumulative_total_duration": [1.0, 2.0],
                    "time_spent_on_computation": [0.5, 0.25],
                    ("remote_iter_duration" if site == "remote" else "local_iter_duration"): [0.1, 0.3],
                    "test_metrics": [0.5, acc, acc, acc, acc, 0.9]}
            L.write_logs(d, logs)
            L.write_test_metrics(d, [logs["test_metrics"]])
    return out


def test_fold_report_summary(tmp_path):
    out = _tree(tmp_path, [10, 20, 30, 40], [0.8, 0.9, 0.85, 0.95])
    r = analysis.fold_report(out)
    assert [f["fold"] for f in r["folds"]] == [0, 1, 2, 3]
    s = r["summary"]
    assert abs(s["best_val_epoch"]["mean"] - 25.0) < 1e-9
    assert abs(s["Accuracy"]["median"] - 0.875) < 1e-9
    assert s["AUC"]["min"] == 0.9


def test_engine_and_iteration_reports(tmp_path):
    out = _tree(tmp_path, [5], [0.9], engine="rankDAD")
    er = analysis.engine_report(out)
    assert {r["site"] for r in er} == {"local0", "local1", "remote"}
    assert all(r["agg_engine"] == "rankDAD" and abs(r["cumulative_total_s"] - 3.0) < 1e-9 for r in er)
    ir = analysis.iteration_report(out)
    assert abs(ir["remote/fold_0"]["mean"] - 0.2) < 1e-9
    md = analysis.report_markdown(out)
    assert "best_val_epoch" in md and "rankDAD" in md


def test_compare_and_zip_extract(tmp_path):
    a = _tree(tmp_path / "a", [60, 70], [0.9, 0.9])
    b = _tree(tmp_path / "b", [40, 45], [0.92, 0.9])
    c = analysis.compare(a, b)
    assert c["a"]["best_val_epoch"]["mean"] > c["b"]["best_val_epoch"]["mean"]
    rdir = os.path.join(a, "remote", "FS-Classification", "fold_0")
    L.zip_results(rdir, os.path.join(rdir, "res.zip"))
    dst = analysis.extract_zips(a)
    assert dst and os.path.exists(os.path.join(dst[0], "logs.json"))
    assert json.load(open(os.path.join(dst[0], "logs.json")))["agg_engine"] == "dSGD"
