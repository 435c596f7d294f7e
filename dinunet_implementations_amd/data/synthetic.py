"""Synthetic site data with the reference formats.

* FS: per-site ``inputspec.json`` + ``input/local<i>/simulatorRun/`` holding a covariate CSV
  ``freesurferfile,isControl,age`` and one ``subjectN_aseg_stats.txt`` per subject (header +
  66 ``region\\tvolume`` rows), with a weak class signal so AUC can rise above 0.5.
* ICA: ``[N, C, T]`` float32 ``.npy`` of band-limited "time courses" whose spectrum depends on
  the label in a subset of components, plus a labels CSV of ``[data_index, label]`` rows (the
  real dataset is git-ignored in the reference, ``.gitignore:123``).
"""
from __future__ import annotations

import csv
import json
import os
from typing import Dict, Optional, Sequence

import numpy as np

FS_REGIONS = 66


def make_fs_sites(root: str, sites: int = 2, subjects: Sequence[int] = (40, 40), seed: int = 0,
                  signal: float = 0.35) -> str:
    rng = np.random.default_rng(seed)
    base_vol = rng.uniform(2e3, 5e4, FS_REGIONS)
    base_vol[-1] = 1.6e6  # MaskVol: always the per-subject max (quirk A8)
    effect = rng.normal(0, 1, FS_REGIONS) * (rng.random(FS_REGIONS) < 0.3)
    specs = []
    for s in range(sites):
        d = os.path.join(root, "input", f"local{s}", "simulatorRun")
        os.makedirs(d, exist_ok=True)
        n = subjects[s % len(subjects)]
        cov = f"site{s + 1}_Covariate.csv"
        rows = []
        for j in range(n):
            y = bool(rng.random() < 0.5)
            vol = base_vol * (1 + 0.08 * rng.normal(size=FS_REGIONS) + signal * 0.1 * effect * (1 if y else -1))
            vol[-1] = base_vol[-1] * (1 + 0.02 * rng.normal())
            fn = f"subject{j}_aseg_stats.txt"
            with open(os.path.join(d, fn), "w") as f:
                f.write(f"Measure:volume\tsubject{j}\n")
                for k in range(FS_REGIONS):
                    f.write(f"Region-{k}\t{vol[k]:.2f}\n")
            rows.append([fn, str(y), f"{rng.uniform(20, 80):.1f}"])
        with open(os.path.join(d, cov), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["freesurferfile", "isControl", "age"])
            w.writerows(rows)
        specs.append({"labels_file": {"value": cov}, "data_column": {"value": "freesurferfile"},
                      "labels_column": {"value": "isControl"}, "mode": {"value": "train"},
                      "gpus": {"value": []}, "input_size": {"value": FS_REGIONS},
                      "hidden_sizes": {"value": [256, 128, 64, 32]}, "num_class": {"value": 2},
                      "num_workers": {"value": 0}, "learning_rate": {"value": 0.001}})
    with open(os.path.join(root, "inputspec.json"), "w") as f:
        json.dump(specs, f, indent=1)
    return root


def ica_timecourses(n: int, comps: int = 100, T: int = 980, seed: int = 0, signal: float = 0.6,
                    labels: Optional[np.ndarray] = None):
    """``[n, comps, T]`` float32 + labels; label-dependent oscillation in 10% of components."""
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 2, n) if labels is None else np.asarray(labels)
    t = np.arange(T, dtype=np.float32)
    x = rng.normal(0, 1, (n, comps, T)).astype(np.float32)
    # temporal smoothing (AR(1)) so windows carry structure
    for k in range(1, T):
        x[:, :, k] = 0.6 * x[:, :, k - 1] + 0.8 * x[:, :, k]
    sel = rng.choice(comps, max(1, comps // 10), replace=False)
    freq = np.where(y == 1, 0.05, 0.02).astype(np.float32)
    phase = rng.uniform(0, 2 * np.pi, (n, 1)).astype(np.float32)
    osc = np.sin(2 * np.pi * freq[:, None] * t[None, :] + phase)
    x[:, sel, :] += signal * osc[:, None, :].astype(np.float32)
    x = (x - x.mean(-1, keepdims=True)) / (x.std(-1, keepdims=True) + 1e-6)
    return x.astype(np.float32), y.astype(np.int64)


def ica_cohort_hard(n: int, comps: int = 100, T: int = 980, seed: int = 0, site: int = 0,
                    signal: float = 0.5, label_noise: float = 0.1, n_net: int = 8,
                    cohort_seed: int = 7):
    """A cohort where the label is a CONNECTIVITY pattern, not a spectral one (time-to-AUC and
    fidelity benchmarks; the easy :func:`ica_timecourses` is separable within ~30 steps).

    * Both classes carry the same oscillation power in the ``n_net`` network components (subject
      frequency ~ U(0.02, 0.06), so the spectrum says nothing about the label).  In class 1 one
      latent oscillation drives all of them with cohort-fixed loadings (coherent network); in
      class 0 every component oscillates with its own phase.
    * Subject-level nuisance: AR(1) coefficient ~ N(0.55, 0.1) per subject.
    * Site shift: per-site component gains (log-normal, sigma 0.3) and a site-specific mean AR
      coefficient offset, applied before the per-component standardisation.
    * ``label_noise`` of the labels are flipped (caps the attainable AUC below 1).
    The network components and loadings depend only on ``cohort_seed`` (shared by all sites)."""
    crng = np.random.default_rng(cohort_seed)
    net = crng.choice(comps, n_net, replace=False)
    load = crng.choice([-1.0, 1.0], n_net) * crng.uniform(0.7, 1.3, n_net)
    srng = np.random.default_rng(cohort_seed * 1000 + site + 1)
    gain = np.exp(srng.normal(0, 0.3, comps)).astype(np.float32)
    ar_site = srng.normal(0, 0.05)
    rng = np.random.default_rng(seed)
    y_true = rng.integers(0, 2, n)
    ar = np.clip(rng.normal(0.55 + ar_site, 0.1, (n, 1)), 0.05, 0.9).astype(np.float32)
    x = rng.normal(0, 1, (n, comps, T)).astype(np.float32)
    # the AR(1) recursion on a time-major copy (contiguous slabs; 3x faster, same values)
    xt = np.ascontiguousarray(x.transpose(2, 0, 1))
    del x
    for k in range(1, T):
        xt[k] = ar * xt[k - 1] + xt[k]
    x = np.ascontiguousarray(xt.transpose(1, 2, 0))
    del xt
    x /= np.sqrt(1.0 / (1.0 - ar[:, :, None] ** 2))  # unit variance noise
    t = np.arange(T, dtype=np.float32)
    f = rng.uniform(0.02, 0.06, (n, 1, 1)).astype(np.float32)
    shared = rng.uniform(0, 2 * np.pi, (n, 1, 1))
    own = rng.uniform(0, 2 * np.pi, (n, n_net, 1))
    phase = np.where(y_true[:, None, None] == 1, shared, own).astype(np.float32)
    osc = np.sin(2 * np.pi * f * t[None, None, :] + phase)
    x[:, net, :] += signal * load[None, :, None].astype(np.float32) * osc
    x *= gain[None, :, None]
    x = (x - x.mean(-1, keepdims=True)) / (x.std(-1, keepdims=True) + 1e-6)
    flip = rng.random(n) < label_noise
    y = np.where(flip, 1 - y_true, y_true)
    return x.astype(np.float32), y.astype(np.int64)


def make_ica_sites(root: str, sites: int = 2, subjects: Sequence[int] = (64, 64), comps: int = 100,
                   T: int = 980, seed: int = 0, window_size: int = 10, window_stride: int = 10,
                   hidden_size: int = 384, input_size: int = 256, cohort: str = "easy",
                   **cohort_kw) -> str:
    """Per-site ICA data + inputspec in the reference layout; ``cohort="hard"`` draws
    :func:`ica_cohort_hard` (site-shifted, connectivity labels, label noise)."""
    specs = []
    for s in range(sites):
        d = os.path.join(root, "input", f"local{s}", "simulatorRun")
        os.makedirs(d, exist_ok=True)
        n = subjects[s % len(subjects)]
        if cohort == "hard":
            x, y = ica_cohort_hard(n, comps, T, seed=seed * 100 + s, site=s, **cohort_kw)
        else:
            x, y = ica_timecourses(n, comps, T, seed=seed * 100 + s)
        np.save(os.path.join(d, "ica_data.npy"), x)
        with open(os.path.join(d, "labels.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["data_index", "label"])
            w.writerows([[i, int(v)] for i, v in enumerate(y)])
        specs.append({"task_id": {"value": "ICA-Classification"}, "mode": {"value": "train"},
                      "gpus": {"value": [s]}, "num_class": {"value": 2},
                      "learning_rate": {"value": 0.001}, "data_file": {"value": "ica_data.npy"},
                      "labels_file": {"value": "labels.csv"}, "input_size": {"value": input_size},
                      "hidden_size": {"value": hidden_size}, "window_size": {"value": window_size},
                      "window_stride": {"value": window_stride}, "temporal_size": {"value": T},
                      "num_components": {"value": comps}})
    with open(os.path.join(root, "inputspec.json"), "w") as f:
        json.dump(specs, f, indent=1)
    return root
