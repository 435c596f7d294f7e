"""Configuration: compspec/inputspec loading, defaults, precedence and ``<task>_args`` flattening.

Parity targets (reference behaviour, reconstructed in SURVEY.md §2.7 / §5.6):

* ``compspec.json:14-282`` declares every GUI parameter with a default.  The per-site
  ``inputspec.json`` (``datasets/test_fsl/inputspec.json``) is a JSON *list* with one
  ``{key: {"value": v}}`` object per site.
* ``local.py:31-37`` passes code defaults as ``COINNLocal`` kwargs; values delivered in
  ``data['input']`` override them (dispatch reads ``cache['task_id']`` at ``local.py:40``).
* Task-specific objects ``<task_id>_args`` (``compspec.json:225-281``) are flattened into the
  single cache dict that trainers read (``comps/fs/__init__.py:47`` reads ``cache['input_size']``).
* The compspec's ICA block uses names the ICA code never reads (``seq_len``,
  ``full_comp_size``); the code reads ``temporal_size``/``num_components``
  (``comps/icalstm/__init__.py:21-24``).  We accept both and map the compspec names onto the
  code names so compspec-only ICA runs no longer ``KeyError`` (SURVEY.md §2.7 "Mismatch").

Precedence (lowest → highest): framework defaults < compspec defaults < constructor kwargs <
site input (inputspec / COINSTAC message) < explicit overrides.
"""
from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, Iterable, List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
COMPSPEC_PATH = os.path.join(_HERE, "compspec.json")

TASK_FS = "FS-Classification"
TASK_ICA = "ICA-Classification"

# Framework defaults: the union of every key the reference reads or declares.
# Where the reference disagrees with itself (epochs 101 vs 21, patience 35 vs 31) the compspec
# value wins, matching the GUI-visible contract; ``local.py``-style callers still pass their own
# kwargs on top.
FRAMEWORK_DEFAULTS: Dict[str, Any] = {
    "task_id": TASK_FS,
    "mode": "train",
    "agg_engine": "dSGD",
    "num_reducers": 2,
    "batch_size": 16,
    "local_iterations": 1,
    "learning_rate": 1e-3,
    "epochs": 101,
    "pretrain": False,
    "pretrain_args": {
        "epochs": 0, "learning_rate": 1e-3, "batch_size": 16, "local_iterations": 1,
        "validation_epochs": 1, "pin_memory": False, "num_workers": 0, "patience": 51,
    },
    "validation_epochs": 1,
    "precision_bits": "32",
    "pin_memory": False,
    "num_workers": 0,
    "patience": 35,
    "split_ratio": [0.8, 0.1, 0.1],
    "num_folds": None,
    "split_files": [],
    "dataloader_args": {"train": {"drop_last": True}},
    "num_class": 2,
    "monitor_metric": "auc",
    "metric_direction": "maximize",
    "log_header": "loss|auc",
    "seed": 0,
    # GPU ids of a site (inputspec "gpus"): None = this process's GPU, [] = CPU, [k] = GPU k
    # (parallel.group.resolve_device)
    "gpus": None,
    # rank-dAD / PowerSGD knobs (compspec.json:236-238, 268-270)
    "dad_reduction_rank": 10,
    "dad_num_pow_iters": 5,
    "dad_tol": 1e-3,
    "powersgd_rank": 4,
    "powersgd_warm_start": True,
    # collective plan for the xGMI mesh (README "Collective plan"): dSGD bucket size, RCCL
    # algorithm / protocol (None = RCCL's own choice), per-collective timeout
    "dsgd_bucket_mb": 4.0,
    "rccl_algo": None,
    "rccl_proto": None,
    "collective_timeout_s": 1800,
    # the non-pretraining sites' wait for the pretraining site (not a collective: see
    # runtime.site.FederatedSite._await_pretrain)
    "pretrain_timeout_s": 7 * 86400,
    # the pretraining site's heartbeat period (None: collective_timeout_s / 4, 0.5-30 s); a site
    # silent for collective_timeout_s ends the wait with an error
    "pretrain_heartbeat_s": None,
    # site loop: train epochs device-fed (runtime.feed: HBM-resident bf16 split, K-step graphs,
    # on-device train records) when the step supports it
    "device_feed": True,
    # classifier / MLP normalisation: "batch" = the reference's BatchNorm1d, "layer" = the
    # optional LayerNorm on its own gfx950 kernels (ops.layernorm)
    "norm_layer": "batch",
    # "fused": gfx950 kernels (bf16 MFMA operands, fp32 accumulation / state);
    # "reference": the fp32 oracle math of ops/reference.py on the same device (fidelity baseline)
    "compute_path": "fused",
}

TASK_DEFAULTS: Dict[str, Dict[str, Any]] = {
    TASK_FS: {
        "labels_file": "site_covariates.csv",
        "data_column": "freesurferfile",
        "labels_column": "isControl",
        "input_size": 66,
        "hidden_sizes": [256, 128, 64, 32],
        "num_class": 2,
        "dropout_in": [],
    },
    TASK_ICA: {
        "num_class": 2,
        "monitor_metric": "auc",
        "metric_direction": "maximize",
        "log_header": "Loss|AUC",
        "num_components": 100,
        "window_size": 10,
        "window_stride": 10,
        "temporal_size": 980,
        "input_size": 256,
        "hidden_size": 384,
        "num_layers": 1,
        "bidirectional": True,
        "data_file": None,
        "labels_file": None,
    },
}

# compspec ICA names -> names the ICA code reads (SURVEY.md §2.7 mismatch row).
ICA_KEY_ALIASES = {"full_comp_size": "num_components"}

# The reference compspec's input keys (``/root/reference/compspec.json:14-282``), with the keys of
# each task's args object; ``tests/test_config_data.py`` pins the generated compspec to these
# modulo the documented extras below.
REFERENCE_INPUT_KEYS = (
    "covariates", "data", "task_id", "mode", "agg_engine", "num_reducers", "batch_size",
    "local_iterations", "learning_rate", "epochs", "pretrain", "pretrain_args",
    "validation_epochs", "precision_bits", "pin_memory", "num_workers", "patience", "split_ratio",
    "num_folds", f"{TASK_FS}_args", f"{TASK_ICA}_args")
REFERENCE_TASK_ARG_KEYS = {
    TASK_FS: ("labels_column", "input_size", "hidden_sizes", "num_class", "dad_reduction_rank",
              "dad_num_pow_iters", "dad_tol", "split_files"),
    TASK_ICA: ("num_class", "monitor_metric", "metric_direction", "log_header", "full_comp_size",
               "spatial_dim", "window_size", "window_stride", "seq_len", "data_file",
               "labels_file", "components_file", "split_files", "input_size", "hidden_size",
               "dad_reduction_rank", "dad_num_pow_iters", "dad_tol"),
}
# inputs this framework adds to the GUI contract (documented in README "Configuration")
EXTRA_INPUT_KEYS = ("norm_layer",)


def unwrap_values(site_input: Dict[str, Any]) -> Dict[str, Any]:
    """Turn ``{key: {"value": v}}`` (inputspec / COINSTAC form) into ``{key: v}``.

    Plain values pass through untouched so callers may hand in either form.
    """
    out = {}
    for k, v in (site_input or {}).items():
        if isinstance(v, dict) and set(v.keys()) == {"value"}:
            out[k] = v["value"]
        else:
            out[k] = v
    return out


def load_inputspec(path: str) -> List[Dict[str, Any]]:
    """Read a simulator inputspec (one object per site, ``datasets/*/inputspec.json``)."""
    with open(path) as f:
        spec = json.load(f)
    if isinstance(spec, dict):
        spec = [spec]
    return [unwrap_values(s) for s in spec]


def load_compspec(path: Optional[str] = None) -> Dict[str, Any]:
    with open(path or COMPSPEC_PATH) as f:
        return json.load(f)


def compspec_defaults(compspec: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Default value of every declared compspec input (``compspec.json:14-282``)."""
    spec = compspec or load_compspec()
    out = {}
    for k, v in spec["computation"]["input"].items():
        if isinstance(v, dict) and "default" in v and v["default"] is not None:
            out[k] = copy.deepcopy(v["default"])
    return out


def _flatten_task_args(cfg: Dict[str, Any], user: Optional[set] = None) -> Dict[str, Any]:
    """Merge ``<task_id>_args`` of the *selected* task into the top level (E2(b)).

    ``user``: the keys the site input / overrides set (top level or inside the task args).  The
    compspec's ICA names map onto the names the ICA code reads: ``full_comp_size`` ->
    ``num_components`` and ``seq_len`` (windows per subject) -> ``temporal_size = seq_len *
    window_size`` -- when the user set the compspec name and not the code name.  ``covariates``
    (the member's covariate CSV, reference ``compspec.json:15-17``) names the FS labels file
    unless ``labels_file`` is set."""
    user = set() if user is None else user
    task = cfg.get("task_id", TASK_FS)
    flat = dict(cfg)
    args = cfg.get(f"{task}_args")
    if isinstance(args, dict):
        # task args beat framework/compspec/kwarg defaults; site input and explicit
        # overrides are re-applied on top by build_config.
        flat.update(args)
    for t in TASK_DEFAULTS:
        flat.pop(f"{t}_args", None)
    if task == TASK_ICA:
        for src, dst in ICA_KEY_ALIASES.items():
            if src in flat and (dst not in flat or (src in user and dst not in user)):
                flat[dst] = flat[src]
        # the compspec names the temporal length only as a number of windows ("seq_len")
        if "seq_len" in flat and "window_size" in flat and (
                "temporal_size" not in flat or ("seq_len" in user and "temporal_size" not in user)):
            flat["temporal_size"] = int(flat["seq_len"]) * int(flat["window_size"])
    if task == TASK_FS and "covariates" in user and "labels_file" not in user:
        flat["labels_file"] = flat["covariates"]
    return flat


def build_config(*, site_input: Optional[Dict[str, Any]] = None,
                 use_compspec: bool = True, overrides: Optional[Dict[str, Any]] = None,
                 **code_defaults: Any) -> Dict[str, Any]:
    """Produce the flat run cache for one site.

    ``code_defaults`` plays the role of the ``COINNLocal(**kw)`` kwargs (``local.py:31-37``);
    ``site_input`` is ``data['input']`` (wins over kwargs); ``overrides`` beat everything.
    """
    cfg: Dict[str, Any] = copy.deepcopy(FRAMEWORK_DEFAULTS)
    if use_compspec and os.path.exists(COMPSPEC_PATH):
        cfg.update(compspec_defaults())
    cfg.update(copy.deepcopy(code_defaults))
    site = unwrap_values(site_input or {})
    ov = dict(overrides or {})
    task = ov.get("task_id", site.get("task_id", cfg.get("task_id", TASK_FS)))
    key = f"{task}_args"
    base = copy.deepcopy(TASK_DEFAULTS.get(task, {}))
    base.update(cfg.get(key) or {})
    # a task-args object from the site / overrides refines the defaults key by key (it does not
    # drop the keys it leaves out)
    user = set()
    for src in (site, ov):
        if isinstance(src.get(key), dict):
            base.update(copy.deepcopy(src[key]))
            user.update(src[key])
        user.update(k for k in src if not k.endswith("_args"))
    cfg.update(site)
    cfg.update(ov)
    cfg[key] = base
    cfg["task_id"] = task
    flat = _flatten_task_args(cfg, user)
    # anything still explicitly present in site input / overrides wins over task args
    for src in (site, overrides or {}):
        for k, v in src.items():
            if not k.endswith("_args"):
                flat[k] = v
    return validate(flat)


def validate(cfg: Dict[str, Any]) -> Dict[str, Any]:
    eng = cfg.get("agg_engine")
    if eng not in ("dSGD", "rankDAD", "powerSGD"):
        raise ValueError(f"unknown agg_engine {eng!r} (expected dSGD|rankDAD|powerSGD)")
    if str(cfg.get("precision_bits")) not in ("16", "32"):
        raise ValueError("precision_bits must be '16' or '32'")
    cfg["precision_bits"] = str(cfg["precision_bits"])
    if cfg.get("num_folds") in (0, "", "null"):
        cfg["num_folds"] = None
    sr = cfg.get("split_ratio")
    if cfg.get("num_folds") is None and sr is not None:
        if len(sr) not in (2, 3) or abs(sum(sr) - 1.0) > 1e-6:
            raise ValueError(f"split_ratio must have 2-3 entries summing to 1, got {sr}")
    cfg["mode"] = str(cfg.get("mode", "train")).lower()
    cfg["metric_direction"] = cfg.get("metric_direction", "maximize")
    return cfg


def write_compspec(path: str) -> None:
    """Regenerate ``compspec.json`` from the framework defaults (keeps the GUI contract)."""
    with open(path, "w") as f:
        json.dump(generate_compspec(), f, indent=2)


def generate_compspec() -> Dict[str, Any]:
    order = iter(range(1, 200))

    def item(label, typ, default, source="owner", group="NN Params", conditional=None, **extra):
        d = {"label": label, "type": typ, "default": default, "source": source,
             "group": group, "order": next(order)}
        if conditional:
            d["conditional"] = conditional
        d.update(extra)
        return d

    train = {"variable": "mode", "value": "train"}
    inputs = {
        # the member's covariate CSV (FS: the labels file unless labels_file is set)
        "covariates": {"value": "site0_covariates.csv", "label": "Covariates", "type": "csv",
                       "source": "member", "group": "Data", "order": next(order)},
        "data": item("Data", "files", None, source="member", group="Data",
                     items=["Files"], extensions=[["csv", "txt", "h5", "npy", "npz"]]),
        "task_id": item("Task", "select", TASK_FS, values=[TASK_FS, TASK_ICA]),
        "mode": item("Mode", "select", "train", values=["train", "test"]),
        "agg_engine": item("Aggregation engine", "select", "dSGD", conditional=train,
                           values=["dSGD", "rankDAD", "powerSGD"]),
        "num_reducers": item("Reducer workers", "number", 2),
        "batch_size": item("Batch size", "number", 16),
        "local_iterations": item("Local iterations (grad accumulation)", "number", 1),
        "learning_rate": item("Learning rate", "number", 1e-3, conditional=train),
        "epochs": item("Epochs", "number", 101, conditional=train),
        "pretrain": item("Pretrain on the largest site", "boolean", False),
        "pretrain_args": item("Pretrain args", "object",
                              copy.deepcopy(FRAMEWORK_DEFAULTS["pretrain_args"]),
                              conditional={"variable": "pretrain", "value": True}),
        "validation_epochs": item("Validate every N epochs", "number", 1, conditional=train),
        "precision_bits": item("Payload precision bits", "select", "32", conditional=train,
                               values=["32", "16"]),
        "norm_layer": item("Classifier normalisation", "select", "batch",
                           values=["batch", "layer"]),
        "pin_memory": item("Pin memory", "boolean", False, source="member"),
        "num_workers": item("Loader workers", "number", 0, source="member"),
        "patience": item("Early-stopping patience", "number", 35, conditional=train),
        "split_ratio": item("Train/val/test split ratio", "object", [0.8, 0.1, 0.1]),
        "num_folds": item("K-fold (overrides split ratio)", "number", None),
        f"{TASK_FS}_args": item("FreeSurfer args", "object", {
            "labels_column": "isControl", "input_size": 66, "hidden_sizes": [256, 128, 64, 32],
            "num_class": 2, "dad_reduction_rank": 10, "dad_num_pow_iters": 5, "dad_tol": 1e-3,
            "split_files": []}, group="Computation",
            conditional={"variable": "task_id", "value": TASK_FS}),
        # the reference's ICA key set (compspec names: full_comp_size -> num_components,
        # seq_len windows -> temporal_size = seq_len * window_size) on the inputspec geometry
        # (datasets/icalstm/inputspec.json: 100 components, W = stride = 10, T = 980)
        f"{TASK_ICA}_args": item("ICA args", "object", {
            "num_class": 2, "monitor_metric": "auc", "metric_direction": "maximize",
            "log_header": "Loss|AUC", "full_comp_size": 100, "spatial_dim": 140,
            "window_size": 10, "window_stride": 10, "seq_len": 98,
            "data_file": "<Required!>", "labels_file": "<Required!>", "components_file": "",
            "split_files": [], "input_size": 256, "hidden_size": 384, "dad_reduction_rank": 10,
            "dad_num_pow_iters": 5, "dad_tol": 1e-3}, group="Computation",
            conditional={"variable": "task_id", "value": TASK_ICA}),
    }
    return {
        "meta": {
            "name": "Decentralized deep neural networks (MI355X-native dinunet)",
            "id": "dinunet-mi355x",
            "version": "v0.1.0",
            "repository": "local",
            "description": "FS-MLP / ICA-LSTM across sites with dSGD, rank-dAD or PowerSGD; "
                           "one MI355X per site, RCCL collectives over xGMI.",
        },
        "computation": {
            "type": "docker",
            "dockerImage": "dinunet-mi355x",
            "command": ["python", "entry.py"],
            "remote": {"type": "docker", "dockerImage": "dinunet-mi355x",
                       "command": ["python", "entry.py"]},
            "input": inputs,
            "output": {},
            "display": {},
        },
    }


def site_seed(cfg: Dict[str, Any], rank: int) -> int:
    return int(cfg.get("seed", 0) or 0) * 1000 + rank


__all__ = [
    "TASK_FS", "TASK_ICA", "FRAMEWORK_DEFAULTS", "TASK_DEFAULTS", "REFERENCE_INPUT_KEYS",
    "REFERENCE_TASK_ARG_KEYS", "EXTRA_INPUT_KEYS", "build_config",
    "load_inputspec", "load_compspec", "compspec_defaults", "unwrap_values", "validate",
    "generate_compspec", "write_compspec", "site_seed",
]
