"""COINSTAC site callback (reference ``local.py``): code defaults as in ``local.py:31-37``;
the COINSTAC input overrides them.  State persists across iterations in module globals (one
node per ``clientId``, so several sites can also be simulated in one process)."""
import time

from dinunet_implementations_amd.compat.nodes import LocalNode
from dinunet_implementations_amd.utils.logs import duration

CACHE = {}
NODES = {}


def run(data):
    _start = time.time()
    start_time = CACHE.setdefault("start_time", _start)
    cid = (data.get("state") or {}).get("clientId", "local0")
    node = NODES.get(cid)
    if node is None:
        node = NODES[cid] = LocalNode(batch_size=16, epochs=21, patience=31,
                                      split_ratio=[0.7, 0.15, 0.15], pretrain_args=None,
                                      dataloader_args={"train": {"drop_last": True}}, num_class=2,
                                      monitor_metric="auc", log_header="loss|auc")
    out = node(data)
    duration(CACHE, _start, key="time_spent_on_computation")
    duration(CACHE, start_time, key="cumulative_total_duration")
    return out
