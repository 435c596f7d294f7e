"""COINSTAC aggregator callback (reference ``remote.py``): learns the task from site messages."""
import time

from dinunet_implementations_amd.compat.nodes import RemoteNode
from dinunet_implementations_amd.utils.logs import duration

CACHE = {}
NODE = None


def run(data):
    global NODE
    _start = time.time()
    start_time = CACHE.setdefault("start_time", _start)
    if NODE is None:
        NODE = RemoteNode()
    out = NODE(data)
    duration(CACHE, _start, key="time_spent_on_computation")
    duration(CACHE, start_time, key="cumulative_total_duration")
    return out
