"""Task plugins and registries (reference ``comps/__init__.py:7-16``)."""
from enum import Enum

from .fs import FreeSurferDataset, FreeSurferTrainer, FSVDataHandle, read_stats_file
from .ica import ICADataHandle, ICADataset, ICATrainer, load_array, read_lines


class NNComputation(str, Enum):
    """Available tasks."""
    TASK_FREE_SURFER = "FS-Classification"
    TASK_ICA = "ICA-Classification"


class AggEngine(str, Enum):
    DECENTRALIZED_SGD = "dSGD"
    RANK_DAD = "rankDAD"
    POWER_SGD = "powerSGD"


TASKS = {
    NNComputation.TASK_FREE_SURFER.value: (FreeSurferTrainer, FreeSurferDataset, FSVDataHandle),
    NNComputation.TASK_ICA.value: (ICATrainer, ICADataset, ICADataHandle),
}


def register_task(task_id: str, trainer, dataset, datahandle):
    """Add a new computation (the reference's "Add new NN computation Here", local.py:39)."""
    TASKS[str(task_id)] = (trainer, dataset, datahandle)


def get_task(task_id: str):
    key = task_id.value if isinstance(task_id, Enum) else str(task_id)
    if key not in TASKS:
        raise ValueError(f"Invalid task: {task_id!r}; known: {sorted(TASKS)}")
    return TASKS[key]


__all__ = ["NNComputation", "AggEngine", "TASKS", "register_task", "get_task",
           "FreeSurferDataset", "FreeSurferTrainer", "FSVDataHandle", "ICADataset", "ICATrainer",
           "ICADataHandle", "read_stats_file", "load_array", "read_lines"]
