"""Vertex partition function, verbatim from S/core/utils/Utils.scala:32-35.

getPartition(id, managerCount) = (|id| mod 10*managerCount) div 10   (Partition Manager / GPU)
getWorker(id, managerCount)    = (|id| mod 10*managerCount) mod 10   (storage shard in a PM)
"""
from __future__ import annotations

import numpy as np


def get_partition(ids, manager_count: int):
    a = np.abs(np.asarray(ids, dtype=np.int64))
    return (a % (manager_count * 10)) // 10


def get_worker(ids, manager_count: int):
    a = np.abs(np.asarray(ids, dtype=np.int64))
    return (a % (manager_count * 10)) % 10
