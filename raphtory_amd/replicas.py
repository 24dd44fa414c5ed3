"""Replica mode for N GPUs of one node: every rank holds the whole packed graph
and answers its own share of a Range query's hop grid; no data-path collective.

weak scaling: rank r of N runs the base grid offset by r*jump/N (the union is the same Range
job at jump/N granularity, so per-GPU work is constant as N grows).
"""
from __future__ import annotations

import numpy as np


def replica_hops(base: np.ndarray, jump: int, rank: int, world: int) -> np.ndarray:
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return np.asarray(base, np.int64) + (rank * int(jump)) // world


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a per-rank float over the process group (the timing rule of bench.py)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
