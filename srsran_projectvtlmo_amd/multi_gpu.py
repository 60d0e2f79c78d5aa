"""Multi-GPU partitioning of codeblock batches: independent CB batches are sharded across the GPUs
of one node by batch index, one process per GPU, no data-path collective. torch.distributed (gloo) is used only for
the control plane (barriers, max of the elapsed time)."""
from __future__ import annotations

import os


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(
        os.environ.get("LOCAL_RANK", "0"))


def shard(n: int, rank: int, world: int):
    """Contiguous slice [start, end) of n CBs for `rank` of `world` ([g n / G, (g + 1) n / G))."""
    return (rank * n) // world, ((rank + 1) * n) // world


def cell_to_device(cell_id: int, nof_devices: int) -> int:
    """C5: one cell per GPU (device = cell_id mod G)."""
    return cell_id % nof_devices


def max_over_ranks(values, group=None):
    """Element-wise max of a list of floats over all ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(x) for x in t]


def job_window(start: float, end: float, group=None) -> float:
    """The job's wall time from per-rank timestamps on a common clock (the ranks of one node share CLOCK_REALTIME):
    latest end minus earliest start over all ranks. It counts the skew with which ranks leave the start barrier as job
    time, so it is never below the max over ranks of each rank's own window."""
    neg_start, last_end = max_over_ranks([-start, end], group)
    return last_end + neg_start
