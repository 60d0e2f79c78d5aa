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


def device_identity(device_index: int) -> dict:
    """Which physical GPU this rank drives: its HIP device index plus the PCI location and UUID the runtime reports
    (the fields a shared GPU would repeat across ranks). Host name too, so ranks of different nodes never collide."""
    import socket

    import torch
    p = torch.cuda.get_device_properties(device_index)
    pci = None
    if getattr(p, "pci_bus_id", None) is not None:
        pci = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0) or 0, p.pci_bus_id, getattr(p, "pci_device_id", 0) or 0)
    uuid = getattr(p, "uuid", None)
    return {"host": socket.gethostname(), "device": int(device_index), "pci": pci,
            "uuid": str(uuid) if uuid is not None else None, "name": p.name}


def gather_objects(obj, group=None) -> list:
    """Every rank's `obj`, in rank order (just [obj] when not distributed). Control plane only (gloo)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def check_distinct_devices(idents, allow_shared: bool = False) -> bool:
    """Fail loudly when two ranks drive the same GPU (same host and same PCI location / UUID / device index): a
    multi-GPU line whose ranks share a device would overstate the GPU count. With allow_shared (a rehearsal of N ranks
    on fewer GPUs) the duplicate is tolerated and reported: returns whether every rank has its own GPU."""
    seen = {}
    for r, d in enumerate(idents):
        key = (d.get("host"), d.get("pci") or d.get("uuid") or d.get("device"))
        if key in seen:
            if not allow_shared:
                raise RuntimeError(f"ranks {seen[key]} and {r} share one GPU ({key[0]} {key[1]}): one process per GPU "
                                   f"is required for an N-GPU measurement")
            return False
        seen[key] = r
    return True


def job_window(start: float, end: float, group=None) -> float:
    """The job's wall time from per-rank timestamps on a common clock (the ranks of one node share CLOCK_REALTIME):
    latest end minus earliest start over all ranks. It counts the skew with which ranks leave the start barrier as job
    time, so it is never below the max over ranks of each rank's own window."""
    neg_start, last_end = max_over_ranks([-start, end], group)
    return last_end + neg_start
