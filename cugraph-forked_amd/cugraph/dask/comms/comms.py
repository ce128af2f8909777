"""One-process-per-GPU communicator setup for ``cugraph.dask`` (reference
``python/cugraph/cugraph/dask/comms/comms.py:82-260``).

The reference starts a dask-cuda cluster and builds raft/NCCL communicators on
its workers (``initialize``: p2p, ``prows`` x ``pcols`` 2D grid).  Here every GPU is
its own process launched by ``torch.distributed.run``; ``initialize`` builds the
libcugraph_c communicators over the default ``torch.distributed`` group -- RCCL
(the default: world, row and column communicators inside libcugraph_c) or the
torch.distributed callbacks (``backend="torch"``: gloo, several ranks on one GPU,
for tests).  The 2D grid follows the reference: ``prows x pcols`` given, or pcols
= the largest divisor of the world size not above its square root
(``__get_2D_div``, comms.py:40-45), so 8 GPUs make R x C = 4 x 2 (row communicators
of 2).
"""
from __future__ import annotations

import os

_state = {"ctx": None, "handle": None, "R": 1, "C": 1, "backend": None, "own_pg": False}


def _plc():
    import pylibcugraph
    return pylibcugraph


def initialize(comms=None, p2p=False, prows=None, pcols=None, partition_type=1, backend="rccl"):
    """Collective: every rank calls it once.  ``comms`` (a dask client's comms
    object in the reference) is not used; ``p2p`` is implied (RCCL over xGMI)."""
    import torch
    import torch.distributed as dist
    if _state["ctx"] is not None:
        raise RuntimeError("cugraph.dask comms already initialized")
    if partition_type != 1:
        raise ValueError("only the 2D partition (partition_type=1) is supported")
    if not dist.is_initialized():
        # bootstrap + host collectives only; the data path is RCCL inside libcugraph_c
        dist.init_process_group("gloo")
        _state["own_pg"] = True
    world = dist.get_world_size()
    if prows is not None and pcols is not None:
        if prows * pcols != world:
            raise ValueError("prows * pcols must equal the number of GPUs")
        C = pcols
    elif prows is not None:
        if world % prows:
            raise ValueError("prows must divide the number of GPUs")
        C = world // prows
    elif pcols is not None:
        if world % pcols:
            raise ValueError("pcols must divide the number of GPUs")
        C = pcols
    else:
        C = _plc().comms.default_row_comm_size(world)
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    p = _plc()
    ctx = p.comms.init_rccl(C) if backend == "rccl" else p.comms.init_torch(C)
    _state.update(ctx=ctx, handle=p.ResourceHandle(ctx.ptr), R=world // C, C=C, backend=backend)


def collective_device():
    """Device for the small host-side collectives of the Python driver (max id,
    edge counts, start-vertex checks): CPU when the default group runs them on
    gloo ("gloo" or "cpu:gloo,cuda:nccl"), else the GPU (an RCCL-only group
    refuses CPU tensors)."""
    import torch
    import torch.distributed as dist
    b = str(dist.get_backend())
    if b == "gloo" or "cpu:gloo" in b:
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def is_initialized():
    return _state["ctx"] is not None


def get_default_handle():
    if _state["ctx"] is None:
        raise RuntimeError("cugraph.dask.comms.comms.initialize() has not been called")
    return _state["handle"]


def get_2D_partition():
    """(prows, pcols) of the grid (reference get_2D_partition)."""
    return _state["R"], _state["C"]


def get_n_workers(sID=None):
    import torch.distributed as dist
    return dist.get_world_size()


def get_worker_id(sID=None):
    import torch.distributed as dist
    return dist.get_rank()


def destroy():
    """Collective: frees the communicators (and the process group it created)."""
    import torch.distributed as dist
    if _state["ctx"] is None:
        return
    dist.barrier()
    _state["handle"] = None
    _state["ctx"].free()
    _state["ctx"] = None
    if _state["own_pg"]:
        dist.destroy_process_group()
        _state["own_pg"] = False
