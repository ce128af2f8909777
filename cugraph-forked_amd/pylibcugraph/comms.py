"""Multi-GPU communicator contexts for the MG entry points (include/cugraph_amd/comm.h).

Role of the reference's ``cugraph.dask.comms.comms`` + raft's NCCL bootstrap
(``python/cugraph/cugraph/dask/comms/comms.py``; 2D sub-communicators as
``cpp/tests/utilities/mg_utilities.cpp:52-68``): one process per GPU, launched by
``torch.distributed.run``; the returned context pointer goes into
``ResourceHandle(ctx.ptr)``.

* ``init_rccl()``: production path.  Rank 0 makes an RCCL unique id, it is
  broadcast over the default torch.distributed group, and every rank builds the
  world / row / column RCCL communicators inside libcugraph_c (xGMI).
* ``init_torch()``: the collectives are callbacks into torch.distributed on the
  current process groups (gloo stages device buffers through host memory).  RCCL
  refuses two ranks on one GPU, so this is how the MG path is tested on a single
  MI355X; it also runs with ``memory="host"`` on a CPU-only machine, where the
  "device" pointers are host pointers (tests of the adapter itself).

Grid: P = R x C ranks, rank = r * C + c, row communicator = the C ranks of row r,
column communicator = the R ranks of column c (``default_row_comm_size``).
"""
from __future__ import annotations

import ctypes
import math
import traceback

from . import _lib

CGX_COMM_U8, CGX_COMM_I32, CGX_COMM_I64, CGX_COMM_U64, CGX_COMM_F32, CGX_COMM_F64 = range(6)
CGX_COMM_SUM, CGX_COMM_MIN, CGX_COMM_MAX = range(3)

_ELEM = {CGX_COMM_U8: 1, CGX_COMM_I32: 4, CGX_COMM_I64: 8, CGX_COMM_U64: 8, CGX_COMM_F32: 4, CGX_COMM_F64: 8}
_TYPESTR = {CGX_COMM_U8: "|u1", CGX_COMM_I32: "<i4", CGX_COMM_I64: "<i8", CGX_COMM_U64: "<i8",
            CGX_COMM_F32: "<f4", CGX_COMM_F64: "<f8"}


class CommOps(ctypes.Structure):
    _fields_ = [
        ("ctx", ctypes.c_void_p),
        ("rank", ctypes.c_int),
        ("size", ctypes.c_int),
        ("allreduce", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)),
        ("allgather", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p)),
        ("reduce_scatter", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)),
        ("alltoallv", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_void_p)),
    ]


def default_row_comm_size(world_size: int) -> int:
    """C of the R x C grid: the reference's rule (mg_utilities.cpp:60-63), the largest
    divisor of P that is <= sqrt(P) -- 2 at 8 GPUs (R = 4), 2 at 4, 1 at 2.

    ``row_comm_size=P`` (1 x P) is the alternative for one fully connected node: the
    x~ allgather then runs over all P-1 xGMI links and the column reduce-scatter of
    the fixed-point sums disappears.  bench.py times both grids at
    N > 1 so the choice rests on a measurement of the driver's node."""
    c = max(1, int(math.isqrt(world_size)))
    while world_size % c:
        c -= 1
    return c


def flat_row_comm_size(world_size: int) -> int:
    """1 x P: every rank in one row."""
    return world_size


def grid_groups(world_size: int, row_comm_size: int):
    """(row group rank lists, column group rank lists) of the R x C grid."""
    C = row_comm_size
    R = world_size // C
    rows = [[r * C + c for c in range(C)] for r in range(R)]
    cols = [[r * C + c for r in range(R)] for c in range(C)]
    return rows, cols


class MGContext:
    """Owns a cugraph_amd_mg_context_t (and the callbacks it calls, if any)."""

    def __init__(self, ptr, row_comm_size, keep=None):
        self.ptr = ptr
        self.row_comm_size = row_comm_size
        self._keep = keep

    def free(self):
        if self.ptr:
            _lib.lib.cugraph_amd_mg_context_free(ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self, _sd=_lib.SHUTDOWN):
        if getattr(self, "ptr", None) and not _sd[0]:
            self.free()


def init_rccl(row_comm_size=None):
    """RCCL communicators for the default torch.distributed group (one process per GPU)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    C = row_comm_size or default_row_comm_size(world)
    n = _lib.lib.cugraph_amd_comm_unique_id_size()
    buf = (ctypes.c_char * n)()
    if rank == 0:
        _lib.call("cugraph_amd_comm_get_unique_id", buf)
    obj = [bytes(buf) if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    ctypes.memmove(buf, obj[0], n)
    ctx = ctypes.c_void_p()
    _lib.call("cugraph_amd_mg_context_create_rccl", buf, world, rank, C, ctypes.byref(ctx))
    return MGContext(ctx.value, C)


_OP_TAGS = {"allreduce": 1, "allgather": 2, "reduce_scatter": 3, "alltoallv": 4}


class CollectiveMismatch(RuntimeError):
    """Ranks of one group entered different collectives (or the same one with other
    arguments) at the same call number."""


class _TorchComm:
    """Collectives of one torch.distributed group over buffers handed in by libcugraph_c.

    Every call first checks, on every rank of the group, that all ranks are at the same
    call number of this group and in the same operation with the same element type,
    reduction and (except for alltoallv) element count: one all_gather of 5 int64.  A
    rank that skipped or reordered a collective then fails with CollectiveMismatch
    naming every rank's call, instead of pairing its buffers with another operation's
    (gloo would hang or mix data).  This adapter is the multi-rank rehearsal path; the
    RCCL context does not pay for the check."""

    def __init__(self, group, memory, check=True):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.group = group
        self.memory = memory
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.stage = memory == "host" or dist.get_backend(group) == "gloo"
        self._ops = {CGX_COMM_SUM: dist.ReduceOp.SUM, CGX_COMM_MIN: dist.ReduceOp.MIN,
                     CGX_COMM_MAX: dist.ReduceOp.MAX}
        self._streams = {}
        self.check = check
        self.seq = 0  # calls made on this group

    def _check(self, name, count, dt, op=-1):
        """The per-call agreement check (class doc)."""
        self.seq += 1
        if not self.check or self.size == 1:
            return
        torch = self.torch
        dev = "cpu" if self.stage else "cuda"
        mine = torch.tensor([self.seq, _OP_TAGS[name], int(count), int(dt), int(op)], dtype=torch.int64, device=dev)
        rows = [torch.empty_like(mine) for _ in range(self.size)]
        self.dist.all_gather(rows, mine, group=self.group)
        got = [r.cpu().tolist() for r in rows]
        if any(g != got[0] for g in got):
            names = {v: k for k, v in _OP_TAGS.items()}
            desc = ", ".join(f"rank {q}: call {g[0]} {names.get(g[1], g[1])}(count={g[2]}, dtype={g[3]}, op={g[4]})"
                             for q, g in enumerate(got))
            raise CollectiveMismatch(f"collective mismatch in a group of {self.size}: {desc}")

    # -- buffers
    def _view(self, ptr, count, dt):
        torch = self.torch
        if self.memory == "host":
            if count == 0:
                return torch.empty(0, dtype=_torch_dtype(torch, dt))
            raw = (ctypes.c_char * (count * _ELEM[dt])).from_address(ptr)
            return torch.frombuffer(raw, dtype=_torch_dtype(torch, dt))
        if count == 0:
            return torch.empty(0, dtype=_torch_dtype(torch, dt), device="cuda")
        return torch.as_tensor(_CudaArray(ptr, count, dt), device="cuda")

    # The buffers belong to the library's stream (`stream`, the handle's HIP stream):
    # staging copies run on that stream and only that stream is waited for -- no
    # device-wide synchronize and no legacy-default-stream copies, whose implicit
    # ordering against every other stream of the process is not needed here.  Host
    # staging uses pinned tensors.
    def _stream(self, ptr):
        if self.memory == "host":
            return None
        st = self._streams.get(ptr)
        if st is None:
            st = self._streams[ptr] = self.torch.cuda.ExternalStream(int(ptr or 0))
        return st

    def _sync(self, st):
        if st is not None:
            st.synchronize()

    def _in(self, t, st):
        if not (self.stage and t.device.type != "cpu"):
            if st is None:
                return t.clone()
            with self.torch.cuda.stream(st):
                out = t.clone()
            self._sync(st)
            return out
        h = self.torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        if t.numel():
            with self.torch.cuda.stream(st):
                h.copy_(t, non_blocking=True)
            self._sync(st)
        return h

    def _out(self, dst, t, st):
        if st is None:
            dst.copy_(t)
            return
        if t.device.type == "cpu" and t.numel() and not t.is_pinned():
            t = self.torch.empty(t.shape, dtype=t.dtype, pin_memory=True).copy_(t)
        elif t.device.type != "cpu":  # a device collective's result (nccl): its stream first
            st.wait_stream(self.torch.cuda.current_stream())
        with self.torch.cuda.stream(st):
            dst.copy_(t, non_blocking=True)
        self._sync(st)

    # -- collectives (return 0 on success; exceptions never cross into C).  The library
    # calls them with its stream's work enqueued, so that stream is drained first.
    def allreduce(self, _ctx, send, recv, count, dt, op, stream):
        try:
            self._check("allreduce", count, dt, op)
            st = self._stream(stream)
            self._sync(st)
            t = self._in(self._view(send, count, dt), st)
            if count:
                self.dist.all_reduce(t, op=self._ops[op], group=self.group)
            self._out(self._view(recv, count, dt), t, st)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    def allgather(self, _ctx, send, recv, count, dt, stream):
        try:
            self._check("allgather", count, dt)
            st = self._stream(stream)
            self._sync(st)
            t = self._in(self._view(send, count, dt), st)
            parts = [self.torch.empty_like(t) for _ in range(self.size)]
            self.dist.all_gather(parts, t, group=self.group)
            self._out(self._view(recv, count * self.size, dt), self.torch.cat(parts), st)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    def reduce_scatter(self, _ctx, send, recv, recvcount, dt, op, stream):
        try:
            self._check("reduce_scatter", recvcount, dt, op)
            st = self._stream(stream)
            self._sync(st)
            t = self._in(self._view(send, recvcount * self.size, dt), st)
            out = self.torch.empty(recvcount, dtype=t.dtype, device=t.device)
            if recvcount:
                self.dist.reduce_scatter_tensor(out, t, op=self._ops[op], group=self.group)
            self._out(self._view(recv, recvcount, dt), out, st)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    def alltoallv(self, _ctx, send, sc, sd, recv, rc, rd, dt, stream):
        try:
            self._check("alltoallv", -1, dt)  # (counts differ per rank by design)
            st = self._stream(stream)
            self._sync(st)
            P = self.size
            scnt = [int(sc[q]) for q in range(P)]
            rcnt = [int(rc[q]) for q in range(P)]
            sdis = [int(sd[q]) for q in range(P)]
            rdis = [int(rd[q]) for q in range(P)]
            if sdis != _prefix(scnt) or rdis != _prefix(rcnt):
                raise ValueError("alltoallv: only packed displacements are supported")
            t = self._in(self._view(send, sum(scnt), dt), st)
            out = self.torch.empty(sum(rcnt), dtype=t.dtype, device=t.device)
            self.dist.all_to_all_single(out, t, output_split_sizes=rcnt, input_split_sizes=scnt, group=self.group)
            self._out(self._view(recv, sum(rcnt), dt), out, st)
            return 0
        except Exception:  # noqa: BLE001
            traceback.print_exc()
            return 1

    def ops(self):
        o = CommOps()
        o.ctx = None
        o.rank = self.rank
        o.size = self.size
        f = CommOps._fields_
        o.allreduce = f[3][1](self.allreduce)
        o.allgather = f[4][1](self.allgather)
        o.reduce_scatter = f[5][1](self.reduce_scatter)
        o.alltoallv = f[6][1](self.alltoallv)
        return o


class _CudaArray:
    def __init__(self, ptr, count, dt):
        self.__cuda_array_interface__ = {"shape": (int(count),), "typestr": _TYPESTR[dt], "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def _torch_dtype(torch, dt):
    return {CGX_COMM_U8: torch.uint8, CGX_COMM_I32: torch.int32, CGX_COMM_I64: torch.int64,
            CGX_COMM_U64: torch.int64, CGX_COMM_F32: torch.float32, CGX_COMM_F64: torch.float64}[dt]


def _prefix(c):
    out, acc = [], 0
    for x in c:
        out.append(acc)
        acc += x
    return out


def torch_comms(row_comm_size=None, memory="device"):
    """(world, row, column) _TorchComm adapters over the default process group; every
    rank must call this (torch.distributed.new_group is collective)."""
    import torch.distributed as dist
    world = dist.get_world_size()
    C = row_comm_size or default_row_comm_size(world)
    if world % C:
        raise ValueError("row_comm_size must divide the world size")
    rows, cols = grid_groups(world, C)
    rank = dist.get_rank()
    row_g = col_g = None
    for ranks in rows:
        g = dist.new_group(ranks)
        if rank in ranks:
            row_g = g
    for ranks in cols:
        g = dist.new_group(ranks)
        if rank in ranks:
            col_g = g
    return C, _TorchComm(dist.group.WORLD, memory), _TorchComm(row_g, memory), _TorchComm(col_g, memory)


def init_torch(row_comm_size=None, memory="device"):
    """MG context whose collectives run through torch.distributed (see module doc)."""
    C, w, r, c = torch_comms(row_comm_size, memory)
    ow, orow, ocol = w.ops(), r.ops(), c.ops()
    ctx = ctypes.c_void_p()
    vp = lambda o: ctypes.cast(ctypes.pointer(o), ctypes.c_void_p)  # noqa: E731
    _lib.call("cugraph_amd_mg_context_create_ops", vp(ow), vp(orow), vp(ocol), C, ctypes.byref(ctx))
    return MGContext(ctx.value, C, keep=(w, r, c, ow, orow, ocol))
