"""Multi-GPU host logic on CPU (gloo, world sizes 2 and 4): the 2D grid helpers and
the torch.distributed communicator adapter that libcugraph_c's MG path calls
(pylibcugraph/comms.py, include/cugraph_amd/comm.h).  Buffers are host memory here
(memory="host"); on the GPU the same adapter moves device buffers
(tests/test_gpu_mg.py)."""
import os
import socket

import numpy as np
import pytest

from conftest import PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_grid_helpers():
    import sys
    sys.path.insert(0, PKG)
    pytest.importorskip("torch")
    from pylibcugraph.comms import default_row_comm_size, grid_groups
    # the reference's rule, mg_utilities.cpp:60-63: largest divisor <= sqrt(P)
    assert [default_row_comm_size(p) for p in (1, 2, 4, 8, 6, 16, 32)] == [1, 1, 2, 2, 2, 4, 4]
    rows, cols = grid_groups(8, 4)
    assert rows == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert cols == [[0, 4], [1, 5], [2, 6], [3, 7]]


def _worker(rank, world, port, C):
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pylibcugraph import comms as cm
    Cc, w, row, col = cm.torch_comms(C, memory="host")
    R = world // C
    r, c = rank // C, rank % C
    assert (row.rank, row.size, col.rank, col.size) == (c, C, r, R)

    def ptr(a):
        return a.ctypes.data

    # world allreduce (sum / max)
    send = np.array([rank + 1.0, -rank], dtype=np.float64)
    recv = np.zeros(2)
    assert w.allreduce(None, ptr(send), ptr(recv), 2, cm.CGX_COMM_F64, cm.CGX_COMM_SUM, None) == 0
    assert recv.tolist() == [world * (world + 1) / 2, -sum(range(world))]
    mx = np.array([rank], dtype=np.int64)
    out = np.zeros(1, dtype=np.int64)
    assert w.allreduce(None, ptr(mx), ptr(out), 1, cm.CGX_COMM_I64, cm.CGX_COMM_MAX, None) == 0
    assert out[0] == world - 1
    # row allgather: the C ranks of my row, in column order
    g_send = np.array([rank, rank], dtype=np.int32)
    g_recv = np.zeros(2 * C, dtype=np.int32)
    assert row.allgather(None, ptr(g_send), ptr(g_recv), 2, cm.CGX_COMM_I32, None) == 0
    assert g_recv.tolist() == [x for q in range(C) for x in (r * C + q, r * C + q)]
    # column reduce-scatter of u64 fixed-point sums (wraps like the GPU integers)
    k = 3
    rs_send = np.array([(rank * 100 + i) for i in range(R * k)], dtype=np.uint64)
    rs_recv = np.zeros(k, dtype=np.uint64)
    assert col.reduce_scatter(None, ptr(rs_send), ptr(rs_recv), k, cm.CGX_COMM_U64, cm.CGX_COMM_SUM, None) == 0
    members = [q * C + c for q in range(R)]
    assert rs_recv.tolist() == [sum(m * 100 + r * k + i for m in members) for i in range(k)]
    # world alltoallv with ragged counts
    scnt = [rank + q + 1 for q in range(world)]
    a_send = np.concatenate([np.full(n, rank * 1000 + q, dtype=np.int64) for q, n in enumerate(scnt)])
    rcnt = [q + rank + 1 for q in range(world)]
    a_recv = np.zeros(sum(rcnt), dtype=np.int64)
    arr = (lambda v: (np.ctypeslib.as_ctypes(np.asarray(v, dtype=np.uint64))))
    sc, sd = arr(scnt), arr(np.cumsum([0] + scnt[:-1]))
    rc, rd = arr(rcnt), arr(np.cumsum([0] + rcnt[:-1]))
    assert w.alltoallv(None, ptr(a_send), sc, sd, ptr(a_recv), rc, rd, cm.CGX_COMM_I64, None) == 0
    exp = np.concatenate([np.full(n, q * 1000 + rank, dtype=np.int64) for q, n in enumerate(rcnt)])
    assert np.array_equal(a_recv, exp)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C", [(2, 2), (2, 1), (4, 2)])
def test_torch_comm_adapter_gloo(world, C):
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as tmp
    lib = os.path.join(PKG, "lib", "libcugraph_c.so")
    if not os.path.exists(lib):
        pytest.skip("libcugraph_c.so not built")
    tmp.spawn(_worker, args=(world, _free_port(), C), nprocs=world, join=True)
    del torch


def _mismatch_worker(rank, world, port):
    """Rank 0 calls an allreduce where rank 1 calls an allgather (the same call number):
    both must fail with CollectiveMismatch naming the two calls, not hang or mix data."""
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pylibcugraph import comms as cm
    _, w, _, _ = cm.torch_comms(world, memory="host")
    send = np.ones(4, dtype=np.float64)
    recv = np.zeros(4 * world, dtype=np.float64)
    p = lambda a: a.ctypes.data  # noqa: E731
    # a matching call first: call numbers agree
    assert w.allreduce(None, p(send), p(recv), 4, cm.CGX_COMM_F64, cm.CGX_COMM_SUM, None) == 0
    try:
        if rank == 0:
            w._check("allreduce", 4, cm.CGX_COMM_F64, cm.CGX_COMM_SUM)
        else:
            w._check("allgather", 4, cm.CGX_COMM_F64)
        raise AssertionError("mismatch not detected")
    except cm.CollectiveMismatch as e:
        msg = str(e)
        assert "rank 0: call 2 allreduce" in msg and "rank 1: call 2 allgather" in msg, msg
    # the C-facing entry point reports the failure as a nonzero return
    if rank == 0:
        rc = w.allreduce(None, p(send), p(recv), 4, cm.CGX_COMM_F64, cm.CGX_COMM_SUM, None)
    else:
        rc = w.allgather(None, p(send), p(recv), 4, cm.CGX_COMM_F64, None)
    assert rc == 1
    dist.barrier()
    dist.destroy_process_group()


def test_torch_comm_detects_mismatched_collectives():
    pytest.importorskip("torch")
    import torch.multiprocessing as tmp
    tmp.spawn(_mismatch_worker, args=(2, _free_port()), nprocs=2, join=True)
