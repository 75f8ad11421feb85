"""Communicator layer: reference tests/test_mpi.py::test_reduce_sum at several world
sizes, plus the previously untested split/scatter/object paths."""
import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.parallel import comm as C
from multigrad_amd.parallel.subcomm import (distribute_data, reduce_sum, scatter_nd,
                                            split_subcomms)

from distributed import run_distributed


def _reduce_sum_body(rank, size):
    comm = mg.get_world_comm()
    assert comm.size == size and comm.rank == rank
    # reference test: value = rank, total = size(size-1)/2 on every rank
    res_tensor = mg.reduce_sum(torch.tensor(rank))
    res_scalar = mg.reduce_sum(rank)
    res_float = mg.reduce_sum(float(rank) + 0.5)
    res_np = mg.reduce_sum(np.arange(3) + rank)
    gathered = comm.allgather(int(res_tensor))
    expect = size * (size - 1) // 2
    assert all(x == expect for x in gathered)
    assert isinstance(res_scalar, int) and res_scalar == expect
    assert isinstance(res_float, float) and res_float == pytest.approx(expect + 0.5 * size)
    assert isinstance(res_np, np.ndarray)
    np.testing.assert_array_equal(res_np, np.arange(3) * size + expect)
    # reduce to root
    r = reduce_sum(torch.ones(4) * (rank + 1), root=0)
    if rank == 0:
        assert torch.allclose(r, torch.full((4,), float(size * (size + 1) // 2)))
    # mpi4py-style buffer API
    buf = np.zeros(5)
    comm.Allreduce(np.full(5, rank, dtype=np.float64), buf)
    np.testing.assert_allclose(buf, expect)
    return int(res_tensor)


@pytest.mark.parametrize("size", [1, 2, 3, 4])
def test_reduce_sum(size):
    if size == 1:
        C.set_world_comm(None)
        assert _reduce_sum_body(0, 1) == 0
        return
    res = run_distributed(_reduce_sum_body, size)
    assert res == [size * (size - 1) // 2] * size


def test_reduce_sum_comm_none():
    assert reduce_sum(3.0, comm=None) == 3.0


def _split_body(rank, size, num_groups, rpg):
    sub, ng, g = split_subcomms(num_groups=num_groups, ranks_per_group=rpg)
    total = reduce_sum(1, comm=sub)
    members = sub.allgather(rank)
    # nested split of the sub-communicator by parity of the sub-rank
    subsub = sub.split(color=sub.rank % 2)
    nested = reduce_sum(torch.tensor([float(rank)]), comm=subsub)
    return (g, ng, sub.name, sub.rank, sub.size, total, members, subsub.name, float(nested[0]))


def test_split_subcomms_num_groups_size5():
    res = run_distributed(_split_body, 5, 2, None)
    groups = [r[0] for r in res]
    # reference assignment (multigrad/multigrad.py:115-128): {0,1}->0, {2,3,4}->1
    assert groups == [0, 0, 1, 1, 1]
    assert [r[2] for r in res] == ["0", "0", "1", "1", "1"]
    assert [r[4] for r in res] == [2, 2, 3, 3, 3]
    assert [r[5] for r in res] == [2, 2, 3, 3, 3]
    assert res[2][6] == [2, 3, 4]
    # nested names "<group>.<color>" and sums over the nested groups
    assert res[2][7] == "1.0" and res[3][7] == "1.1"
    assert res[2][8] == 2.0 + 4.0 and res[3][8] == 3.0


def test_split_subcomms_ranks_per_group():
    res = run_distributed(_split_body, 4, None, [1, 3])
    assert [r[0] for r in res] == [0, 1, 1, 1]
    assert [r[4] for r in res] == [1, 3, 3, 3]


def test_split_assignment_matches_reference_formula():
    import math

    def ref(size, ng):
        sub = (np.ones(math.ceil(size / ng))[None, :] * np.arange(ng)[:, None])[:size]
        sub = sub.ravel().astype(int)
        return [int(np.array_split(sub, size)[r][0]) for r in range(size)]

    class Fake(C.SerialComm):
        pass

    for size in range(1, 12):
        for ng in range(1, size + 1):
            per = math.ceil(size / ng)
            labels = np.repeat(np.arange(ng), per)
            mine = [int(np.array_split(labels, size)[r][0]) for r in range(size)]
            assert mine == ref(size, ng), (size, ng)


def _by_node_body(rank, size):
    sub, nn, node = mg.split_subcomms_by_node()
    return nn, node, sub.size, sub.name


def test_split_by_node_single_host():
    res = run_distributed(_by_node_body, 3)
    assert all(r == (1, 0, 3, "0") for r in res)


def _objects_body(rank, size):
    comm = mg.get_world_comm()
    obj = comm.bcast({"a": [1, 2, 3], "r": rank}, root=1)
    assert obj == {"a": [1, 2, 3], "r": 1}
    if rank == 0:
        comm.send(np.arange(5), dest=size - 1, tag=3)
    if rank == size - 1:
        got = comm.recv(source=0, tag=3)
        np.testing.assert_array_equal(got, np.arange(5))
    arr = np.arange(20).reshape(10, 2) if rank == 0 else None
    piece = scatter_nd(arr, axis=0)
    expect = np.array_split(np.arange(20).reshape(10, 2), size, axis=0)[rank]
    np.testing.assert_array_equal(piece, expect)
    t = torch.arange(7.0) if rank == 0 else None
    tp = scatter_nd(t)
    assert torch.equal(tp, torch.tensor_split(torch.arange(7.0), size)[rank])
    chunk = distribute_data(list(range(10)))
    comm.barrier()
    # tensor collectives on CPU
    x = torch.arange(4.0) + rank
    out = torch.empty(4 * size)
    comm.all_gather_into_tensor(out, x)
    assert torch.equal(out, torch.cat([torch.arange(4.0) + r for r in range(size)]))
    rs = torch.empty(2)
    comm.reduce_scatter_tensor(rs, torch.arange(2.0 * size))
    assert torch.equal(rs, (torch.arange(2.0 * size) * size)[2 * rank:2 * rank + 2])
    b = torch.full((3,), float(rank))
    comm.broadcast(b, root=size - 1)
    assert torch.equal(b, torch.full((3,), float(size - 1)))
    mx = torch.tensor([float(rank)])
    comm.all_reduce(mx, op="max")
    assert mx.item() == size - 1
    return chunk


def test_object_and_tensor_collectives():
    res = run_distributed(_objects_body, 3)
    assert res == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]


def test_serial_comm_semantics():
    c = C.SerialComm()
    assert c.rank == 0 and c.size == 1 and c.Get_size() == 1
    assert c.bcast(5) == 5 and c.allgather(1) == [1]
    c.send("x", dest=0, tag=2)
    assert c.recv(source=0, tag=2) == "x"
    s = c.split(3)
    assert s.name == "3" and s.size == 1
    buf = np.zeros(2)
    c.Allreduce(np.ones(2), buf)
    np.testing.assert_array_equal(buf, 1)
    assert split_subcomms(num_groups=1, comm=c)[0].name == "0"


def test_launcher_env_fallbacks(monkeypatch):
    for k in ["RANK", "WORLD_SIZE", "LOCAL_RANK"]:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "3")
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "8")
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "3")
    env = C.launcher_env()
    assert env["rank"] == 3 and env["size"] == 8 and env["local_rank"] == 3


def _host_count_body(rank, size):
    import multigrad_amd as mg
    from multigrad_amd.optim._reduce import DeviceReducer
    comm = mg.get_world_comm()
    n0 = comm.host_collectives
    t = torch.ones(3)
    comm.all_reduce(t)
    comm.barrier()
    n1 = comm.host_collectives
    # the optimizers' reducer on CPU tensors: the host path, one sum and one max all-reduce
    red = DeviceReducer(comm, sharded=True, device="cpu")
    out = red.reduce(sums=[torch.tensor([rank + 1.0, 2.0])], maxes=[torch.tensor([float(rank)])],
                     local=[torch.tensor([7.0])])
    return n1 - n0, comm.host_collectives - n1, red.describe(), out.tolist(), t.tolist()


def test_host_collectives_are_counted_and_reducer_layout():
    """TorchComm counts its host (gloo) collectives -- the device optimizers report the
    count per run (0 on GPUs with peer memory or RCCL) -- and DeviceReducer returns
    [sums, maxes, local] in one vector on every path."""
    res = run_distributed(_host_count_body, 2)
    for rank, (d_direct, d_red, path, out, t) in enumerate(res):
        assert d_direct == 2 and d_red == 2 and path == "host"
        assert out == [3.0, 4.0, 1.0, 7.0]
        assert t == [2.0, 2.0, 2.0]
