"""World-size-2 gloo run of bench.py's multi-rank plumbing on CPU.

bench.py --gpus N runs one process per GPU, each classifying its own
independent fragment set: the only cross-rank traffic is
the barrier around the timed region and the reductions of fragment counts
(sum) and times (max).  This covers that path without a GPU.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    import repkiller_amd as rk
    r, w, local = bench.dist_setup()
    assert (r, w, local) == (rank, world, rank)
    f = rk.synth(1000, 100_000, seed=bench.rank_seed(r))
    bench.barrier(w)
    total, dt = bench.aggregate(w, f.n + r, 0.5 + r)  # ranks differ in size and time
    q.put((r, total, dt, int(f.x_start[:16].sum())))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    # every rank sees the whole-job count (1000 + 1001) and the slowest time
    assert [r[1] for r in res] == [2001.0, 2001.0]
    assert [r[2] for r in res] == [1.5, 1.5]
    # independent fragment sets per rank
    assert res[0][3] != res[1][3]


def test_single_rank_is_local():
    import bench
    assert bench.aggregate(1, 7, 0.25) == (7.0, 0.25)
    assert bench.rank_seed(0) != bench.rank_seed(1)


def _gather_worker(rank, world, port, q):
    """bench.gather_result: rank r holds output rows [off_r, off_r + k_r) of one
    whole result (ragged shares, one empty), rank 0 reassembles it."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    bench.dist_setup()
    n = 1000
    rng = np.random.default_rng(7)
    order = rng.permutation(n).astype(np.uint32)
    gid = np.sort(rng.integers(0, 300, n)).astype(np.uint32)
    rep = rng.integers(0, 3, n).astype(np.uint8)
    # ragged shares; at world 3 rank 0's share is empty
    cuts = {2: [0, 517, n], 3: [0, 0, 613, n]}[world]
    a, b = cuts[rank], cuts[rank + 1]
    whole = bench.gather_result(world, rank, a, order[a:b], gid[a:b], rep[a:b], n)
    if rank == 0:
        same = all(np.array_equal(u, v) for u, v in zip(whole, (order, gid, rep)))
        q.put((rank, same, bench.arrays_sha256(*whole) == bench.arrays_sha256(order, gid, rep)))
    else:
        q.put((rank, whole is None, True))
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_result_reassembles_shares(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(r[1] and r[2] for r in res), res


def test_strong_scaling_blocks_tile_the_set():
    import bench
    n = 50_000_000
    for world in (1, 2, 3, 4, 8):
        blocks = [bench.row_block(n, r, world) for r in range(world)]
        assert blocks[0][0] == 0 and blocks[-1][1] == n
        assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    assert bench.config_seed("cfg3") == 3 and bench.config_seed("cfg4") == 4


def _comm_worker(rank, world, port, q):
    """The gloo host-callback collectives behind rk.Comm.torch_host (the comm the
    multi-rank GPU tests run rk_classify_sharded on), called as the C side does."""
    import ctypes
    import torch.distributed as dist
    import repkiller_amd as rk
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = rk.Comm.torch_host(rank, world)
    allgather, alltoallv = comm._keep[0], comm._keep[1]
    mine = (ctypes.c_uint8 * 3)(*[10 * rank + i for i in range(3)])
    allg = (ctypes.c_uint8 * (3 * world))()
    assert allgather(None, ctypes.addressof(mine), ctypes.addressof(allg), 3) == 0
    # rank r sends r+1+q bytes of value 16*r+q to rank q
    sb = (ctypes.c_uint64 * world)(*[rank + 1 + q for q in range(world)])
    rb = (ctypes.c_uint64 * world)(*[q + 1 + rank for q in range(world)])
    send = bytes(b for q in range(world) for b in [16 * rank + q] * (rank + 1 + q))
    sbuf = (ctypes.c_uint8 * len(send)).from_buffer_copy(send)
    rbuf = (ctypes.c_uint8 * sum(rb))()
    assert alltoallv(None, ctypes.addressof(sbuf), sb, ctypes.addressof(rbuf), rb) == 0
    q.put((rank, list(allg), list(rbuf)))
    comm.close()
    dist.destroy_process_group()


def test_host_comm_callbacks_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    for rank, allg, recv in res:
        assert allg == [0, 1, 2, 10, 11, 12]
        want = [16 * src + rank for src in range(2) for _ in range(src + 1 + rank)]
        assert recv == want
