"""Multi-rank column (and row) sharding on CPU (gloo, world_size 2 and 3): each rank
takes its column block (tcsc_amd.shard.column_range), slices W/B exactly as
the GPU ranks do, computes its block with the oracle, and the gathered blocks
must equal the single-process result bit for bit.  No collective is used for
the data itself in the real path; the all_gather here is only the check."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ORACLE_DIR_FOR_WORKERS, PKG_DIR_FOR_WORKERS  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _row_worker(rank, world, port, q):
    """bench.py --scaling strong --shard rows: rank r stages rows
    column_range(M, world, r) of X (the same X everywhere) against the whole W."""
    import sys

    sys.path.insert(0, PKG_DIR_FOR_WORKERS)
    sys.path.insert(0, ORACLE_DIR_FOR_WORKERS)
    import pyoracle
    from tcsc_amd.shard import all_ranges, column_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = pyoracle.load_oracle()
        M, K, N = 23, 300, 64
        X = o.uniform((M, K), 4)
        Wd = o.ternary((K, N), 0.1, 5)
        B = o.uniform((N,), 6)
        W = o.tcsc_from_dense(Wd)
        r0, r1 = column_range(M, world, rank)
        Yb = o.sgemm("prelu_onthego", np.ascontiguousarray(X[r0:r1]), W, B, 0.2)
        hmax = max(b - a for a, b in all_ranges(M, world))
        buf = torch.zeros((hmax, N), dtype=torch.float32)
        buf[: r1 - r0] = torch.from_numpy(Yb)
        outs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf)
        if rank == 0:
            Y = np.concatenate([outs[r][: b - a].numpy() for r, (a, b) in enumerate(all_ranges(M, world))], 0)
            q.put(bool(np.array_equal(Y, o.sgemm("prelu_onthego", X, W, B, 0.2))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_shards_concat_to_full(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_row_worker, args=(world, _free_port(), q), nprocs=world, join=True, start_method="spawn")
    assert q.get(timeout=60)


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, PKG_DIR_FOR_WORKERS)
    sys.path.insert(0, ORACLE_DIR_FOR_WORKERS)
    import pyoracle
    from tcsc_amd.shard import all_ranges, column_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = pyoracle.load_oracle()
        M, K, N = 17, 300, 101
        X = o.uniform((M, K), 1)
        Wd = o.ternary((K, N), 0.1, 2)
        B = o.uniform((N,), 3)
        W = o.tcsc_from_dense(Wd)
        c0, c1 = column_range(N, world, rank)
        Ws = W.column_slice(c0, c1)
        Yb = o.sgemm("prelu_basic", X, Ws, B[c0:c1], 0.2)
        # pad blocks to the same width for all_gather
        wmax = max(b - a for a, b in all_ranges(N, world))
        buf = torch.zeros((M, wmax), dtype=torch.float32)
        buf[:, : c1 - c0] = torch.from_numpy(Yb)
        outs = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(outs, buf)
        # timing protocol of bench.py: max over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            Y = np.concatenate([outs[r][:, : b - a].numpy() for r, (a, b) in enumerate(all_ranges(N, world))], 1)
            full = o.sgemm("prelu_basic", X, W, B, 0.2)
            q.put((bool(np.array_equal(Y, full)), float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_column_shards_concat_to_full(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, q), nprocs=world, join=True, start_method="spawn")
    ok, tmax = q.get(timeout=60)
    assert ok
    assert tmax == float(world)


def test_column_range_partition():
    from tcsc_amd.shard import all_ranges

    for n in (0, 1, 7, 16384, 16385):
        for g in (1, 2, 3, 8):
            r = all_ranges(n, g)
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[i][1] == r[i + 1][0] for i in range(g - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1
