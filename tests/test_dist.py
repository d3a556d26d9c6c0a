"""Multi-GPU sharding logic on CPU (gloo, world_size 2).

SURVEY §8e: buffers are independent, so a batch shards over GPUs by a
contiguous byte-balanced split with no collective on the data path.  Here
each rank checksums its shard with the oracle (stand-in for its GPU, no GPU
in this container), results are gathered, and rank 0 checks the gathered
vector equals the unsharded batch -- plus bench.py's MAX-over-ranks timing
reduction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pech_amd.crc32c import shard_ranges


def test_shard_ranges_cover_and_balance():
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 4, 8):
        lens = rng.integers(0, 1 << 22, 1000)
        rs = shard_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        tot = lens.sum()
        biggest = lens.max()
        for lo, hi in rs:
            assert abs(int(lens[lo:hi].sum()) - tot / world) <= biggest
    assert shard_ranges([], 4) == [(0, 0)] * 4
    assert shard_ranges([5], 3)[-1] == (1, 1) or sum(hi - lo for lo, hi in shard_ranges([5], 3)) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, result):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib as O

    rng = np.random.default_rng(123)
    lens = rng.integers(0, 70000, 300)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    lo, hi = shard_ranges(lens, world)[rank]
    mine = O.crcs(data, offs[lo:hi], lens[lo:hi])
    # gather variable-size shards (pad to max)
    n_max = len(lens)
    buf = torch.zeros(n_max, dtype=torch.int64)
    buf[: hi - lo] = torch.from_numpy(mine.astype(np.int64))
    bufs = [torch.zeros(n_max, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(bufs, buf)
    # bench.py timing: MAX over ranks of the elapsed time
    t = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        got = np.concatenate([bufs[r][: b - a].numpy() for r, (a, b) in enumerate(shard_ranges(lens, world))])
        want = O.crcs(data, offs, lens).astype(np.int64)
        result["ok"] = bool(np.array_equal(got, want))
        result["tmax"] = float(t.item())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shard_gather_matches_unsharded():
    world = 2
    with mp.Manager() as m:
        result = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), result), nprocs=world, join=True)
        assert result["ok"]
        assert abs(result["tmax"] - 0.2) < 1e-9
