"""world_size-2 gloo test (CPU) of bench.py's distributed harness: warmup, barrier-bracketed
timed region, and the MAX-over-ranks reduction that the driver's contract requires."""
import os
import socket
import time

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step(r):
        calls.append(r)
        time.sleep(0.05 * (rank + 1))   # rank 1 is the slow one

    dt = bench.timed_region(step, steps=3, warmup=2, sync=lambda: None)
    q.put((rank, dt, calls))
    dist.destroy_process_group()


def test_timed_region_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    dts = [r[1] for r in res]
    # both ranks report the max, which covers the slow rank's 3 timed steps (3 x 0.1 s)
    assert dts[0] == pytest.approx(dts[1])
    assert dts[0] >= 0.3
    for _, _, calls in res:
        assert calls == [0, 1, 2, 3, 4]   # 2 warmup + exactly 3 timed steps


def test_max_over_ranks_single_process():
    import bench
    assert bench.max_over_ranks(1.5) == 1.5
