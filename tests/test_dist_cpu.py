"""World (toued/dist.py) collectives and agent slicing on CPU with gloo, world size 2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size),
                      LOCAL_RANK=str(rank))
    from toued.dist import init_from_env
    from toued.train import reduce_metrics
    w = init_from_env("gloo")
    lo, hi, n = w.agent_slice(8)
    g = torch.arange(lo, hi, dtype=torch.float32)
    full = w.all_gather_cat(g)
    s = w.all_reduce_sum(g.clone())
    m = reduce_metrics({"x": g * 2, "nested": {"y": torch.ones(hi - lo) * rank}}, w)
    q.put((rank, (lo, hi, n), full.tolist(), s.tolist(), m))
    dist.barrier()
    dist.destroy_process_group()


def test_world_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, sl0, full0, s0, m0), (r1, sl1, full1, s1, m1) = res
    assert sl0 == (0, 4, 8) and sl1 == (4, 8, 8)
    assert full0 == full1 == [float(i) for i in range(8)]
    assert s0 == s1 == [4.0, 6.0, 8.0, 10.0]
    assert m0 == m1 == {"x": 7.0, "nested": {"y": 0.5}}


def test_agent_slice_rejects_uneven():
    from toued.dist import World
    with pytest.raises(ValueError):
        World(0, 3).agent_slice(8)
