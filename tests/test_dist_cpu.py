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


def test_world_nccl_branch_passes_device_tensors(monkeypatch):
    """Under backend "nccl" (RCCL on the GPU box) World hands the tensor itself to the collective: no host staging,
    the all-reduce in place on the caller's buffer, the gather's parts allocated like the source.  The
    collectives are stubbed (no process group on the CPU); the gloo branch is covered by the tests above."""
    from toued.dist import World
    calls = []

    def fake_all_reduce(t, op=None):
        calls.append(("all_reduce", t))
        t.mul_(2)

    def fake_all_gather(parts, src):
        calls.append(("all_gather", src))
        for i, p in enumerate(parts):
            p.copy_(src + i)

    monkeypatch.setattr(dist, "is_initialized", lambda: True)
    monkeypatch.setattr(dist, "all_reduce", fake_all_reduce)
    monkeypatch.setattr(dist, "all_gather", fake_all_gather)
    w = World(rank=1, size=2, local_rank=1, backend="nccl")
    assert w.active and not w._staged(torch.zeros(1))
    g = torch.arange(3, dtype=torch.float32)
    out = w.all_reduce_sum(g)
    assert out is g and calls[-1][1] is g and g.tolist() == [0.0, 2.0, 4.0]
    src = torch.arange(2, dtype=torch.int32)
    cat = w.all_gather_cat(src)
    assert calls[-1][1] is src and cat.tolist() == [0, 1, 1, 2]


@pytest.mark.parametrize("size", [8])
def test_world_gloo_eight_ranks_c5_slices(size):
    """C5's layout on eight gloo ranks: 4096 agents in contiguous slices of 512, gathered back in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker8, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(size))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, (lo, hi, n), ok, s in res:
        assert (lo, hi, n) == (512 * r, 512 * (r + 1), 4096) and ok
        assert s == float(sum(range(size)))


def _worker8(rank, size, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from toued.dist import init_from_env
    w = init_from_env("gloo")
    lo, hi, n = w.agent_slice(4096)
    full = w.all_gather_cat(torch.arange(lo, hi, dtype=torch.int32))
    s = w.all_reduce_sum(torch.tensor([float(rank)]))
    q.put((rank, (lo, hi, n), bool(torch.equal(full, torch.arange(n, dtype=torch.int32))), float(s[0])))
    dist.barrier()
    dist.destroy_process_group()


def test_nccl_rank_without_a_gpu_fails_clearly(monkeypatch):
    """More nccl (RCCL) ranks on a node than GPUs: init_from_env refuses before RCCL's communicator init, naming the
    cause (here: local rank 1 on a one-GPU node)."""
    from toued import dist as tdist
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(tdist.dist, "init_process_group", lambda **kw: pytest.fail("reached init_process_group"))
    with pytest.raises(RuntimeError, match="no GPU of its own"):
        tdist.init_from_env("nccl")
