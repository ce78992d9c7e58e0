"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 path: sharding of
utterances and the packet gather that bench.py runs over RCCL on GPUs."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from janus_amd.dist import shard


def test_shard_covers_everything():
    for total in (0, 1, 7, 64, 513):
        for world in (1, 2, 3, 8):
            spans = [shard(r, world, total) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from janus_amd.dist import gather_packets
    from oracle import packet as opk
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard(rank, world, 5)
    pk = [opk.serialize(f"utt {i}", 0, {"energy": "Normal", "pitch": "High"}, "auto", float(i))
          if i != 3 else None for i in range(b, e)]
    got = gather_packets(pk, torch.device("cpu"))
    from janus_amd.dist import gather_results
    st = torch.tensor([[0.1 * i, 100.0 + i, float(i % 3)] for i in range(b, e)], dtype=torch.float32)
    pk2, st_all = gather_results(pk, st, torch.device("cpu"))
    assert pk2 == got
    q.put((rank, (got, st_all.tolist())))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_packets_two_ranks():
    from oracle import packet as opk
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [opk.serialize(f"utt {i}", 0, {"energy": "Normal", "pitch": "High"}, "auto", float(i))
            if i != 3 else None for i in range(5)]
    want_st = torch.tensor([[0.1 * i, 100.0 + i, float(i % 3)] for i in range(5)], dtype=torch.float32).tolist()
    for r in (0, 1):
        assert res[r][0] == want and res[r][1] == want_st
