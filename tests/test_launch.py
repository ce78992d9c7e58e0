"""bench.py's multi-GPU launch on the CPU (no GPU): ``--gpus N`` without a launcher spawns N
rank processes (gloo here), the ranks see the right RANK / WORLD_SIZE and utterance / channel
shards, a failing rank fails the job, and a mismatched --gpus exits non-zero before any
work; config 5's latency gather over two gloo ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

from janus_amd import launch

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _bench(*argv, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=e,
                          capture_output=True, text=True, timeout=timeout)


def test_check_world():
    assert launch.check_world(1, env={}, visible=1) is None
    assert launch.check_world(8, env={}, visible=8) is None
    assert "only 1 GPU" in launch.check_world(2, env={}, visible=1)
    assert launch.check_world(0, env={}, visible=8) is not None
    # under torch.distributed.run: WORLD_SIZE must equal --gpus, local ranks must fit
    assert launch.check_world(4, env={"WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "4"}, visible=8) is None
    assert "disagree" in launch.check_world(1, env={"WORLD_SIZE": "8"}, visible=8)
    assert "visible" in launch.check_world(8, env={"WORLD_SIZE": "8"}, visible=1)


def test_rank_env():
    e = launch.rank_env(3, 8, 12345, base={"PATH": "/bin"})
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"]) == \
        ("3", "3", "8", "127.0.0.1", "12345")
    assert e["PATH"] == "/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_gpus_2_spawns_two_ranks():
    r = _bench("--gpus", "2", "--launch-check", "--batch", "64", "--streams", "16")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                      # rank 0 alone prints
    got = lines[0]
    assert got["world"] == 2
    assert [x["rank"] for x in got["ranks"]] == [0, 1]
    assert all(x["world"] == 2 for x in got["ranks"])
    # weak scaling: 64 utterances per rank; channel s on rank s mod 2
    assert [x["shard"] for x in got["ranks"]] == [[0, 64], [64, 128]]
    assert [x["channels"] for x in got["ranks"]] == [16, 16]
    assert [x["first_channel"] for x in got["ranks"]] == [0, 1]


def test_bench_gpus_mismatch_fails_loudly():
    # more GPUs than visible (none in this container): non-zero before any work
    r = _bench("--gpus", "2")
    assert r.returncode == 2 and "visible" in r.stderr
    # an external launcher's WORLD_SIZE that disagrees with --gpus
    r = _bench("--gpus", "1", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "disagree" in r.stderr
    # configs 1-3 are single-GPU
    r = _bench("--gpus", "2", "--config", "3")
    assert r.returncode == 2 and "single-GPU" in r.stderr


def test_spawn_propagates_a_failing_rank(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "if r == 1:\n    sys.exit(7)\n"
                      "time.sleep(60)\n")   # rank 0 would wait forever without the stop
    import time
    t0 = time.time()
    assert launch.spawn(2, [str(script)]) == 7
    assert time.time() - t0 < 40
    ok = tmp_path / "ok.py"
    ok.write_text("import os\nassert os.environ['WORLD_SIZE'] == '3'\n")
    assert launch.spawn(3, [str(ok)]) == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lat_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from janus_amd.dist import gather_values
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = [0.001 * (10 * rank + i) for i in range(3 + rank)]   # ranks hold different counts
    q.put((rank, gather_values(mine, torch.device("cpu"))))
    dist.barrier()
    dist.destroy_process_group()


def test_latency_gather_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lat_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [0.001 * i for i in range(3)] + [0.001 * (10 + i) for i in range(4)]
    for r in (0, 1):
        assert res[r] == pytest.approx(want, rel=1e-6)
