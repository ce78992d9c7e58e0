"""One process per GPU for ``bench.py --gpus N``.

The reference processes phrases independently (backend/services/engine.py:499-552), so
N GPUs are N processes, each owning a shard of the utterances (``dist.shard``), joined by
RCCL only for the result gather. Two ways to get there:

* an external launcher (``torch.distributed.run --nproc-per-node N``, as the driver does)
  sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; ``check_world`` then only verifies that
  ``--gpus`` agrees with WORLD_SIZE and that the node shows enough GPUs;
* no launcher (WORLD_SIZE unset) and ``--gpus N > 1``: ``spawn`` starts N fresh child
  processes of the same script with those variables set, BEFORE the parent makes any
  HIP call (counting devices with ``torch.cuda.device_count`` does not initialise the
  runtime), waits for all of them and exits with the first failure's code. A child that
  fails takes the others down (they would otherwise wait in a barrier forever).

Never N = 1 numbers under an N-GPU label: a mismatch exits non-zero before any work.
"""
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus() -> int:
    """GPUs this process may use, without initialising HIP (device_count only reads the
    visible-device list on this image)."""
    import torch
    return int(torch.cuda.device_count())


def check_world(gpus: int, env=None, visible=None):
    """None when ``--gpus`` is consistent with the launch, else an error message.
    env: the process environment (os.environ); visible: GPUs shown to the process (None:
    counted). Under an external launcher WORLD_SIZE must equal --gpus and the local
    ranks must fit the node's GPUs; without one, --gpus N needs N visible GPUs."""
    env = os.environ if env is None else env
    if gpus < 1:
        return f"--gpus {gpus}: need at least one GPU"
    ws = env.get("WORLD_SIZE")
    vis = visible_gpus() if visible is None else visible
    if ws is not None:
        if int(ws) != gpus:
            return f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree"
        local_ws = int(env.get("LOCAL_WORLD_SIZE", ws))
        if local_ws > vis:
            return f"{local_ws} ranks on this node but only {vis} GPU(s) visible"
        return None
    if gpus > vis:
        return f"--gpus {gpus} but only {vis} GPU(s) visible"
    return None


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    """The environment of child ``rank`` (torch.distributed.run's variables)."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn(world: int, argv, python=None, port=None, poll_s: float = 0.2) -> int:
    """Run ``python argv`` as ranks 0 .. world-1 (children, not exec: the parent may not
    replace itself once anything touched the GPU) and wait. Returns 0 when every rank
    exits 0, else the first non-zero exit code (a rank killed by a signal s reports 128 +
    s); the remaining ranks are terminated then, by PID."""
    python = python or sys.executable
    port = port or free_port()
    procs = [subprocess.Popen([python] + list(argv), env=rank_env(r, world, port))
             for r in range(world)]

    def _stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    old = signal.signal(signal.SIGTERM, lambda s, f: (_stop(), sys.exit(128 + s)))
    code = 0
    try:
        live = set(range(world))
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    print(f"[launch] rank {r} exited {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    _stop()
            if live:
                time.sleep(poll_s)
    finally:
        # ranks that outlive a terminate by more than 30 s are killed
        deadline = time.time() + 30
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
        signal.signal(signal.SIGTERM, old)
    return code
