"""CPU: bench.py's launcher. `python bench.py --gpus N` with no launcher
around it starts N rank processes itself (torch.distributed.run on
127.0.0.1) before anything touches a GPU, and a launcher whose WORLD_SIZE is
not --gpus is refused (the driver's `bench.py --gpus 8` must
produce 8 ranks, never a line claiming one)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_cmd_shape():
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29999)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29999"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_world_mismatch_is_refused():
    bench.check_world(4, 4)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1)


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=240)


def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--spawn-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    ranks = sorted(json.loads(l)["rank"] for l in r.stdout.splitlines() if l.startswith("{"))
    worlds = {json.loads(l)["world"] for l in r.stdout.splitlines() if l.startswith("{")}
    assert ranks == [0, 1] and worlds == {2}


def test_launcher_with_wrong_world_fails_loudly():
    r = _run(["--gpus", "2", "--spawn-probe"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def _agree_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        oks = [bench.agree_ok(True, torch, dist, world, "cpu"),
               bench.agree_ok(rank != 1, torch, dist, world, "cpu")]

        class Boom:  # the workload build fails on rank 1 only
            def __init__(self, *a):
                if rank == 1:
                    raise MemoryError("synthetic OOM")

        bench.VecWorkload = Boom

        class A:
            records = 0
            config = "c2"
        try:
            bench.run_config("c4", A, torch, dist, world, rank, "cpu", 1, 0, 0, cpu=False)
            raised = None
        except bench.ConfigFailed as e:
            raised = str(e)
        # the ranks are still in step: one more collective completes
        after = bench.agree_ok(True, torch, dist, world, "cpu")
        q.put((rank, oks, raised, after))
    finally:
        dist.destroy_process_group()


def test_config_failure_agreed_across_ranks():
    """a config that fails on one rank must fail on every rank
    before any collective of the config runs (no rank left waiting)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g[1] for g in got] == [[True, False], [True, False]]
    assert "another rank" in got[0][2] and "synthetic OOM" in got[1][2]
    assert all(g[3] for g in got)
