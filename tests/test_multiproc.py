"""N>1 orchestration of bench.py on the CPU (gloo, world size 2): the
barrier-bracketed timing takes the MAX over ranks, and every rank gets its
own stream (weak scaling, no shared state, no data-path collective)."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step():
        time.sleep(0.02 * (rank + 1))    # rank 1 is the slow one
        calls.append(1)
        return rank

    dt, res = bench.timed_steps(step, steps=3, warmup=2, world=world)
    q.put((rank, dt, len(calls), res, bench.rank_ssrc(rank)))
    dist.destroy_process_group()


def test_timed_steps_world2_takes_max_over_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, dt0, n0, res0, s0), (r1, dt1, n1, res1, s1) = out
    assert n0 == n1 == 5                  # warmup 2 + timed 3 on each rank
    assert res0 == [0] * 3 and res1 == [1] * 3
    assert dt0 == pytest.approx(dt1)      # both report the max ...
    assert dt1 >= 3 * 0.04                # ... which is the slow rank's time
    assert s0 != s1                       # one stream per rank


def _key_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # every rank starts from different key material; rank 0's must win
    mine = bench.stream_keys(3, seed=100 + rank)
    got = bench.distribute_keys(mine, world, "cpu")
    q.put((rank, got))
    dist.destroy_process_group()


def test_key_broadcast_world2():
    """the session (re)key step: rank 0's master keys reach every rank in
    one broadcast (RCCL in bench.py on GPUs, gloo here)"""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_key_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = bench.stream_keys(3, seed=100)
    assert out[0] == out[1] == want
    assert all(len(bytes.fromhex(k)) == 46 for k in want)


def _bench(args, env=None):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] +
                          args, capture_output=True, text=True, env=e,
                          timeout=180)


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` (the driver's N>1 form, here without a launcher)
    starts two ranks itself; rank 0 prints the one JSON line, whose time is
    the slower rank's (the stub step takes (rank + 1) ms)"""
    import json
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "5", "--warmup", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    assert rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["packets_total"] == 2 * rec["config"]["packets_per_gpu"]
    assert rec["ms_per_step"] >= 2.0            # max over ranks: rank 1's 2 ms
    assert rec["value"] == pytest.approx(
        2 * rec["config"]["packets_per_gpu"] * 5 / (rec["ms_per_step"] * 5e-3))


def test_bench_gpus1_and_world_mismatch():
    import json
    r = _bench(["--dry-run", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["parallelism"] == "dp1"
    assert rec["config"]["baseline_config"] == 1
    # under a launcher, --gpus must equal WORLD_SIZE
    r = _bench(["--dry-run", "--gpus", "2"], env={"WORLD_SIZE": "1"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
