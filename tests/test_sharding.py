"""Multi-GPU path on CPU: image sharding and the final byte-string gather,
run as world_size 2 over gloo (the same code runs over RCCL in bench.py)."""
import os
import socket

import pytest

from guetzli_amd import sharding


def test_shard_partition():
    for world in (1, 2, 3, 8):
        got = sorted(i for r in range(world) for i in sharding.shard(64, world, r))
        assert got == list(range(64))
        assert all(len(sharding.shard(64, world, r)) in (64 // world, 64 // world + 1)
                   for r in range(world))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import guetzli_amd as gz
        # each rank "encodes" its shard: synthetic frames -> bytes (host-only
        # stand-in payloads of different lengths, incl. an empty one)
        mine = sharding.shard(5, world, rank)
        blobs = [gz.synthetic_frame(i, 9 + i, 7).tobytes()[: 50 * i] for i in mine]
        got = sharding.gather_bytes(blobs, dist, "cpu")
        q.put((rank, [[len(b) for b in r] for r in got], got[rank] == blobs,
               [b[:16] for r in got for b in r]))
    finally:
        dist.destroy_process_group()


def test_gather_bytes_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # rank 0 encoded frames 0, 2, 4 and rank 1 frames 1, 3 -> lengths 50*i
    expect = [[0, 100, 200], [50, 150]]
    for rank, lens, own_ok, heads in res:
        assert lens == expect
        assert own_ok
    assert res[0][3] == res[1][3]


def test_bench_launches_ranks_itself_world2():
    """`bench.py --gpus 2` outside torch.distributed.run starts the two ranks
    itself (torch.distributed.run on 127.0.0.1, one process per GPU); the CPU
    self-test mode runs the same launcher, process group, byte gather and
    max-over-ranks timing over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    res = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                          "--frames-per-step", "3", "--dist-selftest"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stderr[-2000:]
    line = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, res.stdout
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["gather_ok"] and out["frames"] == 6
