"""Multi-GPU path of bench.py rehearsed on CPU with gloo, world_size 2:
weak-scaling shards (no data-path collective), barrier, max-over-ranks time,
and that the shards of one global counter-based stream tile it exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    import bench
    import oracle as O
    d = bench.Dist(world, "gloo", None)      # bench.py's process group (--dist-backend gloo)
    per = 3
    first, count = bench.shard(per, rank)
    x = O.fill_uniform(count, "p-I", 0x5EED0002, first)       # this rank's shard
    X = O.poly_ntt(x, "p-I")                                    # independent work, no exchange
    d.barrier()
    t = d.max(0.5 + rank)
    out[rank] = (first, count, t, X.tobytes())
    d.close()


def test_gloo_world2_sharding():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle as O
    assert [out[r][0] for r in range(world)] == [0, 3]
    assert all(out[r][2] == 1.5 for r in range(world))            # max over ranks
    whole = O.poly_ntt(O.fill_uniform(6, "p-I", 0x5EED0002, 0), "p-I")
    got = np.concatenate([np.frombuffer(out[r][3], np.uint32).reshape(-1, 1024) for r in range(world)])
    assert np.array_equal(got, whole)


def test_bench_launcher_free_ranks_fail_loudly_without_devices():
    """bench.py --gpus 2 with no launcher starts its own two ranks; with fewer
    visible devices than ranks (none here) every rank exits non-zero and so
    does the parent -- it never falls back to measuring fewer GPUs."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    # no device visible to the children, whatever the machine has (on an
    # 8-GPU box this CPU test must not start a real 2-rank bench)
    env.update(HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--batch", "64",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode != 0
    assert "error:" in r.stderr, r.stderr       # the failing rank says why (the others are stopped)
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_rejects_launcher_world_mismatch():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {**os.environ, "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--batch", "64",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
