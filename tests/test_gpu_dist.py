"""World-size-2 rehearsal of the multi-GPU path THROUGH the HIP library:
two ranks (torch.distributed.run or bench.py's own launcher, gloo), each
running ntt_amd on its shard of the batch -- on two GPUs when present, else
both on the one device (--allow-shared-devices).  The 8-GPU scaling run
itself is the driver's (one rank per GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}"] + args
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def test_shards_concatenate_to_single_process_result(ntt, tmp_path):
    out = tmp_path / "dist.json"
    r = _torchrun([os.path.join(ROOT, "tests", "dist_worker.py"), str(out)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads(out.read_text())
    assert set(res) == {"p-III", "p-I"}
    for ps, v in res.items():
        assert v["world"] == 2 and v["ntt"] and v["mul"], (ps, v)


def test_bench_two_ranks_counts_both(ntt):
    batch, steps = 8192, 3
    r = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", str(batch), "--steps", str(steps),
                   "--warmup", "1", "--dist-backend", "gloo", "--no-cpu-baseline",
                   "--allow-shared-devices"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout        # rank 0 prints one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * batch
    assert d["config"]["dist_backend"] == "gloo"
    assert d["check"]["all_ranks_ok"] is True
    # value = polys of BOTH ranks / the max-over-ranks wall time
    assert abs(d["value"] - 2 * batch * steps / (d["ms_per_step"] * steps * 1e-3)) <= 1e-6 * d["value"]


def test_bench_default_backend_is_gloo(ntt):
    """The bench's only collectives are a barrier and a scalar max/min on
    CPU tensors (north_star: no data-path collective), so the default
    process group is gloo; the line names it and the per-rank spread."""
    r = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "4096", "--steps", "2",
                   "--warmup", "1", "--no-cpu-baseline", "--allow-shared-devices"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["dist_backend"] == "gloo"
    spread = d["rank_ms_per_step"]
    assert 0 < spread["min"] <= spread["max"] == pytest.approx(d["ms_per_step"])


def test_bench_two_ranks_rccl(ntt):
    """The RCCL (nccl) process group, kept as an option: exercised only where
    two devices exist (RCCL refuses two ranks on one device)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one device per rank; this box has one GPU")
    r = _torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "4096", "--steps", "2",
                   "--warmup", "1", "--dist-backend", "nccl", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["dist_backend"] == "nccl" and d["check"]["all_ranks_ok"] is True


def _bench(args, timeout=240):
    env = {**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


def test_bench_spawns_ranks_without_launcher(ntt):
    """python3 bench.py --gpus 2 (no torchrun): the script starts both ranks
    itself and the line counts both ranks' polynomials."""
    batch, steps = 4096, 3
    r = _bench(["--gpus", "2", "--allow-shared-devices", "--batch", str(batch), "--steps", str(steps),
                "--warmup", "1", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * batch
    assert d["check"]["all_ranks_ok"] is True
    assert abs(d["value"] - 2 * batch * steps / (d["ms_per_step"] * steps * 1e-3)) <= 1e-6 * d["value"]


def test_bench_refuses_more_ranks_than_devices(ntt):
    """--gpus N with fewer than N visible devices and no --allow-shared-devices
    exits non-zero instead of measuring fewer GPUs."""
    import torch
    n = torch.cuda.device_count() + 1
    r = _bench(["--gpus", str(n), "--batch", "64", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert "visible device" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("config", [4, 5])
def test_bench_two_ranks_product_configs(ntt, config):
    """BASELINE's multi-GPU config is the poly-mul (config 4, 2^23 sharded
    over 8 GPUs); config 5 (Nussbaumer) shards the same way.  Rehearsed here
    through bench.py's own launcher-free spawn, its checker legs and its
    global_batch accounting, with the VALU roofline block of a product line."""
    batch, steps = 4096, 2
    r = _bench(["--config", str(config), "--gpus", "2", "--allow-shared-devices", "--batch", str(batch),
                "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * batch
    assert d["check"]["all_ranks_ok"] is True
    assert d["check"]["sampled_vs_oracle"]["ok"] is True
    assert d["unit"] == "products/s"
    roof = d["roofline"]
    assert roof["bound"] == "valu" and roof["unit"] == "G SIMD-cycles/s" and roof["hbm"]["bound"] == "hbm"
    assert roof["kernel"] == ("mul" if config == 4 else "nus")
    assert abs(d["value"] - 2 * batch * steps / (d["ms_per_step"] * steps * 1e-3)) <= 1e-6 * d["value"]
