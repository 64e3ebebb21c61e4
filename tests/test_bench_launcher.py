"""bench.py honours --gpus N (the driver's contract): run directly with N > 1 it starts
N ranks under torch.distributed.run itself, under torchrun it insists WORLD_SIZE == N,
and it refuses N larger than the visible device count. The CPU rehearsal (--dry-run)
runs the real launcher and rendezvous (gloo) and reports n_gpus from the collective."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", **kw)
    return env


def test_launcher_spawns_n_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one line
    out = lines[0]
    assert out["n_gpus"] == 3 and out["ranks_seen"] == 3 and out["rank_sum"] == 0 + 1 + 2


def test_eight_rank_rehearsal():
    """The N=8 shape the driver runs on an 8-GPU node, rehearsed on the CPU over gloo: eight ranks
    rendezvous, time a region between barriers, and rank 0 alone reports the whole-job value
    from the summed solutions and the slowest rank's time."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=480)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = lines[0]
    assert out["n_gpus"] == 8 and out["ranks_seen"] == 8 and out["rank_sum"] == sum(range(8))
    assert out["total_solutions"] == sum(100 + r for r in range(8))
    assert out["max_rank_seconds"] >= 0.08 > out["rank0_seconds"]  # the slowest rank (7) sets the time
    assert abs(out["value"] - out["total_solutions"] / out["max_rank_seconds"]) < 1e-6


def test_refuses_more_gpus_than_visible():
    # this container has no GPU: asking for 2 real ranks must fail before anything starts
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], capture_output=True, text=True,
                       env=_env(), timeout=240)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr


def test_world_size_must_match():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), timeout=240)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr


def test_launch_command_shape():
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    def fake(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 7
    rc = bench.launch_ranks(["--gpus", "8", "--steps", "5"], 8, launcher=fake)
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
