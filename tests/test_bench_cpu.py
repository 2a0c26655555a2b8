"""bench.py's multi-rank launch on the CPU (BASELINE config 1, gloo): ``--gpus 2`` without a
launcher starts torch.distributed.run as a child process, both ranks run the step, and rank 0
prints one JSON line whose world size, backend and per-rank times say two ranks really ran.
The GPU configs use the same launch path (one rank per GPU over RCCL)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    e["OMP_NUM_THREADS"] = "2"
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "baseline_cpu",
                           "--steps", "2", "--warmup", "1", "--image-size", "32"] + extra,
                          capture_output=True, text=True, timeout=timeout, env=e, cwd="/tmp")


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (out.stdout[-2000:], out.stderr[-2000:])
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    out = _run(["--gpus", "2"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_ranks"] == 2 and d["dist"]["world_size"] == 2 and d["dist"]["backend"] == "gloo"
    assert len(d["dist"]["rank_ms_per_step"]) == 2 and all(x > 0 for x in d["dist"]["rank_ms_per_step"])
    assert d["config"]["global_batch"] == 8 and d["config"]["parallelism"].startswith("dp2")
    # value = all ranks' images / the slowest rank's time
    assert abs(d["value"] - 2 * 4 * 2 / (max(d["dist"]["rank_ms_per_step"]) * 2 / 1e3)) < 0.05 * d["value"]


def test_bench_single_rank():
    out = _run(["--gpus", "1"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = _line(out)
    assert d["n_ranks"] == 1 and d["dist"]["world_size"] == 1


def test_bench_rejects_world_size_mismatch():
    """Under a launcher whose world size differs from --gpus the bench refuses to report."""
    out = _run(["--gpus", "2"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0
    assert "launcher started 1 rank" in out.stderr
