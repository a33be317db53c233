"""CPU: `python bench.py --gpus N` (no WORLD_SIZE) is the 1 -> N scaling
launcher: the parent never initialises a GPU, starts one
fresh process per rank for 1, 2, 4, ... N ranks, each its own rendezvous,
and prints ONE line carrying the N-rank figures and the whole curve."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT", "O3DX_BENCH_SHARED_GPU"):
        env.pop(k, None)
    return env


def test_rank_counts_and_argv():
    sys.path.insert(0, ROOT)
    import bench

    assert bench._rank_counts(1) == [1]
    assert bench._rank_counts(2) == [1, 2]
    assert bench._rank_counts(8) == [1, 2, 4, 8]
    assert bench._rank_counts(6) == [1, 2, 4, 6]
    assert bench._strip_gpus(["--gpus", "8", "--steps", "3", "--gpus=4", "--warmup", "1"]) == \
        ["--steps", "3", "--warmup", "1"]


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_flag_reaches_the_launcher(n):
    """--gpus N spawns real child processes (gloo rendezvous, --dry-run: no
    GPU work) for every rank count and reports each count's world size."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "3", "--warmup", "1", "--no-cpu",
                        "--dry-run", "--child-timeout", "120"], env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 3 and d["warmup"] == 1
    assert d["extra"]["world_size_observed"] == n
    assert d["extra"]["scaling_child"] is False and d["extra"]["no_cpu"] is True
    counts = [str(c) for c in ([1, 2] if n == 2 else [1, 2, 4])]
    assert list(d["scaling_curve"]["weak_c2_per_gpu"]) == counts
    for c in counts:
        pt = d["scaling_curve"]["weak_c2_per_gpu"][c]
        assert pt["value"] == float(c) and pt["efficiency"] == 1.0
        assert d["scaling_curve"]["strong_c4_50M"][c]["efficiency"] == 1.0
    assert d["launcher"]["rank_counts"] == [int(c) for c in counts] and not d["launcher"]["errors"]


def test_launcher_reports_a_failed_rank_count():
    """A rank count whose processes fail ends the sweep: one line, the error
    named, exit status 1 (here: no GPU for the real step)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu",
                        "--child-timeout", "120"], env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 1
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] is None
    assert d["launcher"]["errors"] and "1 ranks" in d["launcher"]["errors"][0]
