"""bench.py's multi-rank plumbing on the CPU (no GPU call is reached):
`--gpus N` against the launcher's WORLD_SIZE, and `python bench.py --gpus N`
starting its own N ranks and propagating a failing rank's exit status
instead of hanging at the barrier."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_must_match_the_launchers_world_size():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="1", RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "--gpus 2 but WORLD_SIZE=1" in p.stderr
    assert not p.stdout.strip()


def test_self_launch_starts_n_ranks_and_propagates_failure():
    """Without a launcher, `--gpus 2` starts two rank processes (RANK 0 and 1,
    WORLD_SIZE 2).  On this GPU-less host each rank fails at its device
    selection; the parent returns non-zero and prints no bench line."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"],
                       env=_env(BDL_BENCH_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=600)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "No HIP GPUs" in p.stderr  # a rank started and failed; the others were stopped
