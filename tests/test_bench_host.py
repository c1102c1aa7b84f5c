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


RANK_SCRIPT = r"""
import json, os, signal, sys, time
out = sys.argv[1]
r = int(os.environ["RANK"])
with open(os.path.join(out, f"rank{r}.json"), "w") as f:
    json.dump({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                          "MASTER_PORT")}, f)
if r == int(os.environ["FAIL_RANK"]):
    time.sleep(0.5)
    sys.exit(7)
if os.environ.get("IGNORE_TERM"):
    signal.signal(signal.SIGTERM, signal.SIG_IGN)
time.sleep(120)  # stands for a barrier the failed rank never reaches
"""


def _launch(tmp_path, world, fail_rank, ignore_term=False, kill_after=20.0):
    import importlib.util
    import time
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    os.environ["FAIL_RANK"] = str(fail_rank)
    if ignore_term:
        os.environ["IGNORE_TERM"] = "1"
    try:
        t0 = time.monotonic()
        rc = bench.launch_ranks(world, cmd=[sys.executable, str(script), str(tmp_path)],
                                kill_after=kill_after)
        return rc, time.monotonic() - t0
    finally:
        os.environ.pop("FAIL_RANK", None)
        os.environ.pop("IGNORE_TERM", None)


def test_launch_ranks_stops_the_others_and_returns_the_failing_code(tmp_path):
    """bench.launch_ranks at world 4: every rank gets its RANK / LOCAL_RANK, the
    same WORLD_SIZE and rendezvous; rank 2 exits 7 while the others wait at a
    'barrier'; they are stopped and the parent returns 7, not a hang."""
    import json
    rc, dt = _launch(tmp_path, 4, fail_rank=2)
    assert rc == 7 and dt < 30
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_launch_ranks_kills_ranks_that_ignore_sigterm(tmp_path):
    rc, dt = _launch(tmp_path, 3, fail_rank=0, ignore_term=True, kill_after=1.0)
    assert rc == 7 and dt < 30


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod_ids", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_distinct_device_check_refuses_shared_or_missing_gpus():
    """bench.check_distinct_devices: under RCCL every rank must report its own
    GPU (PCI address + UUID) and the node must show at least N devices; the
    gloo rehearsal shares one device on purpose."""
    b = _bench_module()
    ids = [{"pci": f"0000:{0x10 + r:02x}:00", "uuid": f"GPU-{r}"} for r in range(8)]
    assert b.check_distinct_devices(ids, "nccl", 8, 8) is None
    assert "only 4 visible" in b.check_distinct_devices(ids[:8], "nccl", 4, 8)
    shared = ids[:7] + [dict(ids[3])]
    assert "same GPU" in b.check_distinct_devices(shared, "nccl", 8, 8)
    assert b.check_distinct_devices([ids[0]] * 8, "gloo", 1, 8) is None


def test_rank_devices_exits_3_when_ranks_share_a_gpu(monkeypatch):
    """bench.rank_devices under RCCL: ranks that report one GPU, or a node
    that shows fewer GPUs than ranks, end the run with exit status 3 (after
    tearing the process group down) before anything is timed."""
    import pytest
    import torch
    b = _bench_module()

    class FakeDist:
        destroyed = 0

        def all_gather_object(self, out, obj):
            for i in range(len(out)):
                out[i] = dict(obj)  # every rank reports the same device

        def get_backend(self):
            return "nccl"

        def destroy_process_group(self):
            FakeDist.destroyed += 1

    monkeypatch.setattr(b, "device_identity",
                        lambda local: {"index": local, "pci": "0000:05:00.0", "uuid": "GPU-0"})
    for ndev in (8, 1):  # shared device; fewer devices than ranks
        monkeypatch.setattr(torch.cuda, "device_count", lambda: ndev)
        with pytest.raises(SystemExit) as e:
            b.rank_devices(FakeDist(), 0, 2)
        assert e.value.code == 3
    assert FakeDist.destroyed == 2
