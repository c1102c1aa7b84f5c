"""bench.py's N-rank path end to end on the box's one GPU: two ranks under
torch.distributed.run (two, and eight as the driver's N=8 run), and two or
four ranks started by bench.py itself, with
the gloo backend (BDL_BENCH_BACKEND=gloo, ranks sharing the device; RCCL
needs one GPU per rank).  Checks the contract the
driver relies on at N>1: one JSON line from rank 0, n_gpus = world size,
value = all ranks' steps / max-over-ranks time, the evaluation collective
(chains.average_predictive) timed after the timed region."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


BENCH_ARGS = ["--steps", "20", "--warmup", "5", "--backbone", "resnet101",
              "--no-autotune", "--e2e-steps", "0"]


# ("torchrun", 8): the driver's own N=8 command shape (torch.distributed.run
# --nproc-per-node 8), eight ranks sharing the one GPU
@pytest.mark.parametrize("launcher,world", [("torchrun", 2), ("self", 2), ("self", 4),
                                            ("torchrun", 8)])
def test_bench_ranks_gloo(launcher, world):
    """Under torch.distributed.run, and as `python bench.py --gpus N` with no
    outside launcher (bench.py starts its own ranks): the same one line, with
    every rank's kernel time and the max-over-ranks wall clock."""
    env = dict(os.environ, BDL_BENCH_BACKEND="gloo")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    bench = os.path.join(ROOT, "bench.py")
    args = ["--gpus", str(world)] + BENCH_ARGS
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
               f"--master-port={_free_port()}", bench] + args
    else:
        cmd = [sys.executable, bench] + args
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 20 and d["warmup"] == 5
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["value"] > 0 and \
        abs(d["value"] - world * 20 / (d["ms_per_step"] * 20 / 1e3)) < 0.02 * d["value"]
    assert d["config"]["parallelism"].startswith(f"{world} independent chains")
    ec = d["eval_collective"]
    assert ec["backend"] == "gloo" and ec["finite"] is True
    assert "cpu_baseline" not in d  # rank 0 at N=1 only
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    pr = d["per_rank"]  # every rank's own dominant-kernel time
    assert [r["rank"] for r in pr] == list(range(world))
    assert all(r["kernel"] == d["roofline"]["kernel"] and r["avg_ms"] > 0 and 0 < r["frac"] < 1
               for r in pr)
    # which physical GPU each rank drove (the gloo rehearsal shares the box's one)
    assert all(r["pci"] and r["name"] and "uuid" in r and r["device_count"] >= 1 for r in pr)
    di = d["distributed"]
    assert di["world_size"] == world and di["backend"] == "gloo"
    assert di["device_count"] == torch.cuda.device_count()
    assert di["distinct_devices"] == len({(r["pci"], r["uuid"]) for r in pr}) == 1


def test_rccl_process_group_init_as_bench_does():
    """The RCCL ("nccl") process-group calls bench.py's N-GPU path makes —
    init_process_group with device_id, barrier, all_reduce(MAX) of the timing,
    the chains collectives on device tensors, all_gather_object of the
    per-rank kernel times — in a one-rank group on the box's
    GPU (several ranks need one GPU each)."""
    code = r'''
import os, torch, torch.distributed as dist
from bayesdll_amd import chains
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
dist.barrier()
t = torch.tensor([1.5], dtype=torch.float64, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.MAX)
x = torch.ones(1 << 20, device="cuda")
dist.all_reduce(x)
lp = torch.log_softmax(torch.randn(8, 10, device="cuda"), 1)
assert torch.equal(chains.average_predictive(lp), lp)
got = [None]
dist.all_gather_object(got, {"rank": 0, "avg_ms": 1.0})
assert got == [{"rank": 0, "avg_ms": 1.0}]
torch.cuda.synchronize()
print("RCCL_OK", dist.get_backend(), float(t.item()), float(x[0].item()))
dist.destroy_process_group()
'''
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "RCCL_OK nccl 1.5 1.0" in p.stdout
