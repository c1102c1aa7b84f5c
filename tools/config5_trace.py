"""Which kernel makes config 5's chain 7 differ in the low bits between the
eight-rank ensemble and a lone process (tests/test_gpu_config5.py)?
(tooling, not product)

Runs tests/config5_worker.py twice on the box's GPU, each time with ONE
process under `rocprofv3 --kernel-trace`: the lone chain-7 process, and rank
7 of the eight-process gloo ensemble (ranks 0-6 unprofiled).  Then diffs the
two kernel sequences (names and grid / workgroup sizes) and prints the theta
bit-sums, which tell the two known variants apart.  Output under
gpurun_out/c5/.

    python tools/config5_trace.py            # run both + diff
    python tools/config5_trace.py --diff     # diff existing traces only
"""
import collections
import csv
import glob
import json
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "c5")
WORKER = os.path.join(ROOT, "tests", "config5_worker.py")
PROF = ["rocprofv3", "--kernel-trace", "--output-format", "csv"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run():
    os.makedirs(OUT, exist_ok=True)
    env0 = dict(os.environ, TMPDIR="/tmp")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env0.pop(k, None)
    lone = PROF + ["-d", os.path.join(OUT, "lone"), "-o", "run", "--",
                   sys.executable, WORKER, "--chain", "7", "--out", os.path.join(OUT, "lone.npz")]
    r = subprocess.run(lone, env=env0, timeout=600, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT)
    open(os.path.join(OUT, "lone.log"), "wb").write(r.stdout)
    if r.returncode != 0:
        sys.exit(f"lone run failed rc={r.returncode}")
    port = _port()
    procs = []
    for rank in range(8):
        env = dict(env0, RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE="8",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        cmd = [sys.executable, WORKER, "--out", os.path.join(OUT, f"rank{rank}.npz")]
        if rank == 7:
            cmd = PROF + ["-d", os.path.join(OUT, "rank7"), "-o", "run", "--"] + cmd
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT))
    rcs = []
    for rank, p in enumerate(procs):
        try:
            out = p.communicate(timeout=900)[0]
        finally:
            if p.poll() is None:
                p.kill()
                p.wait()
        open(os.path.join(OUT, f"rank{rank}.log"), "wb").write(out)
        rcs.append(p.returncode)
    if any(rcs):
        sys.exit(f"ensemble failed: {rcs}")


def kernels(tag):
    path = glob.glob(os.path.join(OUT, tag, "**", "*kernel_trace.csv"), recursive=True)
    if not path:
        sys.exit(f"no kernel trace for {tag}")
    rows = list(csv.DictReader(open(path[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size", "")),
             r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))) for r in rows]


def diff():
    a, b = kernels("lone"), kernels("rank7")
    bits = {}
    for tag, f in (("lone", "lone.npz"), ("rank7", "rank7.npz")):
        p = os.path.join(OUT, f)
        if os.path.exists(p):
            bits[tag] = int(np.load(p)["theta_bits"])
    ca = collections.Counter(k[0] for k in a)
    cb = collections.Counter(k[0] for k in b)
    only_a = {k: v for k, v in ca.items() if k not in cb}
    only_b = {k: v for k, v in cb.items() if k not in ca}
    count_diff = {k: (ca[k], cb[k]) for k in set(ca) & set(cb) if ca[k] != cb[k]}
    first = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), None)
    res = {"theta_bits": bits, "launches": [len(a), len(b)],
           "only_lone": only_a, "only_rank7": only_b, "count_differs": count_diff,
           "first_divergence": None if first is None else
           {"index": first, "lone": a[first], "rank7": b[first],
            "context_lone": a[max(0, first - 3):first + 3],
            "context_rank7": b[max(0, first - 3):first + 3]}}
    with open(os.path.join(OUT, "diff.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1)[:6000])


if __name__ == "__main__":
    if "--diff" not in sys.argv:
        run()
    diff()
