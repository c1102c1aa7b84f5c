"""End-to-end ViT-L/32 cSGHMC steps (bench.e2e_steps: fwd + bwd + fused
update, loss.item() per step) in four modes — eager, eager with the update
overlapped per bucket, HIP graph, HIP graph with the bucket updates captured —
and the graph-overlap mode at several bucket sizes (BDL_OVERLAP_BUCKET_MB).
One JSON line per run.  Each configuration runs in a fresh child process (the
bucket size is read at import).

  python tools/overlap_e2e.py [STEPS]        (default 20; MBS="64,256,1024")
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    import bench
    steps, graph, overlap = int(sys.argv[2]), sys.argv[3] == "1", sys.argv[4] == "1"
    r = bench.e2e_steps(steps, 3, 0, 42, graph=graph, overlap=overlap)
    r.update(graph=graph, overlap=overlap, bucket_mb=os.environ.get("BDL_OVERLAP_BUCKET_MB", "64"))
    r.pop("what", None)
    print(json.dumps(r), flush=True)
    sys.exit(0)

steps = sys.argv[1] if len(sys.argv) > 1 else "20"
runs = [("0", "0", "64"), ("0", "1", "64"), ("1", "0", "64")]
runs += [("1", "1", mb) for mb in os.environ.get("MBS", "64,256,1024").split(",")]
for graph, overlap, mb in runs:
    env = dict(os.environ, BDL_OVERLAP_BUCKET_MB=mb)
    p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", steps, graph, overlap],
                       env=env, capture_output=True, text=True, timeout=600)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    print(line[-1] if line else json.dumps({"graph": graph, "overlap": overlap, "bucket_mb": mb,
                                            "rc": p.returncode, "err": p.stderr[-800:]}),
          flush=True)
    if p.returncode != 0:
        sys.exit(p.returncode)
