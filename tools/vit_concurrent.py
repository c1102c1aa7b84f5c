"""Do concurrent processes sharing one GPU sample the same ViT-L/32 chain
bit for bit (tooling)?  Starts K processes that each run the config-5
worker's chain 7 (no torch.distributed) at the same time and prints their
theta bit-sums; NOCUDNN=1 routes the patch convolution around MIOpen.

  python tools/vit_concurrent.py [K]
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    if os.environ.get("NOCUDNN") == "1":
        torch.backends.cudnn.enabled = False
    from config5_worker import run_chain
    r = run_chain(chain=7)
    print(json.dumps({"bits": int(r["theta_bits"]), "sum": float(r["theta_sum"])}), flush=True)
    sys.exit(0)

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
env = dict(os.environ)
procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for _ in range(k)]
bits = []
for p in procs:
    out = p.communicate(timeout=600)[0].decode(errors="replace")
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    bits.append(json.loads(line[-1])["bits"] if line else out[-500:])
print(json.dumps({"concurrent": k, "nocudnn": os.environ.get("NOCUDNN") == "1", "bits": bits,
                  "all_equal": len(set(map(str, bits))) == 1}), flush=True)
