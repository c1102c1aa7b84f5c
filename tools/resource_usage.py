"""Per-kernel register / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.

    hipcc ... --cuda-device-only -c -o /dev/null X.hip \
        -Rpass-analysis=kernel-resource-usage 2> remarks.txt
    python tools/resource_usage.py remarks.txt [name-filter]

One line per kernel: demangled template arguments, SGPRs, VGPRs, SGPR / VGPR
spills, scratch bytes per lane, occupancy (waves per SIMD).  Exit status 1
when any kernel matching the filter spills (used to check a build)."""
from __future__ import annotations

import re
import subprocess
import sys


def parse(text):
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def main(argv):
    text = open(argv[1]).read()
    filt = argv[2] if len(argv) > 2 else ""
    rows = parse(text)
    names = demangle([r["name"] for r in rows])
    spills = 0
    for r, nm in zip(rows, names):
        if filt and filt not in nm and filt not in r["name"]:
            continue
        s, v = int(r.get("SGPRs Spill", 0)), int(r.get("VGPRs Spill", 0))
        spills += s + v
        print(f"{nm[:70]:70s} sgpr {r.get('TotalSGPRs', '?'):>3} vgpr {r.get('VGPRs', '?'):>3} "
              f"spill s{s:>3} v{v:>3} scratch {r.get('ScratchSize [bytes/lane]', '?'):>3} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}")
    return 1 if spills else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
