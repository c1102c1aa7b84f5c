"""Where a kernel's register spills sit: in its sweep loops or outside them.

    hipcc ... --cuda-device-only -S -o X.s X.hip
    python tools/hot_loop_spills.py X.s [kernel-name-filter]

tools/resource_usage.py counts a kernel's SGPR / VGPR spills; this tool says
where the spill code is.  It splits each kernel's assembly into basic blocks,
finds the natural loops (back edges of the control-flow graph) and, for every
loop that issues 16-B vector loads (a sweep loop), prints its size and the
spill traffic inside it: v_writelane / v_readlane (SGPRs spilled into VGPR
lanes) and scratch accesses (VGPRs spilled to memory).  A kernel whose spill
code lies outside every sweep loop pays for it once per launch, not per
element.  One line per kernel: the largest sweep loop (the fast path's) and
the sum over all sweep loops."""
from __future__ import annotations

import re
import subprocess
import sys

LABEL = re.compile(r"^(\.LBB\d+_\d+):")
FALL = re.compile(r"^; %bb\.(\d+):")
BR = re.compile(r"^\s+s_branch\s+(\.LBB\d+_\d+)")
CBR = re.compile(r"^\s+s_cbranch_\w+\s+(\.LBB\d+_\d+)")
LOAD16 = re.compile(r"^\s+(global|flat|buffer)_load_dwordx4")
RL = re.compile(r"^\s+v_readlane_b32")
WL = re.compile(r"^\s+v_writelane_b32")
SCR = re.compile(r"^\s+(scratch_|buffer_(load|store)_dword\w*.*s\[0:3\])")


def kernels(text):
    """(mangled name, body lines) per kernel of an amdgcn .s file."""
    out, name, body = [], None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s", line + " ")
        if m and not line.startswith("\t"):
            name, body = m.group(1), []
            continue
        if name is not None:
            if line.startswith(".Lfunc_end"):
                out.append((name, body))
                name = None
            else:
                body.append(line)
    return out


def blocks(body):
    """Basic blocks: list of dicts {name, lines, succ}."""
    bl, cur = [], {"name": "entry", "lines": []}
    for line in body:
        m = LABEL.match(line) or FALL.match(line)
        if m:
            bl.append(cur)
            cur = {"name": m.group(1) if LABEL.match(line) else f"bb{m.group(1)}", "lines": []}
            continue
        cur["lines"].append(line)
    bl.append(cur)
    idx = {b["name"]: i for i, b in enumerate(bl)}
    for i, b in enumerate(bl):
        succ, term = [], False
        for line in b["lines"]:
            m = BR.match(line)
            if m:
                succ.append(idx[m.group(1)])
                term = True
            m = CBR.match(line)
            if m:
                succ.append(idx[m.group(1)])
            if re.match(r"^\s+s_endpgm", line):
                term = True
        if not term and i + 1 < len(bl):
            succ.append(i + 1)
        b["succ"] = succ
    return bl


def loops(bl):
    """Natural loops {header: set(blocks)} from the DFS back edges."""
    n = len(bl)
    pred = [[] for _ in range(n)]
    for i, b in enumerate(bl):
        for s in b["succ"]:
            pred[s].append(i)
    state, back = [0] * n, []
    stack = [(0, iter(bl[0]["succ"]))]
    state[0] = 1
    while stack:
        v, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            state[v] = 2
            stack.pop()
            continue
        if state[nxt] == 1:
            back.append((v, nxt))
        elif state[nxt] == 0:
            state[nxt] = 1
            stack.append((nxt, iter(bl[nxt]["succ"])))
    out = {}
    for t, h in back:
        body, work = {h, t}, [t]
        while work:
            v = work.pop()
            for p in pred[v]:
                if p not in body:
                    body.add(p)
                    work.append(p)
        out.setdefault(h, set()).update(body)
    return out


def count(bl, members, rx):
    return sum(1 for i in members for line in bl[i]["lines"] if rx.match(line))


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True, check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def analyse(text, filt=""):
    rows = []
    ks = kernels(text)
    for (name, body), dn in zip(ks, demangle([k[0] for k in ks])):
        if filt and filt not in dn and filt not in name:
            continue
        bl = blocks(body)
        allm = set(range(len(bl)))
        sweeps = []
        for h, mem in loops(bl).items():
            ld = count(bl, mem, LOAD16)
            if ld:
                sweeps.append({"blocks": len(mem), "load16": ld, "readlane": count(bl, mem, RL),
                               "writelane": count(bl, mem, WL), "scratch": count(bl, mem, SCR),
                               "lines": sum(len(bl[i]["lines"]) for i in mem)})
        main = max(sweeps, key=lambda s: s["load16"], default=None)
        inloops = set().union(*[m for h, m in loops(bl).items()
                                if count(bl, m, LOAD16)]) if sweeps else set()
        rows.append({"kernel": dn, "readlane": count(bl, allm, RL),
                     "writelane": count(bl, allm, WL), "scratch": count(bl, allm, SCR),
                     "main": main,
                     "in_sweeps": {"readlane": count(bl, inloops, RL),
                                   "writelane": count(bl, inloops, WL),
                                   "scratch": count(bl, inloops, SCR)}})
    return rows


def main(argv):
    rows = analyse(open(argv[1]).read(), argv[2] if len(argv) > 2 else "")
    for r in rows:
        m = r["main"] or {}
        s = r["in_sweeps"]
        print(f"{r['kernel'][:60]:60s} kernel rl {r['readlane']:>3} wl {r['writelane']:>3} "
              f"scr {r['scratch']:>3} | sweep loops rl {s['readlane']:>3} wl {s['writelane']:>3} "
              f"scr {s['scratch']:>3} | main loop {m.get('lines', 0):>5} lines "
              f"{m.get('load16', 0):>3} x16B-loads rl {m.get('readlane', 0):>3} "
              f"wl {m.get('writelane', 0):>3}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
