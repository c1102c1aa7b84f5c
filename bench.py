"""Benchmark: fused cSGHMC leapfrog update on a ViT-L/32-sized chain (config 4/5).

One step = one cyclical-SGHMC update of a full ViT-L/32 parameter vector
(306,535,400 fp32, 296 tensors, `heads.head` readout), driven exactly like the
reference Runner's batch loop (methods/csghmc.py:265-348): alpha(t) from the
cyclical schedule (M=4 cycles over the run, beta=0.5), noise only on sample
steps, thinning on the batch index, and the per-cycle Welford accumulation of
the posterior moments on thinned sample steps — all in the fused HIP kernel.
Gradients are a synthetic resident buffer (g ~ N(0, 1e-3^2)), re-read every
step; theta ~ N(0, 0.02^2), v = 0 at step 0.

Multi-GPU (`python bench.py --gpus N` starts N rank processes itself;
under `torch.distributed.run --nproc-per-node N` the launcher's ranks are
used, and WORLD_SIZE must equal --gpus): one independent chain per GPU
(seed 42 + rank, Philox chain id = rank); no collective inside the timed
region; value = total chain-steps / max-over-ranks wall time.

Prints one JSON line (rank 0).  Extra fields: hbm_gbs (algorithmic), the
per-kernel-kind table with HIP-event timings, roofline of the dominant
kernel, and the CPU baseline (the oracle's op-for-op torch-CPU restatement of
the reference update, timed on this host on a bounded sample).  After the
timed region (never inside it): every sweep's `mix_ceiling` (the fastest
arithmetic-free form of its own access pattern on its own buffers: bare,
pipelined, paced and, for cSGHMC, the kernel's own loop without its update),
the explore on the Runners' per-tensor gradients, the other configurations'
sweeps (`methods`), and end-to-end ViT-L/32 steps with an interleaved
autograd-only leg (`e2e`, informational).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_ELEM = {"explore": 20, "sample": 20, "collect_init": 28, "collect": 36,
                  # sgld + SGD(momentum): theta rw, g r, theta0 r, buf (w | rw), +m1/m2 rw
                  "sgld_first": 20, "sgld": 24, "sgld_collect": 40,
                  # adam_sghmc + SGD(momentum): theta, v_mom, m, v rw; g, theta0 r; buf (w | rw)
                  "adam_first": 44, "adam": 48, "adam_collect": 64}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--backbone", default="vit_l_32")
    ap.add_argument("--method", default="csghmc", choices=["csghmc", "sgld", "adam_sghmc"])
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--thin", type=int, default=10)
    ap.add_argument("--cycles", type=int, default=4)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--grid-stride", type=int, default=-1)
    ap.add_argument("--no-autotune", action="store_true")
    ap.add_argument("--e2e-steps", type=int, default=10)
    ap.add_argument("--grad-mode", default="flat", choices=["flat", "tensor"],
                    help="gradient source of the timed step: one flat vector, or one tensor "
                         "per parameter read through the per-run base table (the product's "
                         "default with autograd)")
    ap.add_argument("--no-aux", action="store_true",
                    help="skip the posterior-sample / moments sweeps after the timed region")
    ap.add_argument("--prewarm-seconds", type=float, default=0.0,
                    help="untimed back-to-back launches of the method's kernel on scratch "
                         "vectors before the state is built.  The explore sweep runs 1.058 ms "
                         "in the first 0.25 s of sustained load and 1.032-1.035 from ~0.8 s on "
                         "(tools/drift.py, profiles/round5/drift.jsonl), but in the driver's "
                         "command shape (--steps 20 --warmup 5) a 1 s prewarm changed nothing "
                         "(919.5 vs 918.2 steps/s over three fresh processes each, "
                         "profiles/round5/prewarm_ab/): the tuning and warmup already load the "
                         "GPU, and allocation-to-allocation spread is larger; default 0")
    ap.add_argument("--no-methods", action="store_true",
                    help="skip the config-3 SGLD and the Adam-SGHMC lines after the timed region")
    ap.add_argument("--event-stride", type=int, default=0,
                    help="bracket every k-th timed launch (and the first of each kind) with "
                         "HIP events; 1 = all, 0 (default) = max(1, min(5, steps // 10)), i.e. "
                         "2 at the driver's 20 steps, 5 at 200.  Each bracket costs the stream "
                         "~5 us (two event "
                         "packets between kernels): at 1 the line's ms_per_step read 1.0239-1.0248 "
                         "vs 1.0186-1.0191 at 10 on one box, the kernel averages unchanged")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def pool_timing(chains, st, world, dist, out):
    """Informational, after the timed region: chains.pool_moments of one full
    chain vector (1.2 GB for ViT-L/32) over RCCL / xGMI.  Errors are recorded,
    never raised (the bench line must survive)."""
    try:
        chains.pool_moments(st.mom, None, count=1.0)
        torch.cuda.synchronize()
        dist.barrier()
        t2 = time.perf_counter()
        for _ in range(3):
            pooled, _ = chains.pool_moments(st.mom, None, count=1.0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t2) / 3
        nbytes = st.mom.numel() * 4
        out["pool_moments"] = {"bytes": nbytes, "ms": round(dt * 1e3, 3),
                               "algbw_GBs": round(nbytes / dt / 1e9, 1),
                               "busbw_GBs": round(2 * (world - 1) / world * nbytes / dt / 1e9, 1)}
        del pooled
    except Exception as e:  # noqa: BLE001
        out["pool_moments"] = {"error": repr(e)[:200]}


class LaunchTimer:
    """HIP events (torch.cuda.Event, on the stream the kernels run on) around
    every `stride`-th timed launch and around the first launch of each kernel
    kind; per-kind durations in ms."""

    def __init__(self, stride=1):
        self.stride, self.i, self.seen, self.recs = max(1, int(stride)), 0, set(), []

    def begin(self, kind):
        take = self.i % self.stride == 0 or kind not in self.seen
        self.i += 1
        if not take:
            return None
        self.seen.add(kind)
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        self.recs.append((kind, ev))
        return ev

    def durations(self):
        per = {}
        for kind, (e0, e1) in self.recs:
            per.setdefault(kind, []).append(e0.elapsed_time(e1))
        return per


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, cmd=None, kill_after=20.0):
    """`python bench.py --gpus N` without an outside launcher: start N rank
    processes of this same command (`cmd`, default this script with this
    process's arguments; RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on
    127.0.0.1), one per GPU, before this process touches the GPU; wait for all
    of them and return the first non-zero exit status, else 0.  When one rank
    fails the others could never pass their barrier: they get SIGTERM, and
    SIGKILL `kill_after` seconds later if still running.  Rank 0 prints the
    JSON line."""
    import signal
    import subprocess
    if cmd is None:
        cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(cmd, env=env))
    rc, deadline = 0, None
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # one rank failed: the barrier would never complete
                    q.send_signal(signal.SIGTERM)
                deadline = time.monotonic() + kill_after
        if deadline is not None and pending and time.monotonic() > deadline:
            for q in pending:
                q.kill()
            deadline = None
        time.sleep(0.05)
    return rc


def device_identity(local):
    """Which physical GPU this rank drives: index, name, PCI address, UUID."""
    p = torch.cuda.get_device_properties(local)
    ident = {"device": int(local), "name": p.name,
             "pci": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                    f"{getattr(p, 'pci_device_id', 0):02x}"}
    uuid = getattr(p, "uuid", None)
    ident["uuid"] = str(uuid) if uuid is not None else None
    return ident


def check_distinct_devices(idents, backend, device_count, world):
    """Under RCCL every rank must drive its own GPU: refuse a run on fewer
    devices than ranks, or with two ranks on one device (the line's n_gpus
    would be false).  The gloo rehearsal shares devices on purpose.  Returns
    an error message or None."""
    if backend == "gloo":
        return None
    if device_count < world:
        return f"{world} ranks but only {device_count} visible GPUs"
    keys = [(i["pci"], i["uuid"]) for i in idents]
    if len(set(keys)) != len(keys):
        dup = sorted({k for k in keys if keys.count(k) > 1})
        return f"two or more ranks drive the same GPU {dup}"
    return None


def dist_setup(expected):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != expected:
        # a line whose n_gpus differs from --gpus would be mislabelled
        sys.stderr.write(f"bench.py: --gpus {expected} but WORLD_SIZE={world}\n")
        sys.exit(2)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("BDL_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
        ndev = torch.cuda.device_count()
        if backend == "gloo":
            # rehearsal of the N-rank path on fewer GPUs (ranks may share a device)
            local = local % max(1, ndev)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            if local >= ndev:
                sys.stderr.write(f"bench.py: LOCAL_RANK {local} but only {ndev} visible GPUs\n")
                sys.exit(3)
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return dist, rank, world, local
    torch.cuda.set_device(local)
    return None, 0, 1, local


def rank_devices(dist, local, world):
    """Every rank's device identity (all_gather before the timed region); exits
    with status 3 when the ranks do not drive `world` distinct GPUs under RCCL."""
    mine = dict(device_identity(local), device_count=torch.cuda.device_count())
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    err = check_distinct_devices(allr, dist.get_backend(), mine["device_count"], world)
    if err is not None:
        sys.stderr.write(f"bench.py: {err}\n")
        dist.destroy_process_group()
        sys.exit(3)
    return allr


MIX_GEOMS = ((1, 4), (2, 4), (2, 2), (3, 4), (4, 2), (1, 1), (2, 1), (4, 1))


MIX_SCHEDULES = (("bare", 0), ("pipelined", 1), ("paced", 2))  # include/bdl_measure.h


def mix_ceiling(reads, writes, same, kernel_ms, reps=8, step=None):
    """The HBM ceiling of a kernel's exact access pattern on its exact buffers:
    the access mix (bdl_stream_mix_schedule — the same streams read and
    written, no update arithmetic, the step kernels' loop shape) in each issue
    schedule (bare: loads then stores; pipelined: the next iteration's loads
    before this one's stores; paced: a Philox draw per group between loads
    and stores) at every geometry of MIX_GEOMS.  The ceiling is the fastest of
    them (the memory system does not serve every order of the same bytes
    equally fast); `of_ceiling` = ceiling time / kernel time, `same_geometry_ms`
    the bare mix at the kernel's own geometry.  `step` (cSGHMC sweeps): a
    launcher of the kernel's own sweep with its arithmetic removed
    (bdl_sgmcmc_step_bare), timed at every geometry too ("step_shaped": the
    production loop, run table and load / store order).  Destroys the written
    vectors' contents: run last."""
    from bayesdll_amd import kernels as K

    def t(bpc, u, s):
        return float(np.mean(event_times(lambda i: K.stream_mix(reads, writes, bpc, u, s), reps,
                                         warm=2)))
    same_ms = t(*same, 0)
    per = {}
    for name, s in MIX_SCHEDULES:
        per[name] = min((t(b, u, s), (b, u)) for b, u in MIX_GEOMS)
    if step is not None:
        prev = K._ACTIVE[0]
        best = None
        for b, u in MIX_GEOMS:
            K.set_launch_config(b, u, 1)
            ms = float(np.mean(event_times(lambda i: step(), reps, warm=2)))
            best = min(best, (ms, (b, u))) if best else (ms, (b, u))
        K.set_launch_config(*(prev or (0, 0, 0)))
        per["step_shaped"] = best
    bname, (bms, bg) = min(per.items(), key=lambda kv: kv[1][0])
    return {"mix": f"{len(reads)} reads, {len(writes)} writes", "kernel_ms": round(kernel_ms, 4),
            "same_geometry_ms": round(same_ms, 4), "best_ms": round(bms, 4),
            "best_geometry": f"{bg[0]}wg/cu x{bg[1]}", "best_schedule": bname,
            "schedules": {k: {"best_ms": round(v[0], 4), "geometry": f"{v[1][0]}wg/cu x{v[1][1]}"}
                          for k, v in per.items()},
            "of_ceiling": round(bms / kernel_ms, 4)}


def aux_kernels(st, reps=20):
    """Informational, after the timed region: the other full-vector sweeps of
    the path at the same size, HIP-event timed on the launch stream —
    bdl_posterior_sample (theta_s = m1 + sqrt(var) * eps,
    Welford variance, Philox noise; m1 r, m2 r, out w = 12 B/elem) and
    bdl_moments_update (sgld.py:242-245 running mean / second moment: theta r,
    m1 rw, m2 rw = 20 B/elem)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import moment_pair
    n = st.n
    # the draw reads a cycle's Welford moments, allocated as the cSGHMC Runner
    # allocates them (flat.moment_pair: one allocation, two halves)
    m1, m2 = moment_pair(n, st.device)
    out = torch.empty(n, dtype=torch.float32, device=st.device)
    m1.copy_(st.theta)
    m2.fill_(1e-6)
    res = {}

    def timed(name, nbytes, fn):
        for _ in range(3):
            fn(0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i + 3)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = nbytes * n / (ms * 1e-3) / 1e9
        res[name] = {"avg_ms": round(ms, 4), "bytes_per_elem": nbytes, "gbs": round(gbs, 1),
                     "frac": round(gbs / PEAK_HBM_GBS, 4)}

    timed("posterior_sample", 12, lambda i: K.posterior_sample(
        out, m1, m2, var_mode=L.VAR_WELFORD, ratio=4.0, seed=7, chain=0, step=i))
    res["posterior_sample"]["moments"] = "flat.moment_pair"
    # the draw's own launch geometry: its tuned workgroups/CU x 4 groups
    geo = K.sample_geometry(n, st.device) or (2, 4)
    res["posterior_sample"]["geometry"] = f"{geo[0]}wg/cu x{geo[1]}"
    res["posterior_sample"]["mix_ceiling"] = mix_ceiling(
        [m1, m2], [out], geo, res["posterior_sample"]["avg_ms"])
    del m1, m2, out
    # the running moments of sgld / sghmc (methods/sgld.py:95-102 seeds them
    # from theta at burn-in), two allocations as the sgld Runner makes them
    s1, s2 = torch.empty_like(st.theta), torch.empty_like(st.theta)
    s1.copy_(st.theta)
    s2.fill_(1e-6)
    timed("moments_update", 20, lambda i: K.moments_update(
        st.theta, s1, s2, L.COLLECT_MEAN, collect_a=float(i + 1), collect_b=float(i + 2)))
    cfg = getattr(st, "launch_cfg", None) or (2, 4, 1)
    res["moments_update"]["mix_ceiling"] = mix_ceiling(
        [st.theta, s1, s2], [s1, s2], (cfg[0], 4), res["moments_update"]["avg_ms"])
    del s1, s2
    return res


def collect_init_timing(st, m1s, m2s, rank, reps=10):
    """Informational, after the timed region: the cSGHMC step that takes a
    cycle's FIRST sample (Philox noise + Welford init: m1 = theta', m2 = 0;
    methods/csghmc.py:333-337; 28 B/elem), once per cycle in a real run, on one
    of the run's own cycle pairs.  Step scalars as a sample step of config 4."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    c = min(m1s)
    lrs = (1e-5, 1e-3)
    ns = [0.01 * np.sqrt(2 * 0.18 * x) / 1840.0 for x in lrs]
    ms = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - 0.18, prior_sig=1.0, collect=L.COLLECT_WELFORD_INIT,
                      mom1=m1s[c], mom2=m2s[c], collect_a=1.0, seed=42 + rank, chain=rank,
                      step=1_000_000 + i)
        e1.record()
        torch.cuda.synchronize()
        if i:  # the first launch is a warm-up
            ms.append(e0.elapsed_time(e1))
    avg = float(np.mean(ms))
    gbs = BYTES_PER_ELEM["collect_init"] * st.n / (avg * 1e-3) / 1e9
    return {"avg_ms": round(avg, 4), "bytes_per_elem": BYTES_PER_ELEM["collect_init"],
            "gbs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4), "launches": reps}


def event_times(fn, reps, warm=1):
    """`reps` launches of fn(i), each bracketed by its own HIP events on the
    launch stream (after `warm` untimed ones); per-launch ms."""
    for i in range(warm):
        fn(i)
    ev = []
    for i in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(warm + i)
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def kind_stats(ms, bytes_per_elem, n):
    avg = float(np.mean(ms))
    gbs = bytes_per_elem * n / (avg * 1e-3) / 1e9
    return {"timed": len(ms), "avg_ms": round(avg, 4),
            "p10_ms": round(float(np.percentile(ms, 10)), 4),
            "p50_ms": round(float(np.percentile(ms, 50)), 4),
            "p90_ms": round(float(np.percentile(ms, 90)), 4),
            "bytes_per_elem": bytes_per_elem, "gbs": round(gbs, 1),
            "frac": round(gbs / PEAK_HBM_GBS, 4)}


def collect_steady_timing(st, m1s, m2s, spc, rank, reps=12):
    """Informational, after the timed region: the steady-state Welford collect
    (methods/csghmc.py:339-345: Philox noise + m1 / M2 update, 36 B/elem) on
    one of the run's own cycle pairs, `reps` separately bracketed launches
    (the timed region holds one per thin x 2 steps only)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    c = max(m1s)
    lrs = (1e-5, 1e-3)
    ns = [0.01 * np.sqrt(2 * 0.18 * x) / 1840.0 for x in lrs]
    cnt0 = spc[c] + 1

    def fn(i):
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      one_minus_alpha=1 - 0.18, prior_sig=1.0, collect=L.COLLECT_WELFORD,
                      mom1=m1s[c], mom2=m2s[c], collect_a=float(cnt0 + 2 * i), seed=42 + rank,
                      chain=rank, step=2_000_000 + i)
    return kind_stats(event_times(fn, reps), BYTES_PER_ELEM["collect"], st.n)


def explore_tensor_grad_timing(st, reps=20):
    """Informational, after the timed region: the explore step reading the
    gradient as the Runners read autograd's (default "tensor" gradient mode,
    methods/csghmc.py:741-778 reads each p.grad): one gradient tensor per
    parameter tensor (296 for ViT-L/32) through the per-run base table, on the
    same theta / momentum as the timed region, allocated in backward order
    (last tensor first) from torch's default pool, as the Runners' backward
    leaves them.  For comparison, the same 296 tensors from the gradient
    arena's pool (`arena`: arena.GradArena, one reservation, the Runners'
    BDL_GRAD_ARENA=1), and the same per-tensor table over 296 views of the ONE
    flat gradient allocation the headline reads (`one_allocation`: the table's
    own cost, no placement difference)."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import arena as A
    from bayesdll_amd import kernels as K
    flat = st.grad

    def fn(i):
        K.sgmcmc_step(st, L.CSGHMC, lrs=(1e-5, 1e-3), noise_scale=(0.0, 0.0),
                      noise_mode=L.NOISE_NONE, one_minus_alpha=1 - 0.18, prior_sig=1.0,
                      seed=0, chain=0, step=3_000_000 + i)

    def restore():
        st.grad_mode, st.grad, st.gbase, st._untouched = "flat", flat, None, ()
        st.runs, st.nruns = st._base_runs

    def backward_order(alloc):
        out = [None] * len(st.numels)
        for i in reversed(range(len(st.numels))):
            o, k = st.offsets[i], st.numels[i]
            out[i] = alloc(flat[o:o + k])
        return out

    def timed(grads):
        restore()
        st.use_tensor_grads(grads)
        return kind_stats(event_times(fn, reps, warm=2), BYTES_PER_ELEM["explore"], st.n)

    keys = ("avg_ms", "p10_ms", "p50_ms", "p90_ms", "frac")
    try:
        grads = backward_order(lambda v: v.clone())
        res = timed(grads)
        del grads
        arena = A.GradArena(st.device, 4 * st.n)
        with arena.routing():
            grads = backward_order(lambda v: v.clone())
        inside = all(A.contains(st.device, g) for g in grads)
        ar = timed(grads)
        del grads
        one = timed([flat[o:o + k] for o, k in zip(st.offsets, st.numels)])
    finally:
        restore()
    del arena
    res["gradients"] = (f"{len(st.numels)} per-tensor allocations from torch's default pool, "
                        "backward order (as the Runners' backward leaves them)")
    res["runs"] = len(st.numels)
    res["arena"] = dict({k: ar[k] for k in keys}, in_arena=inside)
    res["one_allocation"] = {k: one[k] for k in keys}
    return res


METHOD_LINES = {
    # config 3 (BASELINE.json): ResNet-101 SGLD + SGD(momentum 0.5), Philox
    # noise; sgld.py:469-484 + torch.optim.SGD: theta rw, g r, theta0 r, buf rw
    "sgld_rn101": ("resnet101", "sgld", "sgld", 24),
    # Adam-SGHMC + SGD(momentum 0.5) on ViT-L/32 (adam_sghmc.py:500-553 +
    # :229): theta, v_mom, m, v, buf rw; g, theta0 r
    "adam_vit": ("vit_l_32", "adam", "adam", 48),
}


def method_line(name, num_classes, rank, traffic_path, reps=20):
    """Informational, after the timed region: the steady-state sweep of
    another method on a fresh chain state of its named backbone (synthetic
    theta0 ~ N(0, 0.02^2), theta = theta0 + N(0, 1e-3^2), g ~ N(0, 1e-3^2);
    lr 1e-4 / 1e-2 on the readout, nd 0.01, N = 1840 x 1e3, SGD momentum 0.5,
    Philox noise): one first step (the SGD buffer is created, as in a run),
    then the launch geometry tuned on the state's own vectors at the first
    steady-state launch, then `reps` separately bracketed launches.  With its
    fraction of 8 TB/s, the bare access mix of its own buffers (mix_ceiling)
    and the committed PMC bytes per launch."""
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.flat import FlatState
    from bayesdll_amd.shapes import segments
    backbone, method, kind, nbytes = METHOD_LINES[name]
    segs, readout = segments(backbone, num_classes)
    adam = method == "adam"
    dev = torch.device("cuda", torch.cuda.current_device())
    st = FlatState.from_segments(segs, readout, device=dev, need_prior=True,
                                 extra=K.ADAM_EXTRA if adam else ())
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    st.prior.normal_(0.0, 0.02, generator=gen)
    st.theta.normal_(0.0, 1e-3, generator=gen).add_(st.prior)
    st.grad.normal_(0.0, 1e-3, generator=gen)
    lr, lr_head, nd, N, mu = 1e-4, 1e-2, 0.01, 1840.0 * 1e3, 0.5
    K.request_state_tuning(st, method)

    def fn(i, first=False):
        kw = dict(noise_mode=L.NOISE_PHILOX, sigma2=1.0, n_data=N, mu=mu, first_step=first,
                  momentum=True, seed=42 + rank, chain=rank, step=6_000_000 + i)
        if adam:
            m, v, buf = (st.extra[k] for k in K.ADAM_EXTRA)
            K.adam_step(st, L.ADAM_SGHMC, adam_m=m, adam_v=v, sgd_buf=buf, beta1=0.9,
                        beta2=0.999, eps=1e-8, t=i + 1, momentum_decay=0.18, nd=nd,
                        lrs=(lr, lr_head), **kw)
        else:
            K.sgmcmc_step(st, L.SGLD, lrs=(lr, lr_head),
                          noise_scale=[nd * np.sqrt(2 / (N * x)) for x in (lr, lr_head)],
                          prior_sig=1.0, **kw)
    fn(0, first=True)
    res = kind_stats(event_times(lambda i: fn(i + 1), reps, warm=2), nbytes, st.n)
    cfg = st.launch_cfg or (2, 1, 1)
    res.update({"workload": f"{backbone} {'Adam-SGHMC' if adam else 'SGLD'} + SGD(momentum 0.5)",
                "params": st.n, "tensors": len(segs),
                "geometry": f"{cfg[0]}wg/cu x{cfg[1]}",
                "tuned": (st.tuned.get("step") or {}).get("ms")})
    try:
        tj = json.load(open(traffic_path))
        res["traffic"] = tj.get(backbone, {}).get(kind)
    except Exception:  # noqa: BLE001
        res["traffic"] = None
    if adam:
        m, v, buf = (st.extra[k] for k in K.ADAM_EXTRA)
        rd = [st.theta, st.grad, st.prior, st.mom, m, v, buf]
        wr = [st.theta, st.mom, m, v, buf]
    else:
        rd, wr = [st.theta, st.grad, st.prior, st.mom], [st.theta, st.mom]
    res["mix_ceiling"] = mix_ceiling(rd, wr, cfg[:2], res["avg_ms"])
    del st
    torch.cuda.empty_cache()
    return res


def cpu_baseline(segs, readout, seconds):
    """The reference csghmc per-tensor update (oracle restatement, torch CPU,
    torch.randn_like per tensor) on the full ViT-L/32 shapes, timed for a
    bounded number of steps."""
    from oracle import sgmcmc_oracle as O
    # the box's CPU share (OMP_NUM_THREADS is set to it), not the whole machine
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    params = [torch.randn(s, generator=g) * 0.02 for _, s in segs]
    grads = [torch.randn(s, generator=g) * 1e-3 for _, s in segs]
    moms = [torch.zeros(s) for _, s in segs]
    names = [nm for nm, _ in segs]
    steps, t0 = 0, time.perf_counter()
    while True:
        moms = O.csghmc_step_cpu(params, grads, moms, names, readout, [1e-4, 1e-2], 1.0, 0.18,
                                 1840.0, 0.01, True)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 50:
            break
    cpu_model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": steps / el, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{steps} full ViT-L/32 cSGHMC updates (296 tensors, 306,535,400 params, "
                      f"randn_like noise) in {el:.1f} s on {cpu_model}"}


def e2e_steps(steps, warmup, local, seed, graph=False, overlap=False, arena=False):
    """Informational: full cSGHMC steps on a real ViT-L/32 (random init,
    synthetic [16,3,224,224] batch): forward + backward (PyTorch-ROCm fp32
    autograd; in eager mode with arena=True the gradients come from the
    gradient arena, BDL_GRAD_ARENA=1) + the fused update, reading autograd's
    per-tensor gradients.
    Returns ms/step and the fused update's own mean launch time on those
    gradients (HIP events on every launch after the warm-up)."""
    import bayesdll_amd.csghmc as csghmc
    from bayesdll_amd import kernels as K
    from bayesdll_amd.backbones import backbone
    dev = torch.device("cuda", local)
    prev = os.environ.get("BDL_GRAD_ARENA")
    os.environ["BDL_GRAD_ARENA"] = "1" if arena else "0"
    try:
        torch.manual_seed(seed)
        net = backbone("vit_l_32", 1000).to(dev)
        model = csghmc.Model(ND=1840, prior_sig=1.0, momentum_decay=0.18)
        model.noise_mode = "philox"
        model.graph = graph  # forward + backward replayed from a captured HIP graph
        model.overlap = overlap  # per-bucket update beside backward (captured too in graph mode)
        crit = torch.nn.CrossEntropyLoss()
        g = torch.Generator(device=dev).manual_seed(seed)
        x = torch.randn(16, 3, 224, 224, device=dev, generator=g)
        y = torch.randint(0, 1000, (16,), device=dev, generator=g)
        for k in range(warmup):
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 2 == 0))
    finally:
        if prev is None:
            os.environ.pop("BDL_GRAD_ARENA", None)
        else:
            os.environ["BDL_GRAD_ARENA"] = prev
    torch.cuda.synchronize()
    st = model.flat
    in_arena = None
    if st.arena is not None:
        from bayesdll_amd import arena as A
        in_arena = all(p.grad is None or A.contains(dev, p.grad) for p in st.params)
    t0 = time.perf_counter()
    for k in range(steps):
        model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 10 == 0))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # the sampler's whole per-step cost, host side included: sampler steps and
    # the same forward + backward + loss.item() with no sampler at all (grads
    # set to None as the sampler does) alternate step by step, each step
    # synchronised, so clock drift between the two legs cancels
    plain_ms = sync_ms = None
    if not graph and not overlap:
        params = list(net.parameters())

        def plain():
            for p in params:
                p.grad = None
            loss = crit(net(x), y)
            loss.backward()
            loss.item()
        ts = tp = 0.0
        for k in range(steps + 2):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 10 == 0))
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            plain()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            if k >= 2:
                ts += t2 - t1
                tp += t3 - t2
        sync_ms, plain_ms = ts / steps * 1e3, tp / steps * 1e3
    # the update alone on the Runner's own gradients, after the timed steps
    # (HIP events around each launch; 9 explore + 1 sample step per 10, 20 B/elem)
    st.timer = K.StepTimer(1)
    for k in range(min(steps, 20)):
        model(x, y, net, None, crit, [1e-4, 1e-2], 1.0, 0.01, should_sample=(k % 10 == 0))
    upd = st.timer.summary()
    st.timer = None
    ovl_graphs = sum(1 for k in model._graphs if "overlap" in k)
    rewrite_ms = (1e3 * model.overlap_rewrite_s / model.overlap_replays
                  if getattr(model, "overlap_replays", 0) else None)
    buckets = len(model._ovl_plan[1]) if getattr(model, "_ovl_plan", None) else None
    model.release_graphs()
    del net, model, st
    torch.cuda.empty_cache()
    return {"overlap_graphs": ovl_graphs, "rewrite_ms_per_step": rewrite_ms, "buckets": buckets,
            "steps_per_s": round(1e3 / ms, 2), "ms_per_step": round(ms, 3),
            "update_ms": round(upd["avg_ms"], 4) if upd.get("timed") else None,
            "synchronised_ms_per_step": None if sync_ms is None else round(sync_ms, 3),
            "autograd_only_ms": None if plain_ms is None else round(plain_ms, 3),
            "sampler_added_ms": None if plain_ms is None else round(sync_ms - plain_ms, 3),
            "grad_arena": arena and not graph, "grads_in_arena": in_arena,
            "batch": [16, 3, 224, 224], "what": "ViT-L/32 fp32 fwd+bwd (autograd) + fused cSGHMC "
            "update, loss.item() sync per step as in the reference (informational)"}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus))
    dist, rank, world, local = dist_setup(a.gpus)
    devices = rank_devices(dist, local, world) if dist is not None else None
    from bayesdll_amd import _lib as L
    from bayesdll_amd import kernels as K
    from bayesdll_amd.cyclical import CyclicalSGMCMC
    from bayesdll_amd.flat import FlatState, moment_pair
    from bayesdll_amd.shapes import segments

    segs, readout = segments(a.backbone, a.num_classes)
    # untimed: bring the GPU to its steady-state clocks, then tune the launch
    tune_method = {"csghmc": "csghmc", "sgld": "sgld", "adam_sghmc": "adam"}[a.method]
    n_all = sum(int(np.prod(s)) for _, s in segs)
    prewarm = {"seconds": a.prewarm_seconds,
               "launches": K.prewarm(n_all, local, tune_method, a.prewarm_seconds)
               if a.prewarm_seconds > 0 else 0,
               "why": "untimed setup: clock / power ramp of the first ~0.8 s of load "
                      "(tools/drift.py)"}
    tune_on_state = False
    if a.blocks_per_cu or a.unroll or a.grid_stride >= 0:
        K.set_launch_config(a.blocks_per_cu, a.unroll, max(a.grid_stride, 0))
        launch = {"blocks_per_cu": a.blocks_per_cu, "unroll": a.unroll,
                  "grid_stride": max(a.grid_stride, 0), "autotuned": False}
    elif not a.no_autotune:
        # untimed setup (like cudnn.benchmark): the launch geometry is tuned on
        # the chain's OWN vectors, as the Runners tune it, once the state
        # exists (below); results are identical under every geometry
        tune_on_state = True
        launch = {"autotuned": True, "tuned_on": f"{a.method} on the chain's own vectors "
                                                 "(kernels.request_state_tuning)"}
    else:
        launch = {"default": True, "autotuned": False}
    dev = torch.device("cuda", local)
    adam = a.method == "adam_sghmc"
    sgld = a.method == "sgld" or adam  # adam shares config 3's state/driver shape
    st = FlatState.from_segments(segs, readout, device=dev, need_prior=sgld,
                                 extra=("adam_m", "adam_v", "sgd_buf") if adam else ())
    gen = torch.Generator(device=dev).manual_seed(42 + rank)
    if sgld:  # config 3: theta0 ~ N(0, 0.02^2) (pretrained stand-in), theta = theta0 + N(0, 1e-3^2)
        st.prior.normal_(0.0, 0.02, generator=gen)
        st.theta.normal_(0.0, 1e-3, generator=gen).add_(st.prior)
    else:
        st.theta.normal_(0.0, 0.02, generator=gen)
    st.grad.normal_(0.0, 1e-3, generator=gen)
    n = st.n
    tensor_grads = None
    if a.grad_mode == "tensor":  # one gradient tensor per parameter, as autograd leaves them
        tensor_grads = [st.grad[o:o + k].clone() for o, k in zip(st.offsets, st.numels)]
        st.use_tensor_grads(tensor_grads)

    # config 4 hyper-parameters; config 3 for --method sgld
    lr, lr_head, alpha, nd, ND, Ninflate, prior_sig = 1e-4, 1e-2, 0.18, 0.01, 1840, 1.0, 1.0
    if sgld:
        Ninflate, mu = 1e3, 0.5
    N = ND * Ninflate
    total = a.warmup + a.steps
    sched = CyclicalSGMCMC(lr, a.cycles, 1, 0.5)  # one "epoch" of `total` batches
    m1s, m2s, spc = {}, {}, {}
    # The per-cycle Welford buffers (the reference clones theta at a cycle's
    # first sample, methods/csghmc.py:333-337) are allocated AND initialised
    # before the timed region: a real cycle spans thousands of batches, in
    # which the clone happens once and every later thinned sample step is the
    # steady-state Welford update (:339-345, 36 B/elem), while this bench
    # compresses `cycles` cycles into warmup+steps batches.  So each cycle's
    # pair starts as the Runner leaves it after its first sample (m1 = theta,
    # m2 = 0, samples_per_cycle = 2 by quirk Q2), and every timed collect is
    # the steady-state kind; the init launch (28 B/elem) is timed on its own
    # after the timed region (`collect_init` in aux_kernels).
    pre, t_alloc = {}, time.perf_counter()
    if not sgld:
        for k in range(total):
            if sched.should_sample(0, k, total) and k % a.thin == 0:
                c = sched.get_cycle_number(0, k, total)
                if c not in m1s:  # as the cSGHMC Runner allocates them
                    m1s[c], m2s[c] = moment_pair(n, dev)
                    m1s[c].copy_(st.theta)
                    m2s[c].zero_()
                    spc[c] = 2
                    pre[c] = True
    torch.cuda.synchronize()
    moment_buffers = {"cycles": len(pre), "alloc_ms": round((time.perf_counter() - t_alloc) * 1e3, 1),
                      "state": "initialised before the timed region (first sample of the cycle "
                               "taken): timed collects are the steady-state Welford update"}
    if sgld:  # sgld.py:95-102 burn-in seeding (burnin = 0), outside the timed region
        m1s[0] = torch.empty(n, dtype=torch.float32, device=dev)
        m2s[0] = torch.empty(n, dtype=torch.float32, device=dev)
        K.moments_update(st.theta, m1s[0], m2s[0], L.COLLECT_MEAN_INIT)
        spc[0] = 1

    def sgld_step(k, timer=None):
        """methods/sgld.py:193-250: Model + SGD(momentum 0.5) + running moments
        every `thin` iterations, fused."""
        first = k == 0
        collect = (k + 1) % a.thin == 0
        kind = "sgld_first" if first else ("sgld_collect" if collect else "sgld")
        lrs = (lr, lr_head)
        ns = [nd * np.sqrt(2 / (N * x)) for x in lrs]
        cnt = spc[0]
        ev = timer.begin(kind) if timer is not None else None
        K.sgmcmc_step(st, L.SGLD, lrs=lrs, noise_scale=ns, noise_mode=L.NOISE_PHILOX,
                      prior_sig=prior_sig, sigma2=prior_sig ** 2, n_data=N, mu=mu,
                      first_step=first, momentum=True,
                      collect=L.COLLECT_MEAN if collect else L.COLLECT_NONE, mom1=m1s[0],
                      mom2=m2s[0], collect_a=float(cnt), collect_b=float(cnt + 1),
                      seed=42 + rank, chain=rank, step=k)
        if ev is not None:
            ev[1].record()
        if collect:
            spc[0] = cnt + 1
        return kind

    if adam:
        adam_m, adam_v, sgd_buf = st.extra["adam_m"], st.extra["adam_v"], st.extra["sgd_buf"]

    def adam_step(k, timer=None):
        """methods/adam_sghmc.py:458-553 + SGD(momentum 0.5) (:60, :229) +
        running moments every `thin` iterations, fused."""
        first = k == 0
        collect = (k + 1) % a.thin == 0
        kind = "adam_first" if first else ("adam_collect" if collect else "adam")
        cnt = spc[0]
        ev = timer.begin(kind) if timer is not None else None
        K.adam_step(st, L.ADAM_SGHMC, adam_m=adam_m, adam_v=adam_v, sgd_buf=sgd_buf, beta1=0.9,
                    beta2=0.999, eps=1e-8, t=k + 1, momentum_decay=alpha, nd=nd,
                    lrs=(lr, lr_head), noise_mode=L.NOISE_PHILOX, sigma2=prior_sig ** 2,
                    n_data=N, mu=mu, first_step=first, momentum=True,
                    collect=L.COLLECT_MEAN if collect else L.COLLECT_NONE, mom1=m1s[0],
                    mom2=m2s[0], collect_a=float(cnt), collect_b=float(cnt + 1),
                    seed=42 + rank, chain=rank, step=k)
        if ev is not None:
            ev[1].record()
        if collect:
            spc[0] = cnt + 1
        return kind

    def plan(k):
        cur = sched.calculate_lr(0, k, total)
        ss = sched.should_sample(0, k, total) and k % a.thin == 0
        kind, collect, spec = ("sample" if ss else "explore"), L.COLLECT_NONE, None
        if ss:  # every cycle's pair is initialised before the run (above)
            c = sched.get_cycle_number(0, k, total)
            cnt = spc[c] + 1
            spec = (L.COLLECT_WELFORD, c, float(cnt), cnt)
            kind = "collect"
        return cur, ss, kind, spec

    def step(k, timer=None):
        cur, ss, kind, spec = plan(k)
        lrs = (cur, cur * (lr_head / lr))
        ns = [nd * np.sqrt(2 * alpha * x) / N for x in lrs]
        ckind, m1, m2, ca = L.COLLECT_NONE, None, None, 1.0
        if spec is not None:
            ckind, c, ca, cnt = spec
            m1, m2 = m1s[c], m2s[c]
        ev = timer.begin(kind) if timer is not None else None
        K.sgmcmc_step(st, L.CSGHMC, lrs=lrs, noise_scale=ns,
                      noise_mode=L.NOISE_PHILOX if ss else L.NOISE_NONE,
                      one_minus_alpha=1 - alpha, prior_sig=prior_sig, collect=ckind, mom1=m1,
                      mom2=m2, collect_a=ca, seed=42 + rank, chain=rank, step=k)
        if ev is not None:
            ev[1].record()
        if spec is not None:  # the reference's double increment (quirk Q2)
            spc[c] = cnt + 1
        return kind

    if sgld:
        step = adam_step if adam else sgld_step  # noqa: F811
    if tune_on_state:
        # the first launch of each kind (plain step, collect step) tunes the
        # geometry on this state's buffers with its own arguments (every vector
        # it writes restored after each candidate), then runs once; the state
        # is restored from a snapshot afterwards, so the run starts where it was
        K.request_state_tuning(st, tune_method)
        cyc = min(m1s) if m1s else None
        touched = [st.theta, st.mom] + ([st.extra[k] for k in ("adam_m", "adam_v", "sgd_buf")]
                                        if adam else []) + \
            ([m1s[cyc], m2s[cyc]] if cyc is not None else [])
        snap = [v.clone() for v in touched]
        kw = dict(seed=42 + rank, chain=rank, step=0)
        for collect in (False, True):
            if adam:
                K.adam_step(st, L.ADAM_SGHMC, adam_m=adam_m, adam_v=adam_v, sgd_buf=sgd_buf,
                            beta1=0.9, beta2=0.999, eps=1e-8, t=2, momentum_decay=alpha, nd=nd,
                            lrs=(lr, lr_head), noise_mode=L.NOISE_PHILOX,
                            sigma2=prior_sig ** 2, n_data=N, mu=mu, momentum=True,
                            collect=L.COLLECT_MEAN if collect else L.COLLECT_NONE,
                            mom1=m1s[cyc], mom2=m2s[cyc], collect_a=1.0, collect_b=2.0, **kw)
            elif sgld:
                K.sgmcmc_step(st, L.SGLD, lrs=(lr, lr_head),
                              noise_scale=[nd * np.sqrt(2 / (N * x)) for x in (lr, lr_head)],
                              noise_mode=L.NOISE_PHILOX, prior_sig=prior_sig,
                              sigma2=prior_sig ** 2, n_data=N, mu=mu, momentum=True,
                              collect=L.COLLECT_MEAN if collect else L.COLLECT_NONE,
                              mom1=m1s[cyc], mom2=m2s[cyc], collect_a=1.0, collect_b=2.0, **kw)
            else:
                K.sgmcmc_step(st, L.CSGHMC, lrs=(lr, lr_head),
                              noise_scale=(1e-7, 1e-7) if collect else (0.0, 0.0),
                              noise_mode=L.NOISE_PHILOX if collect else L.NOISE_NONE,
                              one_minus_alpha=1 - alpha, prior_sig=prior_sig,
                              collect=L.COLLECT_WELFORD if collect else L.COLLECT_NONE,
                              mom1=m1s[cyc] if collect else None,
                              mom2=m2s[cyc] if collect else None, collect_a=3.0, **kw)
        if not sgld and cyc is not None:  # a cycle's first collect (Welford init) too
            K.sgmcmc_step(st, L.CSGHMC, lrs=(lr, lr_head), noise_scale=(1e-7, 1e-7),
                          noise_mode=L.NOISE_PHILOX, one_minus_alpha=1 - alpha,
                          prior_sig=prior_sig, collect=L.COLLECT_WELFORD_INIT, mom1=m1s[cyc],
                          mom2=m2s[cyc], collect_a=1.0, **kw)
        torch.cuda.synchronize()
        for v, s0 in zip(touched, snap):
            v.copy_(s0)
        del snap
        # the geometry each kind actually runs at (kernels._use_geometry):
        # the tuned one, or — tuning skipped — whatever is installed
        tuned = getattr(st, "tuned", {})
        best, cbest, ibest = st.launch_cfg, st.collect_cfg, getattr(st, "init_cfg", None)
        launch.update({
            "step": ({"blocks_per_cu": best[0], "unroll": best[1], "grid_stride": best[2],
                      "candidates_ms": tuned.get("step", {}).get("ms")} if best is not None else
                     {"untuned": tuned.get("step"), "installed": K._ACTIVE[0] or "library default"}),
            # the collect steps' own geometry; untuned, they run at the step's
            "collect": ({"blocks_per_cu": cbest[0], "unroll": cbest[1],
                         "candidates_ms": tuned.get("collect", {}).get("ms")} if cbest is not None
                        else {"untuned": tuned.get("collect"), "runs_at": "the step's geometry"}),
            # a cycle's first collect (Welford init)
            "init": ({"blocks_per_cu": ibest[0], "unroll": ibest[1],
                      "candidates_ms": tuned.get("init", {}).get("ms")} if ibest is not None
                     else {"untuned": tuned.get("init"), "runs_at": "the step's geometry"})})
    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize()
    timer = LaunchTimer(a.event_stride or max(1, min(5, a.steps // 10)))
    kinds = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        kinds.append(step(a.warmup + i, timer))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:  # max over ranks (outside the timed region)
        on_dev = dist.get_backend() != "gloo"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(st.theta[:1 << 20]).all()
    collective = None
    if dist is not None:
        # informational, after the timed region: the one cross-chain exchange
        # (posterior-predictive average of a [128, 1000] fp32 batch, bayesdll_amd.chains)
        from bayesdll_amd import chains
        logp = torch.log_softmax(torch.randn(128, 1000, device=dev if dist.get_backend() != "gloo"
                                             else "cpu"), dim=1)
        for _ in range(3):
            chains.average_predictive(logp)
        if logp.is_cuda:
            torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(20):
            out_lp = chains.average_predictive(logp)
        if logp.is_cuda:
            torch.cuda.synchronize()
        collective = {"op": "all_reduce(SUM) of [128, 1000] fp32 predictive (chains.average_predictive)",
                      "backend": dist.get_backend(),
                      "ms": round((time.perf_counter() - t1) / 20 * 1e3, 4),
                      "finite": bool(torch.isfinite(out_lp).all())}
        if dist.get_backend() != "gloo" and os.environ.get("BDL_BENCH_POOL", "1") != "0":
            # the optional cross-chain pooled posterior mean: one full-vector
            # all-reduce (1.2 GB for ViT-L/32) over RCCL / xGMI
            pool_timing(chains, st, world, dist, collective)

    per = timer.durations()
    table = {}
    for kind, ms in per.items():
        avg = float(np.mean(ms))
        gbs = BYTES_PER_ELEM[kind] * n / (avg * 1e-3) / 1e9
        table[kind] = {"launches": kinds.count(kind), "timed": len(ms), "avg_ms": round(avg, 4),
                       "p10_ms": round(float(np.percentile(ms, 10)), 4),
                       "p50_ms": round(float(np.percentile(ms, 50)), 4),
                       "p90_ms": round(float(np.percentile(ms, 90)), 4),
                       "bytes_per_elem": BYTES_PER_ELEM[kind], "gbs": round(gbs, 1)}
    dominant = max(table, key=lambda k: table[k]["launches"] * table[k]["avg_ms"])
    dom = table[dominant]
    alg_bytes = dom["bytes_per_elem"] * n
    achieved = alg_bytes / (dom["avg_ms"] * 1e-3) / 1e9
    traffic = None
    if os.path.exists(a.traffic):
        try:
            tj = json.load(open(a.traffic))
            traffic = tj.get(a.backbone, {}).get(dominant)
        except Exception:
            traffic = None
    total_bytes = sum(BYTES_PER_ELEM[k] * n for k in kinds)
    hbm_gbs = total_bytes / elapsed / 1e9  # per rank, algorithmic, wall-clock

    out = {
        "metric": "SG-HMC leapfrog steps/sec & HBM GB/s on ViT-L/32 params, 1/2/4/8 MI355X",
        "value": round(world * a.steps / elapsed, 2),
        "unit": "steps/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (random-init theta, resident synthetic grad buffer)",
        "config": {"workload": (f"{a.backbone} cSGHMC fused leapfrog update (config 4/5)" if not sgld
                                else f"{a.backbone} Adam-SGHMC + SGD(momentum 0.5) fused update"
                                if adam else
                                f"{a.backbone} SGLD + SGD(momentum 0.5) fused update (config 3)"),
                   "params": n, "tensors": len(segs), "readout": readout,
                   "cycles": a.cycles, "thin": a.thin, "beta": 0.5, "noise": "philox",
                   "parallelism": f"{world} independent chains (1/GPU)",
                   "grad_mode": a.grad_mode, "allocator": "torch caching allocator"},
        "hbm_gbs": round(hbm_gbs * world, 1),
        "eval_collective": collective,
        "launch": launch,
        "prewarm": prewarm,
        "moment_buffers": moment_buffers,
        "kernels": table,
        "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 1),
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": traffic,
                     # not this run's counters: rocprofv3 PMC (FETCH/WRITE_SIZE passes) of the
                     # same kernel on the same workload, per launch, committed under profiles/
                     "traffic_kind": "profile (committed rocprofv3 PMC passes, not this run)",
                     "traffic_source": (f"{os.path.relpath(a.traffic, ROOT)}[{a.backbone}][{dominant}]"
                                        if traffic is not None else None),
                     "alg_bytes_per_launch": alg_bytes},
    }
    # after the timed region, on the same state: the steady-state collect over
    # enough launches for percentiles, and the explore step on per-tensor
    # gradients (the Runners' default gradient mode)
    if not sgld and m1s:
        table["collect_steady"] = dict(collect_steady_timing(st, m1s, m2s, spc, rank),
                                       launches=0, timed_region=False)
    if not sgld and a.grad_mode == "flat":
        ex = explore_tensor_grad_timing(st)
        ex["vs_flat_explore"] = round(ex["avg_ms"] / table["explore"]["avg_ms"], 4) \
            if "explore" in table else None
        table["explore_tensor_grad"] = dict(ex, launches=0, timed_region=False)
    out["methodology"] = {
        "timed_kinds": sorted(set(kinds)),
        "event_stride": timer.stride,
        "collect_init": "timed after the region (aux_kernels.collect_init): every cycle's Welford "
                        "pair is initialised before it",
        "post_region_kinds": [k for k, v in table.items() if v.get("timed_region") is False],
        "since": "round 3 (rounds 1-2: every launch bracketed, the init collect inside the region)"}
    if dist is not None:
        # every rank's own dominant-kernel time (rank 0's is the roofline
        # above): the slowest GPU sets the aggregate's wall clock
        mine = {"rank": rank, "kernel": dominant, "avg_ms": dom["avg_ms"]}
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        out["per_rank"] = [{"rank": r["rank"], "kernel": r["kernel"], "avg_ms": r["avg_ms"],
                            "frac": round(alg_bytes / (r["avg_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                            **devices[i]}
                           for i, r in enumerate(allr)]
        out["distributed"] = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                              "device_count": devices[0]["device_count"],
                              "distinct_devices": len({(d["pci"], d["uuid"]) for d in devices})}
    if not a.no_aux:
        out["aux_kernels"] = aux_kernels(st)
        if not sgld and m1s:
            out["aux_kernels"]["collect_init"] = collect_init_timing(st, m1s, m2s, rank)
        try:  # HBM bytes per launch of the same sweeps from the committed PMC profile
            tj = json.load(open(a.traffic))
            for k, v in out["aux_kernels"].items():
                v["traffic"] = tj.get(a.backbone, {}).get(k)
        except Exception:  # noqa: BLE001
            pass
    # last on this state (they overwrite the vectors): each kind's access mix,
    # bare, on the same buffers — the dominant kernel's, the steady-state
    # Welford collect's (5 reads, 4 writes, in place) and the cycle-init
    # collect's (3 reads, 4 writes), each at its own geometry and the best of
    # MIX_GEOMS
    manual = (max(a.blocks_per_cu, 1), max(a.unroll, 1), 1)
    cfg = (st.launch_cfg or manual) if launch.get("autotuned") else manual
    ccfg = (st.collect_cfg or cfg) if launch.get("autotuned") else manual
    bare_kw = dict(lrs=(1e-5, 1e-3), noise_scale=(0.0, 0.0), noise_mode=L.NOISE_NONE,
                   one_minus_alpha=1 - 0.18, prior_sig=1.0)
    if not adam:
        rd = [st.theta, st.grad] + ([st.prior] if sgld else []) + [st.mom]
        out["roofline"]["mix_ceiling"] = mix_ceiling(
            rd, [st.theta, st.mom], cfg[:2], dom["avg_ms"],
            step=None if sgld else (lambda: K.sgmcmc_step_bare(st, **bare_kw)))
    else:
        ex = st.extra
        out["roofline"]["mix_ceiling"] = mix_ceiling(
            [st.theta, st.grad, st.prior, st.mom, ex["adam_m"], ex["adam_v"], ex["sgd_buf"]],
            [st.theta, st.mom, ex["adam_m"], ex["adam_v"], ex["sgd_buf"]], cfg[:2], dom["avg_ms"])
    if not sgld and m1s:
        cm1, cm2 = m1s[max(m1s)], m2s[max(m1s)]  # the pair collect_steady ran on
        if "collect_steady" in table:
            table["collect_steady"]["mix_ceiling"] = mix_ceiling(
                [st.theta, st.grad, st.mom, cm1, cm2], [st.theta, st.mom, cm1, cm2], ccfg[:2],
                table["collect_steady"]["avg_ms"],
                step=lambda: K.sgmcmc_step_bare(st, collect=L.COLLECT_WELFORD, mom1=cm1, mom2=cm2,
                                                collect_a=3.0, **bare_kw))
        ci = (out.get("aux_kernels") or {}).get("collect_init")
        if ci is not None:
            icfg = (getattr(st, "init_cfg", None) or cfg) if launch.get("autotuned") else manual
            c0 = min(m1s)  # the pair collect_init_timing ran on (placement differs per pair)
            ci["mix_ceiling"] = mix_ceiling(
                [st.theta, st.grad, st.mom], [st.theta, st.mom, m1s[c0], m2s[c0]], icfg[:2],
                ci["avg_ms"],
                step=lambda: K.sgmcmc_step_bare(st, collect=L.COLLECT_WELFORD_INIT, mom1=m1s[c0],
                                                mom2=m2s[c0], collect_a=1.0, **bare_kw))
    del st, m1s, m2s
    torch.cuda.empty_cache()
    if world == 1 and not sgld and not a.no_methods:
        # the other BASELINE configurations' sweeps, driver-timed on their own
        # chain states (config 3: ResNet-101 SGLD; Adam-SGHMC on ViT-L/32)
        out["methods"] = {nm: method_line(nm, a.num_classes, rank, a.traffic)
                          for nm in METHOD_LINES}
    if world == 1 and a.e2e_steps > 0 and a.backbone == "vit_l_32" and not sgld:
        e2e = e2e_steps(a.e2e_steps, 3, local, 42)
        e2e["fused_update_share"] = round(dom["avg_ms"] / e2e["ms_per_step"], 4)
        if e2e["update_ms"] and "explore" in table:
            e2e["update_vs_flat_explore"] = round(e2e["update_ms"] / table["explore"]["avg_ms"], 4)
        # the same Runner with its gradients from the gradient arena (BDL_GRAD_ARENA=1)
        en = e2e_steps(a.e2e_steps, 3, local, 42, arena=True)
        e2e["arena"] = {k: en[k] for k in ("ms_per_step", "update_ms", "grads_in_arena")}
        eg = e2e_steps(a.e2e_steps, 3, local, 42, graph=True)
        e2e["graph_ms_per_step"] = eg["ms_per_step"]
        e2e["graph_steps_per_s"] = eg["steps_per_s"]
        e2e["graph_update_ms"] = eg["update_ms"]
        # the update captured in the graph, bucket by bucket beside backward
        if os.environ.get("BDL_BENCH_GRAPH_OVERLAP", "0") == "1":
            eo = e2e_steps(a.e2e_steps, 3, local, 42, graph=True, overlap=True)
            e2e["graph_overlap_ms_per_step"] = eo["ms_per_step"]
            e2e["graph_overlap_graphs"] = eo["overlap_graphs"]
            e2e["graph_overlap_buckets"] = eo["buckets"]
            e2e["graph_overlap_rewrite_ms_per_step"] = eo["rewrite_ms_per_step"]
        out["e2e"] = e2e
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not sgld:
        out["cpu_baseline"] = cpu_baseline(segs, readout, a.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
