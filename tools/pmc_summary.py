"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/.

* kernel stats (rocprofv3 --kernel-trace --stats) copied as-is;
* FETCH_SIZE / WRITE_SIZE per dispatch of the fused step kernels (separate
  PMC passes), reduced to mean HBM bytes per launch per kernel kind, with the
  gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of a
  16-B/lane streaming read, so bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024;
* profiles/pmc_traffic.json updated (read by bench.py for roofline.traffic).

usage: python tools/pmc_summary.py <tag> [dest subdir, e.g. round1/kernel_v3] [backbone]
"""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KIND = {(0, 0): "explore", (2, 0): "sample", (2, 1): "collect_init", (2, 2): "collect"}


# bdl_step_kernel<METHOD=2 (SGLD), NOISE, COLLECT, UNROLL>
SGLD_KIND = {(2, 0): "sgld", (2, 4): "sgld_collect"}
# bdl_adam_kernel<NOISE, COLLECT, GRADONLY>
ADAM_KIND = {(2, 0): "adam", (2, 4): "adam_collect"}
FIRST_OF = {"sgld": "sgld_first", "adam": "adam_first"}  # SGD buffer created: fewer reads


def kind_of(name):
    # the stand-alone sweeps bench.py times after its timed region (aux_kernels)
    if "bdl_sample_kernel" in name:
        return "posterior_sample"
    if "bdl_moments_kernel" in name:
        return "moments_update"
    m = re.search(r"bdl_step_kernel<(\d+), (\d+), (\d+), (\d+)>", name)
    if m and int(m.group(1)) == 0:
        return KIND.get((int(m.group(2)), int(m.group(3))))
    if m and int(m.group(1)) == 2:
        return SGLD_KIND.get((int(m.group(2)), int(m.group(3))))
    m = re.search(r"bdl_adam_kernel<(\d+), (\d+), false(?:, \d+)?>", name)
    if m:
        return ADAM_KIND.get((int(m.group(1)), int(m.group(2))))
    return None


def main(tag, dest=None, backbone="vit_l_32"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", dest or tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, "bench_kernel_stats.csv"))
    # the bench's timed region is the tail of the trace: the dominant kernel's
    # last `timed` dispatches (setup launches — the autotune candidates — come
    # first and would bias the stats average)
    timed = int(os.environ.get("TIMED_LAUNCHES", "190"))
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(trace):
        rows = list(csv.DictReader(open(trace)))
        by = {}
        for r in rows:
            by.setdefault(r["Kernel_Name"], []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for v in by.values():
            v.sort()
        # the timed loop's dominant kernel = the step kernel dispatched most
        # (bench.py times the collect-init kind after its timed region, so the
        # LAST step dispatch is not the timed loop's)
        step_kernels = {nm: v for nm, v in by.items() if "bdl_step_kernel" in nm or
                        "bdl_adam_kernel" in nm}
        if step_kernels:
            nm = max(step_kernels, key=lambda k: len(step_kernels[k]))
            # SKIP_LAST: launches of the same kernel after the timed region
            # (bench.py explore_tensor_grad: 2 x 22, per-tensor allocations
            # and views of the flat gradient)
            skip = int(os.environ.get("SKIP_LAST", "0"))
            durs = [d for _, d in step_kernels[nm]]
            durs = (durs[:-skip] if skip else durs)[-timed:]
            json.dump({"kernel": nm, "timed_launches": len(durs),
                       "avg_ns": round(sum(durs) / len(durs), 1), "skipped_last": skip,
                       "note": "mean of the last dispatches of the kernel the timed loop ran "
                               "(rocprofv3 --kernel-trace), to compare with bench.py's HIP-event "
                               "average for the same kernel"},
                      open(os.path.join(dst, "timed_region.json"), "w"), indent=1)
    acc = {}
    for sub, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        rows = [r for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv")))
                if any(k in r["Kernel_Name"] for k in ("bdl_step_kernel", "bdl_adam_kernel",
                                                       "bdl_sample_kernel", "bdl_moments_kernel"))]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        with open(os.path.join(dst, f"pmc_{sub}.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name",
                                              "Counter_Value", "VGPR_Count", "SGPR_Count",
                                              "Grid_Size", "LDS_Block_Size"],
                               extrasaction="ignore")
            w.writeheader()
            for r in rows:
                w.writerow(r)
                k = kind_of(r["Kernel_Name"])
                if k:
                    acc.setdefault(k, {}).setdefault(counter, []).append(float(r["Counter_Value"]))
    # keep the full-size dispatches of each kind (counter >= 0.6 x the kind's
    # largest): smaller launches of the same kernel (tests of other sizes in
    # the same process) would bias the mean
    for d in acc.values():
        fetch = d.get("FETCH_SIZE")
        if fetch:
            big = max(fetch)
            d["FETCH_SIZE"] = [v for v in fetch if v >= 0.6 * big]
        write = d.get("WRITE_SIZE")
        if write:
            big = max(write)
            d["WRITE_SIZE"] = [v for v in write if v >= 0.6 * big]
    # the run's first step (SGD buffer created: no buffer read) is the one
    # dispatch of its kind with clearly less FETCH; autotune launches come
    # earlier, so find it by its bytes, not its position
    for k, first in FIRST_OF.items():
        d = acc.get(k)
        if not d or "FETCH_SIZE" not in d or len(d["FETCH_SIZE"]) < 3:
            continue
        f = d["FETCH_SIZE"]
        i = min(range(len(f)), key=f.__getitem__)
        n = len(f)
        if f[i] < 0.95 * sorted(f)[n // 2] and all(len(v) == n for v in d.values()):
            acc[first] = {c: [v.pop(i)] for c, v in d.items()}
    traffic, raw = {}, {}
    for k, d in acc.items():
        raw[k] = {c: sum(v) / len(v) for c, v in d.items()}
        if "FETCH_SIZE" in raw[k] and "WRITE_SIZE" in raw[k]:
            traffic[k] = int((2 * raw[k]["FETCH_SIZE"] + raw[k]["WRITE_SIZE"]) * 1024)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    out.setdefault(backbone, {}).update(traffic)
    out.setdefault("_sources", {})[backbone + ":" + ",".join(sorted(traffic))] = \
        f"profiles/{dest or tag}"
    out["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; bytes "
                      "per launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
                      "reports half of a 16-B/lane streaming read, MI355X_MICROARCH.md)")
    out.setdefault("_raw_kib_per_launch", {}).setdefault(backbone, {}).update(raw)
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({backbone: traffic, "raw": raw}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "vit_l_32")
