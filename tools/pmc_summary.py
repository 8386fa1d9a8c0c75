#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of `bench.py --pmc-plan` per launch unit.

tools/pmc_box.sh runs the bench's own tuning, then K steps on ONE lane at the bench's
per-lane batch (a fixed dispatch order), once per counter pass:
  fetch: FETCH_SIZE          write: WRITE_SIZE          sq: SQ timing + MFMA counters
Each pass's last K x len(plan) `tic::` dispatches are matched, in order, against the
launch plan of one step (bench.py writes it: unit = layer, or 'a+b' for a fused pair, and
the kernel instance it launches), so every number below belongs to one layer at one shape
— a kernel template used at two shapes (model_3's 64x64 and 32x32 residual convs) is two
units.  Per unit the median over the K occurrences.

HBM bytes (MI355X_MICROARCH.md §HBM): WRITE_SIZE is exact for 16-B-per-lane stores.
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read on gfx950,
so it is doubled for the kernels whose loads are 16 B per lane (every f32 conv kernel); the
first-layer kernels read u8 RGB with narrow loads, for which the doubling does not hold
(r01: conv_rgb_s2 measured 6.9 MB raw against 6.3 MB of algorithmic reads plus the
staged halo, so x1), and keep the raw figure.

MFMA busy: SQ_VALU_MFMA_BUSY_CYCLES (cycles summed over the 1024 SIMDs) / (1024 x the
dispatch's duration in the SAME pass x 2.4 GHz) — a lower bound, exact at the maximum
clock.  No clock is derived from GRBM_GUI_ACTIVE: on dispatches shorter than ~0.3 ms that
quotient reads high (MI355X_MICROARCH.md, DVFS give-back).

Every pass replays one tuning state (bench.py --tune-cache), and the plans the three
passes wrote must be identical.

Output: JSON {"_meta": plan meta + source stamp, "units": {unit: {...}}}; bench.py uses it
for roofline.traffic only when the stamp and configuration match."""
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLOCK_GHZ = 2.4
SIMDS = 1024
NARROW_READ = ("conv_rgb_s2_kernel", "enc01_kernel")  # u8 RGB input: FETCH_SIZE not doubled


def norm(name):
    """'void tic::conv3x3_kernel<1, 32, 32, ...>(tic::ConvArgs)' -> 'conv3x3<1,32,32,...>'."""
    n = name.replace("void ", "").split("(")[0].replace(" ", "").replace("tic::", "")
    return n.replace("conv3x3_kernel<", "conv3x3<")


def load(path):
    """dispatch id -> (kernel, duration us, {counter: value}) for the tic:: dispatches."""
    disp = {}
    for r in csv.DictReader(open(path)):
        if "tic::" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        if d not in disp:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            disp[d] = (norm(r["Kernel_Name"]), dur, {}, int(r.get("Grid_Size", 0) or 0))
        disp[d][2][r["Counter_Name"]] = disp[d][2].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[d] for d in sorted(disp)]


def label(dispatches, plan, steps):
    """Match the last steps x len(plan) dispatches against the plan; unit -> [dispatch]."""
    n = steps * len(plan)
    if len(dispatches) < n:
        raise SystemExit(f"only {len(dispatches)} tic dispatches, plan needs {n}")
    tail = dispatches[-n:]
    out = defaultdict(list)
    for i, dsp in enumerate(tail):
        want = plan[i % len(plan)]
        if dsp[0] != want["kernel"]:
            raise SystemExit(f"dispatch {i}: kernel {dsp[0]} but the plan has {want['kernel']} ({want['unit']})")
        out[want["unit"]].append(dsp)
    return out


def main(out_dir, out_path):
    passes, plans = {}, {}
    for kind in ("fetch", "write", "sq"):
        p = os.path.join(out_dir, f"pmc_{kind}", "p_counter_collection.csv")
        pp = os.path.join(out_dir, f"plan_{kind}.json")
        if os.path.exists(p) and os.path.exists(pp):
            plans[kind] = json.load(open(pp))
            passes[kind] = label(load(p), plans[kind]["plan"], plans[kind]["_meta"]["steps"])
    if not plans:
        raise SystemExit("no PMC pass found")
    first = next(iter(plans.values()))
    plan, meta = first["plan"], dict(first["_meta"])
    for kind, pd in plans.items():  # every pass must have launched the same kernels
        if pd["plan"] != plan or pd["_meta"]["source_sha256"] != meta["source_sha256"]:
            raise SystemExit(f"pass {kind} launched a different plan: the tuning replay did not hold")
    med = lambda v: statistics.median(v) if v else None
    units = {}
    print(f"{'unit':34s} {'kernel':44s} {'us':>7s} {'readMB':>8s} {'writeMB':>8s} {'GB/s':>6s} {'mfma%lb':>7s} {'wait%':>6s}")
    for u in [p["unit"] for p in plan]:
        kern = next(p["kernel"] for p in plan if p["unit"] == u)
        e = {"kernel": kern}
        if "fetch" in passes:
            fac = 1 if kern.startswith(NARROW_READ) else 2
            e["read_bytes"] = fac * 1024 * med([d[2].get("FETCH_SIZE", 0) for d in passes["fetch"][u]])
            e["fetch_factor"] = fac
            e["us_fetch_pass"] = med([d[1] for d in passes["fetch"][u]])
            e["grid_size"] = passes["fetch"][u][0][3]
        if "write" in passes:
            e["write_bytes"] = 1024 * med([d[2].get("WRITE_SIZE", 0) for d in passes["write"][u]])
        if "read_bytes" in e and "write_bytes" in e:
            e["bytes"] = e["read_bytes"] + e["write_bytes"]
        if "sq" in passes:
            ds = passes["sq"][u]
            us = med([d[1] for d in ds])
            e["us"] = us
            busy = med([d[2].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in ds])
            e["mfma_busy_pct_lb"] = 100.0 * busy / (SIMDS * us * 1e3 * CLOCK_GHZ) if us else None
            wav = med([d[2].get("SQ_WAVE_CYCLES", 0) for d in ds])
            e["wait_pct"] = 100.0 * med([d[2].get("SQ_WAIT_ANY", 0) for d in ds]) / wav if wav else None
            e["wait_inst_pct"] = 100.0 * med([d[2].get("SQ_WAIT_INST_ANY", 0) for d in ds]) / wav if wav else None
        units[u] = e
        us = e.get("us") or e.get("us_fetch_pass") or float("nan")
        print(f"{u[:34]:34s} {kern[:44]:44s} {us:7.2f} {e.get('read_bytes', float('nan'))/1e6:8.2f} "
              f"{e.get('write_bytes', float('nan'))/1e6:8.2f} {e.get('bytes', float('nan'))/us/1e3:6.0f} "
              f"{(e.get('mfma_busy_pct_lb') or float('nan')):7.1f} {(e.get('wait_pct') or float('nan')):6.1f}")
    meta["tool"] = "tools/pmc_box.sh + tools/pmc_summary.py"
    meta["fetch_correction"] = "FETCH_SIZE x2 for 16-B/lane f32 kernels, x1 for the u8-input first layer"
    json.dump({"_meta": meta, "units": units}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
