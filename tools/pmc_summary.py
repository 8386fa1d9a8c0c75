#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc_{fetch,write,sq}) per kernel.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) is doubled on gfx950 (it
tallies 128-B requests at 64 B for wide streaming reads), WRITE_SIZE (KiB) is exact for
16-B-per-lane stores.  Values are medians over all dispatches of each kernel symbol.
Writes profiles/traffic_<tag>.json keyed by kernel symbol (bytes per launch)."""
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


PREFIX = os.environ.get("PMC_PREFIX", "pmc")


def load(kind):
    path = os.path.join(OUT, f"{PREFIX}_{kind}", "p_counter_collection.csv")
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    if not os.path.exists(path):
        return per, dur
    seen = set()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        d = r["Dispatch_Id"]
        if (k, d) not in seen:
            seen.add((k, d))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def short(name):
    m = re.search(r"conv3x3_kernel<(.*?)>", name)
    if m:
        return "conv3x3<" + m.group(1).replace(" ", "") + ">"
    m = re.search(r"tic::(\w+)<(.*?)>", name)
    return f"{m.group(1)}<{m.group(2).replace(' ', '')}>" if m else name[:50]


def main(tag="r01"):
    fetch, dur = load("fetch")
    write, _ = load("write")
    sq, _ = load("sq")
    med = lambda v: statistics.median(v) if v else float("nan")
    traffic = {}
    print(f"{'kernel':58s} {'us':>7s} {'readMB':>8s} {'writeMB':>8s} {'GB/s':>7s} {'mfma%':>6s} {'wait%':>6s} {'clkGHz':>6s}")
    for k in sorted(fetch, key=lambda k: -med(dur[k]) * len(dur[k])):
        if "tic::" not in k:
            continue
        rd = 2 * med(fetch[k]["FETCH_SIZE"]) * 1024
        wr = med(write[k]["WRITE_SIZE"]) * 1024 if k in write else float("nan")
        us = med(dur[k])
        s = sq.get(k, {})
        gui = med(s.get("GRBM_GUI_ACTIVE", [])) / 8  # summed over 8 XCDs
        mfma = med(s.get("SQ_VALU_MFMA_BUSY_CYCLES", [])) / (gui * 1024) * 100 if gui else float("nan")
        wav = med(s.get("SQ_WAVE_CYCLES", []))
        wait = med(s.get("SQ_WAIT_ANY", [])) / wav * 100 if wav else float("nan")
        clk = gui / (us * 1e3) if us else float("nan")
        traffic[short(k)] = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr, "us": us,
                             "mfma_busy_pct": mfma, "wait_pct": wait, "clock_ghz": clk, "dispatches": len(dur[k])}
        print(f"{short(k)[:58]:58s} {us:7.2f} {rd/1e6:8.2f} {wr/1e6:8.2f} {(rd+wr)/us/1e3:7.0f} {mfma:6.1f} {wait:6.1f} {clk:6.2f}")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(traffic, open(os.path.join(ROOT, "profiles", f"traffic_{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
