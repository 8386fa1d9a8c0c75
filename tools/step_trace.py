#!/usr/bin/env python3
"""Timeline of steady-state bench steps from a rocprofv3 --kernel-trace CSV: per dispatch
start/end relative to the step, per-queue gaps, and how much of the step has 0 / 1 / 2
kernels running.   python3 tools/step_trace.py <kernel_trace.csv> <launches per step>"""
import csv
import sys


def main(path, per_step, steps=5):
    rows = [r for r in csv.DictReader(open(path)) if "tic::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[-per_step * steps:]
    t0 = int(tail[0]["Start_Timestamp"])
    ev = []
    for r in tail:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        ev.append((s, e, r.get("Queue_Id", "?"), r["Kernel_Name"].split("(")[0].replace("void tic::", "")[:60]))
    for s, e, q, k in ev[:per_step + 4]:
        print(f"{s / 1e3:9.2f} {e / 1e3:9.2f} {(e - s) / 1e3:7.2f}  q{q}  {k}")
    end = max(e for _, e, _, _ in ev)
    pts = sorted({p for s, e, _, _ in ev for p in (s, e)})
    busy = {0: 0, 1: 0, 2: 0, 3: 0}
    for a, b in zip(pts, pts[1:]):
        n = sum(1 for s, e, _, _ in ev if s <= a and e >= b)
        busy[min(n, 3)] += b - a
    print(f"span {end / 1e3:.1f} us for {steps} steps = {end / 1e3 / steps:.1f} us/step")
    for k, v in busy.items():
        print(f"  {k} kernels running: {v / end * 100:5.1f} %")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 5)
