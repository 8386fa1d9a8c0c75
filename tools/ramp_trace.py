#!/usr/bin/env python3
"""Step-by-step view of the timed region of `bench.py --trace-only` from a rocprofv3
--kernel-trace CSV: the trace ends with the timed steps (bench exits right after them), so the
last K x per_step dispatches are the K timed steps and the W x per_step before them the
warm-up.  Per step: span (first start -> last end), the sum of kernel durations and the
duration of one named kernel, to show whether the first steps of a short run are slower
(clock ramp, lane start-up) than the later ones.

    python3 tools/ramp_trace.py <kernel_trace.csv> <dispatches per step> <steps> <warmup> [kernel substring]
"""
import csv
import sys


def main(path, per_step, steps, warmup, name="enc01"):
    rows = [r for r in csv.DictReader(open(path)) if "tic::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = per_step * (steps + warmup)
    tail = rows[-n:]
    t_first = int(tail[warmup * per_step]["Start_Timestamp"])
    t_last = max(int(r["End_Timestamp"]) for r in tail)
    print(f"timed region kernel span {(t_last - t_first) / 1e3:.1f} us = {(t_last - t_first) / 1e3 / steps:.2f} us/step")
    for s in range(steps + warmup):
        st = tail[s * per_step:(s + 1) * per_step]
        a = min(int(r["Start_Timestamp"]) for r in st)
        b = max(int(r["End_Timestamp"]) for r in st)
        tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
        k = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st if name in r["Kernel_Name"]]
        tag = "warm" if s < warmup else "timed"
        print(f"{tag} {s:3d} start {(a - t_first) / 1e3:9.1f} span {(b - a) / 1e3:7.1f} sum {tot / 1e3:7.1f} "
              f"{name} {' '.join(f'{x / 1e3:.1f}' for x in k)}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), *(sys.argv[5:6]))
