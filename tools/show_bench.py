#!/usr/bin/env python3
"""Print the bench JSON line summary and the per-layer table from gpurun_out/."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
log = os.path.join(ROOT, "gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "bench.log")
lines = [l for l in open(log).read().splitlines() if l.startswith("{")]
if not lines:
    print(open(log).read()[-3000:])
    sys.exit(1)
d = json.loads(lines[-1])
print(d["value"], d["unit"], "ms/step", d["ms_per_step"], "step-roofline", d.get("roofline_step_frac"))
print("roofline", d["roofline"])
for k in ("parity", "cpu_baseline", "stats_allgather"):
    if k in d:
        print(k, d[k])
lp = os.path.join(ROOT, "gpurun_out", "bench_layers.json")
if os.path.exists(lp):
    L = json.load(open(lp))
    B = L.get("lane_batch", L["config"]["global_batch"] // max(1, d["n_gpus"]))
    tot = 0
    for r in L["layers"]:
        tot += r["ms"]
        print("%-22s %-7s %3d %3d %4d %.4f ms %6.1f TF/s %6.0f GB/s %s" % (
            r["layer"], r["kind"], r["cin"], r["cout"], r["out_hw"], r["ms"],
            r["flops_per_patch"] * B / r["ms"] / 1e9, r["bytes_per_patch"] * B / r["ms"] / 1e6, r.get("tile")))
    print("sum of layer ms", round(tot, 4))
