#!/usr/bin/env python3
"""Per-launch-unit medians of the investigative SQ counter passes (tools/kcounters.sh),
labelled with the bench's launch plan as tools/pmc_summary.py does.  Cycle counters are
shown per wave (/ SQ_WAVES) where that is meaningful; SQ_*_CYCLES-type counters count
quad-cycles per MI355X_MICROARCH.md (compare them with each other, not with the clock)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import label, load  # noqa: E402


def main(out_dir):
    per = {}
    plan = None
    for p in ("a", "b", "c"):
        csvp = os.path.join(out_dir, f"pmc_{p}", "p_counter_collection.csv")
        pp = os.path.join(out_dir, f"plan_{p}.json")
        if not (os.path.exists(csvp) and os.path.exists(pp)):
            continue
        pd = json.load(open(pp))
        plan = plan or pd["plan"]
        for unit, ds in label(load(csvp), pd["plan"], pd["_meta"]["steps"]).items():
            e = per.setdefault(unit, {"us": []})
            for d in ds:
                e["us"].append(d[1])
                for k, v in d[2].items():
                    e.setdefault(k, []).append(v)
    for item in plan:
        u = item["unit"]
        e = {k: statistics.median(v) for k, v in per.get(u, {}).items() if v}
        print(f"== {u}  {item['kernel']}  {e.get('us', 0):.2f} us")
        waves = e.get("SQ_WAVES") or 1
        for k in sorted(e):
            if k in ("us",):
                continue
            print(f"   {k:28s} {e[k]:14.4g}   /wave {e[k] / waves:12.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
