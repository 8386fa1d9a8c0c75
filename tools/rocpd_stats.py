"""Kernel statistics (rocprofv3 --stats equivalent) from a rocprofv3 rocpd database:
name, calls, total / average duration (us), share of kernel time — as CSV.

    python tools/rocpd_stats.py gpurun_out/prof/p_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, total, avg, pct in con.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, f"{total:.3f}", f"{avg:.3f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main(sys.argv[1])
