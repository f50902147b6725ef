"""Summarise a rocprofv3 kernel trace (SQLite .db, or kernel_stats.csv) as markdown.

    python tools/prof_summary.py gpurun_out/prof/run_results.db > profiles/<name>.md
"""
import csv
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)  # drop the argument list
    return name[:110]


def rows_from_db(path):
    c = sqlite3.connect(path)
    # the top_kernels view reports microseconds; normalise to nanoseconds like the CSV
    return [(r[0], int(r[1]), 1e3 * float(r[2]), 1e3 * float(r[3]), float(r[4]))
            for r in c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["Percentage"])))
    return out


def main(path):
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    print(f"# rocprofv3 kernel summary: `{os.path.basename(path)}`\n")
    print("| kernel | calls | total (ms) | avg (us) | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, total, avg, pct in rows:
        print(f"| `{short(name)}` | {calls} | {total / 1e6:.3f} | {avg / 1e3:.1f} | {pct:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
