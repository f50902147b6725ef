"""Aggregate rocprofv3 --pmc CSV passes (tools/pmc_warp.sh output) per kernel dispatch.

    python tools/pmc_summary.py gpurun_out/pmc [--json out.json]
Prints per-counter mean over the profiled dispatches (skipping the first, which is the
bench's input synthesis) and the derived HBM traffic per launch: FETCH_SIZE (KB, x2 for
gfx950's half-counted wide reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE (KB).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            per[(os.path.basename(os.path.dirname(p)), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(
                r["Counter_Value"])
    out = collections.defaultdict(list)
    for (pas, disp), ctrs in sorted(per.items()):
        for c, v in ctrs.items():
            out[c].append(v)
    return {c: v[1:] if len(v) > 1 else v for c, v in out.items()}


def main(d, js=None):
    agg = load(d)
    mean = {c: sum(v) / len(v) for c, v in agg.items()}
    for c in sorted(mean):
        print(f"{c:28s} {mean[c]:.6g}")
    res = {"counters_mean_per_dispatch": mean}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd = 2 * mean["FETCH_SIZE"] * 1024
        wr = mean["WRITE_SIZE"] * 1024
        res.update(read_bytes_corrected=rd, write_bytes=wr, hbm_bytes_per_launch=rd + wr)
        print(f"HBM bytes/launch (FETCH_SIZEx2 + WRITE_SIZE) = {(rd + wr) / 1e9:.3f} GB")
    if js:
        json.dump(res, open(js, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--json" else None)
