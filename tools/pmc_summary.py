"""Aggregate rocprofv3 --pmc CSV passes (tools/pmc_warp.sh output) per kernel dispatch.

    python tools/pmc_summary.py gpurun_out/pmc [--by-kernel] [--json out.json] [--sha <commit>]
With --by-kernel (tools/pmc_kernels.sh output) the means are per kernel name, with the
derived utilisations (SQ_* cycle counters are quad-cycles; GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so the dispatch's cycles are GRBM_GUI_ACTIVE / 8; 256 CUs x 4 SIMDs).
Without it, prints per-counter mean over the profiled dispatches (skipping the first, which is the
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
            key = (os.path.basename(os.path.dirname(p)), int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            per[key]["_dispatch_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = collections.defaultdict(list)
    for (pas, disp), ctrs in sorted(per.items()):
        for c, v in ctrs.items():
            out[c].append(v)
    return {c: v[1:] if len(v) > 1 else v for c, v in out.items()}


def load_by_kernel(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for p in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(p))
        for r in csv.DictReader(open(p)):
            key = (pas, int(r["Dispatch_Id"]))
            names[key] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            per[key]["_dispatch_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, ctrs in sorted(per.items()):
        for c, v in ctrs.items():
            out[names[key]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


CUS, SIMDS = 256, 4


def derived(m):
    res = {}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc and m.get("_dispatch_ns"):
        res["clock_ghz"] = cyc / m["_dispatch_ns"]
    if cyc:
        res["dispatch_cycles"] = cyc
        if "SQ_ACTIVE_INST_VALU" in m:
            res["valu_busy_frac"] = 4 * m["SQ_ACTIVE_INST_VALU"] / (CUS * SIMDS * cyc)
        if "SQ_INSTS_VALU" in m:
            # one wave64 VALU instruction per SIMD per cycle at best (2 passes of 32 lanes: 0.5)
            res["valu_insts_per_simd_cycle"] = m["SQ_INSTS_VALU"] / (CUS * SIMDS * cyc)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            res["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (CUS * SIMDS * cyc)
    f64 = sum(m.get(c, 0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
    f64 += 2 * m.get("SQ_INSTS_VALU_FMA_F64", 0)
    if f64:
        res["f64_flop_per_dispatch"] = 64 * f64  # wave64 instructions -> lane ops (FMA = 2)
    return res


def main_by_kernel(d, js=None):
    agg = load_by_kernel(d)
    res = {}
    for k in sorted(agg):
        print(k)
        for c in sorted(agg[k]):
            print(f"  {c:30s} {agg[k][c]:.6g}")
        dv = derived(agg[k])
        for c, v in dv.items():
            print(f"  => {c:27s} {v:.4g}")
        res[k] = {"counters_mean_per_dispatch": agg[k], "derived": dv}
    if js:
        json.dump(res, open(js, "w"), indent=1)


def main(d, js=None, sha=None):
    agg = load(d)
    mean = {c: sum(v) / len(v) for c, v in agg.items()}
    disp_ns = mean.pop("_dispatch_ns", None)
    for c in sorted(mean):
        print(f"{c:28s} {mean[c]:.6g}")
    res = {"commit": sha, "counters_mean_per_dispatch": mean,
           "kernel_avg_ms": round(disp_ns / 1e6, 4) if disp_ns else None}
    if disp_ns:
        print(f"kernel avg duration in the PMC passes: {disp_ns / 1e6:.4f} ms (profiled runs clock lower)")
    if sha:
        print(f"commit: {sha}")
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd = 2 * mean["FETCH_SIZE"] * 1024
        wr = mean["WRITE_SIZE"] * 1024
        res.update(read_bytes_corrected=rd, write_bytes=wr, hbm_bytes_per_launch=rd + wr)
        print(f"HBM bytes/launch (FETCH_SIZEx2 + WRITE_SIZE) = {(rd + wr) / 1e9:.3f} GB")
    if js:
        json.dump(res, open(js, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    js = a[a.index("--json") + 1] if "--json" in a else None
    sha = a[a.index("--sha") + 1] if "--sha" in a else None
    if "--by-kernel" in a:
        main_by_kernel(a[0], js)
    else:
        main(a[0], js, sha)
