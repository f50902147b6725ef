"""Print the device timeline (kernels + memory copies, with the idle gaps between them)
of a window of a rocprofv3 --kernel-trace --memory-copy-trace CSV run.

    python tools/timeline.py gpurun_out/<prof_dir> [--around warp_affine --index 10 --count 2]
"""
import csv
import glob
import os
import re
import sys


def main():
    a = sys.argv[1:]
    d = a[0]
    key = a[a.index("--around") + 1] if "--around" in a else "warp_affine"
    idx = int(a[a.index("--index") + 1]) if "--index" in a else 10
    cnt = int(a[a.index("--count") + 1]) if "--count" in a else 2
    ev = []

    def nm(s):
        s = s.replace("void ", "").replace("kcmc::", "").replace("(anonymous namespace)::", "")
        return re.split(r"[<(]", s)[0][:30]

    for p in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm(r["Kernel_Name"])))
    for p in glob.glob(os.path.join(d, "*memory_copy_trace.csv")):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r["Direction"].split("_")[-3:][0]
                       + "->" + r["Direction"].split("_")[-1]))
    ev.sort()
    t0 = ev[0][0]
    marks = [e for e in ev if e[2].startswith(key)]
    lo, hi = marks[idx][0], marks[min(idx + cnt, len(marks) - 1)][0]
    busy_end = None
    for s, e, n in ev:
        if lo <= s <= hi:
            gap = (s - busy_end) / 1e3 if busy_end is not None and s > busy_end else 0.0
            print(f"{n:32s} start {(s - t0) / 1e6:10.3f} ms  dur {(e - s) / 1e3:9.1f} us  idle before {gap:7.1f} us")
            busy_end = e if busy_end is None else max(busy_end, e)
    print(f"period ({key} start to start): {(marks[idx + 1][0] - marks[idx][0]) / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
