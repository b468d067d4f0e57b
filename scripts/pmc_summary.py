"""Summarise a gpu_prof.sh output directory: per kernel, the average kernel
duration (kernel trace) and every PMC counter averaged per dispatch.

    python3 scripts/pmc_summary.py gpurun_out/prof
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.split("(")[0]
    return name.replace("void ", "")[:60]


def main(d):
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (disp, cn), v in per.items():
            ctr[names[disp]][cn].append(v)
    for k in sorted(set(dur) | set(ctr)):
        if k.startswith("at::") or "rocclr" in k or "distribution" in k:
            continue
        ds = dur.get(k, [])
        avg = sum(ds) / len(ds) / 1e3 if ds else float("nan")
        print(f"== {k}  calls={len(ds)} avg_us={avg:.2f}")
        for cn, vs in sorted(ctr[k].items()):
            print(f"   {cn:40s} {sum(vs) / len(vs):.6g}")


if __name__ == "__main__":
    main(sys.argv[1])
