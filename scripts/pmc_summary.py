"""Summarise a gpu_prof.sh output directory: per kernel, the average kernel
duration (kernel trace) and every PMC counter averaged per dispatch.

    python3 scripts/pmc_summary.py gpurun_out/prof [--json out.json --channels 32 --box desc]
"""
import argparse
import json
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name.replace("void ", "")[:60]


def collect(d):
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
    res = {}
    for k in sorted(set(dur) | set(ctr)):
        if k.startswith("at::") or "rocclr" in k or "distribution" in k or not k:
            continue
        ds = dur.get(k, [])
        ent = {"calls": len(ds), "avg_us": round(sum(ds) / len(ds) / 1e3, 3) if ds else None}
        for cn, vs in sorted(ctr[k].items()):
            ent[cn] = sum(vs) / len(vs)
        res[k] = ent
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--channels", type=int)
    ap.add_argument("--box", default="")
    a = ap.parse_args()
    res = collect(a.dir)
    for k, ent in res.items():
        print(f"== {k}  calls={ent['calls']} avg_us={ent['avg_us']}")
        for cn, v in ent.items():
            if cn not in ("calls", "avg_us"):
                print(f"   {cn:40s} {v:.6g}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"channels_per_gpu": a.channels, "box": a.box, "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
