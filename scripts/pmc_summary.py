"""Summarise a gpu_prof.sh output directory: per kernel, the average kernel
duration (kernel trace) and every PMC counter averaged per dispatch.

    python3 scripts/pmc_summary.py gpurun_out/prof [--json out.json --channels 256 --box desc]
                                   [--tail vvh::k_stft_pair=20 --tail vvh::k_c2c=50 ...]

--tail PREFIX=N: for kernels whose short name starts with PREFIX, also report
the average over the LAST N dispatches in trace order (avg_us_timed): bench.py's
timed launches, with the warm-up dispatches (clock ramp) excluded.
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


def collect(d, tails=()):
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
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
        for pre, n in tails:
            if k.startswith(pre) and len(ds) >= n:
                last = ds[-n:]
                ent["timed_calls"] = n
                ent["avg_us_timed"] = round(sum(last) / n / 1e3, 3)
                ent["min_us_timed"] = round(min(last) / 1e3, 3)
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
    ap.add_argument("--tail", action="append", default=[], help="PREFIX=N: average of the last N dispatches")
    a = ap.parse_args()
    tails = [(t.rsplit("=", 1)[0], int(t.rsplit("=", 1)[1])) for t in a.tail]
    res = collect(a.dir, tails)
    for k, ent in res.items():
        print(f"== {k}  calls={ent['calls']} avg_us={ent['avg_us']}"
              + (f" avg_us_timed={ent['avg_us_timed']} (last {ent['timed_calls']})" if "avg_us_timed" in ent else ""))
        for cn, v in ent.items():
            if cn not in ("calls", "avg_us", "timed_calls", "avg_us_timed", "min_us_timed"):
                print(f"   {cn:40s} {v:.6g}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"channels_per_gpu": a.channels, "box": a.box, "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
