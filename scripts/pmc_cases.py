#!/usr/bin/env python3
"""Per-case averages of a rocprofv3 --pmc run of `kbench.py --mark`: the torch
fill kernel kbench launches before each case's runs splits the dispatch
sequence; every other dispatch whose name starts with --kernel is averaged
(counters and duration) into the current case.

    python scripts/pmc_cases.py <dir with *counter_collection.csv> --cases a,b,c [--kernel vvh::k_stft_pair]
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--cases", required=True)
ap.add_argument("--kernel", default="vvh::k_stft_pair")
a = ap.parse_args()
names = a.cases.split(",")
disp = collections.OrderedDict()
for f in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            d = disp.setdefault(int(row["Dispatch_Id"]), {"name": row["Kernel_Name"], "c": collections.Counter(),
                                                          "us": (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3})
            d["c"][row["Counter_Name"]] += float(row["Counter_Value"])
case = -1
acc = collections.defaultdict(lambda: {"n": 0, "us": 0.0, "c": collections.Counter()})
for i in sorted(disp):
    d = disp[i]
    if "fill" in d["name"].lower() or "FillFunctor" in d["name"]:
        case += 1
        continue
    if case < 0 or not d["name"].removeprefix("void ").startswith(a.kernel):
        continue
    k = names[case % len(names)]
    acc[k]["n"] += 1
    acc[k]["us"] += d["us"]
    acc[k]["c"].update(d["c"])
for k in names:
    if k not in acc:
        continue
    r = acc[k]
    print(json.dumps({"case": k, "dispatches": r["n"], "avg_us": round(r["us"] / r["n"], 1),
                      **{c: round(v / r["n"], 1) for c, v in sorted(r["c"].items())}}))
