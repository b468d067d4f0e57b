#!/usr/bin/env python3
"""A/B two builds of the library on the GPU box: alternate kbench.py runs
(A, B, A, B, ...) in separate processes (the library is loaded once per
process) and report the median over all runs per case and build.

    python scripts/abbench.py --a scripts/ab/prev.so --b vv-dsp_amd/lib/libvvdsp_amd.so \
        --cases stft,fir,c2c1024 --pairs 3
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(lib, cases, reps, rounds):
    env = dict(os.environ, VVDSP_AMD_LIB=os.path.abspath(lib))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "kbench.py"), "--cases", cases,
                          "--reps", str(reps), "--rounds", str(rounds)], env=env, capture_output=True, text=True,
                         timeout=600)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    return [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    res = {"A": {}, "B": {}}
    for i in range(a.pairs):
        for tag, lib in (("A", a.a), ("B", a.b)) if i % 2 == 0 else (("B", a.b), ("A", a.a)):
            for r in run(lib, a.cases, a.reps, a.rounds):
                res[tag].setdefault(r["case"], []).append(r["ms_median"])
    for case in res["A"]:
        ma, mb = float(np.median(res["A"][case])), float(np.median(res["B"][case]))
        print(json.dumps({"case": case, "A_ms": round(ma, 4), "B_ms": round(mb, 4), "B_over_A": round(mb / ma, 4),
                          "A_runs": res["A"][case], "B_runs": res["B"][case]}))


if __name__ == "__main__":
    main()
