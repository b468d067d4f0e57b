#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy / LDS table from hipcc's resource remarks."""
import glob, re, subprocess, sys
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
pat = sys.argv[1] if len(sys.argv) > 1 else "."
for f in sorted(glob.glob(f"{ROOT}/vv-dsp_amd/csrc/hip/*.hip")):
    out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                          f"-I{ROOT}/include", "-c", f, "-o", "/dev/null",
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
    cur = {}
    for ln in out.splitlines():
        m = re.search(r"remark: (\s*)([^:]+): (.*?) \[-Rpass", ln)
        if not m:
            continue
        k, v = m.group(2).strip(), m.group(3).strip()
        if k == "Function Name":
            if cur and re.search(pat, cur["name"]):
                print(f"{cur['name'][:70]:70s} vgpr={cur.get('VGPRs','?'):>4} scr={cur.get('ScratchSize [bytes/lane]','?'):>4} "
                      f"occ={cur.get('Occupancy [waves/SIMD]','?')} lds={cur.get('LDS Size [bytes/block]','?')}")
            cur = {"name": v}
        else:
            cur[k] = v
    if cur and re.search(pat, cur["name"]):
        print(f"{cur['name'][:70]:70s} vgpr={cur.get('VGPRs','?'):>4} scr={cur.get('ScratchSize [bytes/lane]','?'):>4} "
              f"occ={cur.get('Occupancy [waves/SIMD]','?')} lds={cur.get('LDS Size [bytes/block]','?')}")
