#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: name, VGPRs, scratch, waves/SIMD.

usage: python tools/resource_usage.py [filter-regex]   (compiles tensor_regression_amd/csrc/tr_kernels.hip)
"""
import re
import subprocess
import sys
import os

here = os.path.dirname(os.path.abspath(__file__))
src = os.path.join(here, "..", "tensor_regression_amd", "csrc", "tr_kernels.hip")
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src,
                      "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
flt = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        cur = {"name": body.split(":", 1)[1].strip()}
        rows.append(cur)
    else:
        k, _, v = body.partition(":")
        cur[k.strip()] = v.strip()
for r in rows:
    if flt and not flt.search(r["name"]):
        continue
    print(f'{r["name"][:70]:70s} vgpr={r.get("VGPRs","?"):>4s} agpr={r.get("AGPRs","?"):>3s} '
          f'scratch={r.get("ScratchSize [bytes/lane]","?"):>5s} waves/simd={r.get("Occupancy [waves/SIMD]","?")}')
