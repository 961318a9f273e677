"""VGPRs / scratch / spills of every k_mnl_bsp instantiation from a -Rpass-analysis=kernel-resource-usage
log (tools/duo_res.py LOG): the split body must stay spill-free (duo_kernel_ok rejects spilling ones)."""
import re
import subprocess
import sys

rows, cur = [], None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"f": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
for r in rows:
    if "bsp" not in r["f"]:
        continue
    d = subprocess.run(["c++filt", r["f"]], capture_output=True, text=True).stdout.strip()
    d = re.sub(r"^void tr::k_mnl_bsp", "", d.split("(")[0])
    print(f"{d:40s} vgpr {r.get('VGPRs')} scratch {r.get('ScratchSize')} vspill {r.get('VGPRs Spill')} sspill {r.get('SGPRs Spill')}")
