"""Kernel resources from hipcc -Rpass-analysis=kernel-resource-usage output on
stdin: one line per kernel (VGPRs, SGPRs, scratch, occupancy, LDS), names
filtered by argv[1] (substring) if given."""
import re
import subprocess
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    if flt in n:
        print(f"v{r.get('VGPRs', '?'):>4} s{r.get('TotalSGPRs', '?'):>4} scr{r.get('ScratchSize', '?'):>4} "
              f"occ{r.get('Occupancy', '?'):>2} lds{r.get('LDS', '?'):>6}  {n[:150]}")
