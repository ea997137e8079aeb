#!/usr/bin/env python3
"""Per-kernel resource summary of one HIP source (gfx950):  python3 tools/kres.py <file.hip> [filter]
Prints demangled-ish kernel name, VGPRs, AGPRs, VGPR spills, SGPR spills, LDS bytes, occupancy."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", "include", "-c", src,
       "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
r = subprocess.run(cmd, capture_output=True, text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    if "error" in line:
        print(line)
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for c in rows:
    n = c["name"]
    m = re.search(r"(k_\w+?)I(.*?)EE", n)
    short = (m.group(1) + "<" + ",".join(re.findall(r"Li(\d+)E|Lb(\d)E", m.group(2)).__repr__() and
             [a or b for a, b in re.findall(r"Li(\d+)E|Lb(\d)E", m.group(2))]) + ">") if m else n
    if flt and flt not in short:
        continue
    print(f"{short:28s} vgpr {c.get('VGPRs','?'):>4} agpr {c.get('AGPRs','?'):>3} vspill {c.get('VGPRs Spill','?'):>4} "
          f"sspill {c.get('SGPRs Spill','?'):>3} lds {c.get('LDS Size [bytes/block]','?'):>7} occ {c.get('Occupancy [waves/SIMD]','?')}")
sys.exit(r.returncode)
