#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage):
VGPRs, spills, scratch, occupancy, LDS.   python tools/kres.py csrc/qe_sort.hip [name-regex] [-DFLAG ...]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
flags = [a for a in sys.argv[2:] if a.startswith("-D")]
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
                    "-munsafe-fp-atomics", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + flags,
                   capture_output=True, text=True)
cur = None
rows = {}
for ln in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]):\s*(\S+)", ln)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur]["Spill" if k == "VGPRs Spill" else k.split()[0]] = v
for name, d in rows.items():
    if pat and not re.search(pat, name):
        continue
    print(f"vgpr {d.get('VGPRs','?'):>4} spill {d.get('Spill', '0'):>3} scratch {d.get('ScratchSize','?'):>4} "
          f"occ {d.get('Occupancy','?'):>2} lds {d.get('LDS','?'):>6}  {name[:110]}")
if r.returncode:
    print(r.stderr[-3000:])
