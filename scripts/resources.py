"""Per-kernel register / LDS usage of one HIP source for gfx950 (the compiler's
kernel-resource-usage remarks), one line per kernel:
    python scripts/resources.py basecount_amd/csrc/bc_rc.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-fno-fast-math", "-Iinclude", "-c", "-o", "/tmp/_res.o", src, "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s*(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>3} vspill {r.get('SGPRs Spill', '?'):>3} sspill "
          f"{r.get('LDS Size [bytes/block]', '?'):>6} lds occ {r.get('Occupancy [waves/SIMD]', '?')}  {r['name'][:150]}")
