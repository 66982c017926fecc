#!/usr/bin/env python3
"""tools/regs.py [extra hipcc flags] — one line per megakernel variant: VGPRs, SGPRs,
scratch bytes per lane, waves/SIMD (from -Rpass-analysis=kernel-resource-usage)."""
import re
import subprocess
import sys

PKG = "peter-shirley-ray-tracing-the-next-week_amd"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Iinclude", f"-I{PKG}/csrc",
       f"-I{PKG}/csrc/host", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-c", f"{PKG}/csrc/hip/rt_kernel.hip",
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s*(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    m = re.search(r"rt_megakernelILb(\d)ELb(\d)ELi(\d+)ELi(\d+)ELi(\d)E", name)
    tag = f"mega count={m.group(1)} prof={m.group(2)} width={m.group(3)} feat={m.group(4)} mode={m.group(5)}" if m else name[:40]
    print(f"{tag:44s} VGPR {r.get('VGPRs')} AGPR {r.get('AGPRs')} SGPR {r.get('TotalSGPRs')} "
          f"scratch {r.get('ScratchSize [bytes/lane]')} waves {r.get('Occupancy [waves/SIMD]')} "
          f"LDS {r.get('LDS Size [bytes/block]')}")
if not rows:
    print(err[-3000:])
