"""Per-kernel VGPRs / scratch / occupancy of a HIP source (hipcc -Rpass-analysis), one line
per kernel: python tools/resource_usage.py cc-mpc_amd/csrc/moments.hip [filter]."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC",
       "-Iinclude", "-I../../include", "-ffp-contract=off", "-munsafe-fp-atomics", "-c", src,
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    n = re.sub(r"\(.*", "", r["name"]).replace("void ccmpc::", "")
    if flt in n:
        print(f"{n:45s} vgpr {r.get('vgpr', -1):4d} scratch {r.get('scratch', -1):4d} "
              f"occ {r.get('occ', -1)} lds {r.get('lds', -1)}")
if not rows:
    print(out[-3000:])
