"""VGPR / occupancy per kernel of one source file (hipcc resource-usage remarks).
    python tools/vgprs.py csrc/pwconv.hip [name-filter] [extra hipcc flags...]"""
import re
import subprocess
import sys

P = "light-3d-unet-front_amd"
src, filt = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-function",
       "-Wno-pass-failed", f"-I{P}/csrc", "-Iinclude", "-c", f"{P}/{src}", "-o", "/tmp/vg.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
name = None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True,
                              text=True).stdout.strip()
        name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "")
    m = re.search(r" VGPRs: (\d+)", line)
    if m and name and filt in name:
        vg = m.group(1)
    m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", line)
    if m and name and filt in name:
        print(f"{vg:>4} occ {m.group(1)}  {name}")
