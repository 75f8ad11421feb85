"""Device-only compile of csrc/smf.hip (same flags as the extension build) and a resource
report (VGPRs, spills, private segment, LDS) for kernels whose name matches a pattern.
Usage: python tools/devres.py PATTERN [-DFLAG=V ...]"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multigrad_amd.ops import build as B

pat, extra = sys.argv[1], sys.argv[2:]
src = os.path.join(B.CSRC, "smf.hip")
cmd = B._compile_cmd(src)
i = cmd.index("-o")
cmd[i + 1] = "/tmp/devres.co"
cmd = [c for c in cmd if c != "-c"] + ["--cuda-device-only"] + extra
subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o",
                "--input=/tmp/devres.co", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                "--output=/tmp/devres.elf"], check=True)
notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", "/tmp/devres.elf"],
                       capture_output=True, text=True, check=True).stdout
for blk in notes.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not re.search(pat, name):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, None])[1]
    print(name[:90], "vgpr", g("vgpr_count"), "spill", g("vgpr_spill_count"),
          "priv", g("private_segment_fixed_size"), "lds", g("group_segment_fixed_size"))
