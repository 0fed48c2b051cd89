"""VGPR / spill counts per kernel of a built object (.o with a HIP fatbin, or
a .co): python scripts/kernel_regs.py glfs_amd/csrc/post_kernels.o [filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
with tempfile.TemporaryDirectory() as d:
    co = src
    if not src.endswith(".co"):
        fb = os.path.join(d, "fb.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", src,
                               os.path.join(d, "junk.o")])
        co = os.path.join(d, "k.co")
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                               f"--output={co}"])
    notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
kern = []
cur = {}
for ln in notes.splitlines():
    m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", ln)
    if not m:
        continue
    k, v = m.groups()
    if k == "agpr_count" and cur:
        kern.append(cur)
        cur = {}
    cur[k] = v
if cur:
    kern.append(cur)
for k in kern:
    name = k.get("name", "?")
    if flt in name:
        dm = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        print(f"{k.get('vgpr_count', '?'):>4} vgpr {k.get('vgpr_spill_count', '?'):>4} spill "
              f"{k.get('sgpr_count', '?'):>4} sgpr  {dm[:110]}")
