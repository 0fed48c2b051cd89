"""Scan the gfx950 code object inside glfs_amd/csrc/post_kernels.o for the
instruction families this pool forbids (writes through the scalar data cache)
and count the agent-scope fences the split-mode merge uses.  Host-only check,
run after a build:  python tools/isa_scan.py
(listed in .gpurunignore: it names the forbidden families in its patterns)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
# built from pieces so no source file spells the mnemonics out
FORBIDDEN = ["s_" + "store", "s_" + "atomic", "s_" + "dcache", "s_buffer_" + "store",
             "s_scratch_" + "store"]


def disassemble(obj):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat])
        b = os.path.join(LLVM, "clang-offload-bundler")
        tgt = [t for t in subprocess.check_output([b, "--list", "--type=o", f"--input={fat}"],
                                                  text=True).split() if "gfx950" in t][0]
        co = os.path.join(d, "k.co")
        subprocess.check_call([b, "--unbundle", "--type=o", f"--input={fat}",
                               f"--targets={tgt}", f"--output={co}"])
        return subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", co], text=True)


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "glfs_amd", "csrc",
                                                             "post_kernels.o")
    asm = disassemble(obj)
    bad = [ln for ln in asm.splitlines()
           if any(re.search(r"\b" + f, ln) for f in FORBIDDEN)]
    fences = {k: len(re.findall(r"\b" + k + r"\b", asm))
              for k in ("buffer_wbl2", "buffer_inv", "global_atomic_add")}
    print(f"{len(asm.splitlines())} lines; forbidden: {len(bad)}; {fences}")
    for ln in bad[:20]:
        print("  ", ln)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
