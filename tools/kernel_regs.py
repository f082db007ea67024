#!/usr/bin/env python3
"""Register / LDS / code-size report of the gfx950 kernels in a hipcc object.

    python tools/kernel_regs.py obj.o [substring ...]

Extracts the device code object from the object's .hip_fatbin section
(llvm-objcopy + clang-offload-bundler) and prints, per kernel whose name
holds every substring: arch VGPRs, AGPRs, SGPR spills, scratch, LDS, code
bytes.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj, tmp):
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                    os.path.join(tmp, "junk.o")], check=True)
    co = os.path.join(tmp, "dev.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def main():
    obj, subs = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(obj, tmp)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
        syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", co], check=True,
                              capture_output=True, text=True).stdout
    size = {}
    for ln in syms.splitlines():
        f = ln.split()
        if len(f) >= 8 and f[3] == "FUNC":
            size[f[7]] = int(f[2])
    for blk in notes.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        if not all(s in name for s in subs):
            continue
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
        agpr = blk.split("\n")[0].strip()
        print(f"{name[:100]:100s} vgpr {g('vgpr_count'):>4} agpr {agpr:>4} "
              f"sspill {g('sgpr_spill_count'):>4} scratch {g('private_segment_fixed_size'):>4} "
              f"lds {g('group_segment_fixed_size'):>6} code {size.get(name, '?')}")


if __name__ == "__main__":
    main()
