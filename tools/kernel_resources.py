#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage of a hipcc object (gfx950 code object notes).
Usage: python tools/kernel_resources.py <file.o> [name-substring]"""
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(obj):
    fat = "/tmp/_kr.fatbin"
    co = "/tmp/_kr.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                          text=True, check=True).stdout


def main():
    txt = notes(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    demangle = lambda n: subprocess.run(["c++filt", n], capture_output=True,
                                        text=True).stdout.strip()
    for blk in txt.split("  - .agpr_count:")[1:]:
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
        name = demangle(get("name"))
        if pat in name:
            print(f"vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>3} sgpr {get('sgpr_count'):>3} "
                  f"spill v{get('vgpr_spill_count')}/s{get('sgpr_spill_count')} "
                  f"scratch {get('private_segment_fixed_size'):>5} lds {get('group_segment_fixed_size'):>6}  {name[:110]}")


if __name__ == "__main__":
    main()
