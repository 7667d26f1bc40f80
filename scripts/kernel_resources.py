#!/usr/bin/env python
"""Per-kernel register / spill / LDS usage of a gfx950 object built by csrc/Makefile.

usage: python scripts/kernel_resources.py build/csrc/srnn_bignet.o [name-filter]
(extracts the .hip_fatbin section, unbundles the gfx950 code object, reads its AMDGPU
metadata notes; demangled names)"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    rows, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+-?\s*\.(\w+):\s+(.*)$", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "args":
            continue
        if k in ("agpr_count", "name", "private_segment_fixed_size", "vgpr_count", "vgpr_spill_count",
                 "group_segment_fixed_size", "sgpr_spill_count"):
            cur[k] = v
        if k == "wavefront_size" and "name" in cur:
            rows.append(cur)
            cur = {}
    names = subprocess.run(["c++filt"], input="\n".join(r.get("name", "") for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    print(f"{'vgpr':>5} {'agpr':>5} {'spill':>6} {'priv':>6} {'lds':>6}  kernel")
    for r, n in sorted(zip(rows, names), key=lambda x: x[1]):
        if filt in n:
            print(f"{r.get('vgpr_count', '?'):>5} {r.get('agpr_count', '?'):>5} {r.get('vgpr_spill_count', '?'):>6} "
                  f"{r.get('private_segment_fixed_size', '?'):>6} {r.get('group_segment_fixed_size', '?'):>6}  {n[:150]}")


if __name__ == "__main__":
    main()
