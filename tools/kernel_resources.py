#!/usr/bin/env python3
"""Per-kernel VGPR count and scratch (spill) size of the built gfx950 code
objects in adlsm-tree_amd/lib/libadlbloom.so (the register
attributes' effect, checked from the code object's metadata notes rather than
assumed).

Usage: python tools/kernel_resources.py [path/to/libadlbloom.so]
Prints one line per kernel: scratch bytes per lane, VGPRs, spilled VGPRs,
name.  Needs /opt/rocm/lib/llvm/bin (llvm-objdump, llvm-readelf); the library
is copied to a temporary directory first because llvm-objdump --offloading
writes the extracted bundles next to its input.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "adlsm-tree_amd", "lib", "libadlbloom.so")


def kernel_resources(lib=DEFAULT_LIB):
    """{kernel symbol: {"scratch": B/lane, "vgpr": n, "vgpr_spill": n, "sgpr_spill": n}}"""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "lib.so")
        shutil.copyfile(lib, so)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=td, check=True,
                       stdout=subprocess.DEVNULL)
        for f in sorted(os.listdir(td)):
            if "amdgcn" not in f or "gfx950" not in f:
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(td, f)],
                                   check=True, capture_output=True, text=True).stdout
            cur = None
            # one kernel's keys are indented alike and sorted; '.name' comes
            # after '.max_flat_workgroup_size' and before the counts
            blocks = re.split(r"\n\s+- \.", notes)
            for blk in blocks:
                fields = dict(re.findall(r"^\s*\.?([a-z_]+):\s+(\S+)\s*$", "." + blk, re.M))
                if "symbol" not in fields or "vgpr_count" not in fields:
                    continue
                cur = fields.get("name", fields["symbol"])
                out[cur] = {
                    "scratch": int(fields.get("private_segment_fixed_size", 0)),
                    "vgpr": int(fields["vgpr_count"]),
                    "vgpr_spill": int(fields.get("vgpr_spill_count", 0)),
                    "sgpr_spill": int(fields.get("sgpr_spill_count", 0)),
                }
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    res = kernel_resources(lib)
    print(f"{'scratch':>7} {'vgpr':>4} {'vspill':>6}  kernel")
    for name, r in sorted(res.items(), key=lambda kv: (-kv[1]["scratch"], kv[0])):
        print(f"{r['scratch']:>7} {r['vgpr']:>4} {r['vgpr_spill']:>6}  {name}")


if __name__ == "__main__":
    main()
