#!/usr/bin/env python3
"""tools/isa_stats.py -- instruction mix of the gfx950 kernels in a .hip file.

usage: python tools/isa_stats.py adlsm-tree_amd/csrc/bloom_build.hip [substring]
"""
import re
import subprocess
import sys
from collections import Counter

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                "-S", "-o", "/tmp/isa.s", src], check=True)
s = open("/tmp/isa.s").read()
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    end = s.index(".Lfunc_end", m.end())
    body = s[m.end():end]
    ins = [l.strip().split()[0] for l in body.split("\n")
           if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name[:90]}\n  total {len(ins)}  valu {valu}  mul_lo {c['v_mul_lo_u32']}  mul_hi {c['v_mul_hi_u32']}"
          f"  ds {sum(v for k, v in c.items() if k.startswith('ds_'))}  global {sum(v for k, v in c.items() if k.startswith('global_'))}")
    print("  ", c.most_common(30))
