"""tools/gap_probe.py -- diagnostics: 20 headline builds through the stamps
library (ADL_BLOOM_EXP switches work there), for measuring the gaps between
the two passes under rocprofv3 --kernel-trace.  Results are not checked."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if os.environ.get("STAMPS_LIB", "1") == "1":
    os.environ["ADL_BLOOM_LIB"] = os.path.join(ROOT, "adlsm-tree_amd", "lib_stamps", "libadlbloom.so")
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))
import torch  # noqa: E402

import adlbloom  # noqa: E402

keys = adlbloom.synth_keys16(10_000_000, seed=0x5EED, device="cuda:0")
if os.environ.get("PROFILE") == "1":
    adlbloom.profile_enable(64 * 20)
for _ in range(20):
    bm = adlbloom.build(keys, bits_per_key=10)
torch.cuda.synchronize()
print("done")
