"""tools/stamps.py -- per-phase cycle breakdown of the two build kernels.

Loads the s_memtime-instrumented library (make -C adlsm-tree_amd stamps),
runs the 10M x 16B headline build a few times and prints, per pass, the mean
over workgroups of the cycles wave 0 spent in each phase (phase = the span
between two of the kernel's barriers; see STAMP() in csrc/bloom_build.hip).
Diagnostics only; never part of the product path.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["ADL_BLOOM_LIB"] = os.path.join(ROOT, "adlsm-tree_amd", "lib_stamps", "libadlbloom.so")
sys.path.insert(0, os.path.join(ROOT, "adlsm-tree_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import adlbloom  # noqa: E402

NAMES = {
    0: ["loop-top (clear, hash)", "count+store(prev)", "scan", "table", "scatter", "epilogue", "-", "-"],
    1: ["tile start", "stage segs", "gather+or", "write+zero tile", "-", "-", "-", "-"],
    2: ["loads landed", "count + stage", "scan bins", "scatter slots", "hash + store (wave 0)", "-", "-", "-"],
}
# the generic pass A (bloom_bin_kernel: variable-length keys, WORKLOAD=varlen)
NAMES_GENERIC = ["length sort", "hash setup / rest", "count", "scan+table", "scatter", "store", "window load",
                 "window hash"]


def main():
    n = int(os.environ.get("N", 10_000_000))
    varlen = os.environ.get("WORKLOAD", "single") == "varlen"
    if varlen:
        NAMES[0] = NAMES_GENERIC
        data, offs = adlbloom.synth_varlen(n)
        for _ in range(3):
            bm = adlbloom.build(data, offsets=offs, bits_per_key=10)
    else:
        keys = adlbloom.synth_keys16(n, seed=0x5EED, device="cuda:0")
        for _ in range(3):
            bm = adlbloom.build(keys, bits_per_key=10)
    torch.cuda.synchronize()
    L = adlbloom.lib()
    L.adl_bloom_debug_stamps.restype = ctypes.c_int
    L.adl_bloom_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    if os.environ.get("BK", "1") != "0":  # the bucketed build (bloom_bucket.hip), the default
        raw = np.zeros(3 * 2048 * 8 + 2 * 256 * 16 * 8, dtype=np.uint64)
        assert L.adl_bloom_debug_stamps(raw.ctypes.data, raw.size) == 0
        bk = raw[3 * 2048 * 8:].reshape(2, 256, 16, 8)
        names = [["claims + hash", "claim barrier", "flush", "end barrier", "final flush", "slice set-up", "-", "-"],
                 ["counts + scan", "gather + or", "overflow", "tile barrier", "write + zero", "-", "-", "-"]]
        for p in (0, 1):
            print(f"pass {'AB'[p]} (bucketed): mean over 256 workgroups, cycles per phase, by wave")
            print("  wave " + "".join(f"{n[:13]:>14s}" for n in names[p] if n != "-"))
            for wv in range(16):
                row = bk[p, :, wv, :].astype(np.float64).mean(axis=0)
                print(f"  {wv:4d} " + "".join(f"{row[i]:14.0f}" for i in range(8) if names[p][i] != "-"))
        del bm
        return
    else:
        buf = np.zeros((3, 2048, 8), dtype=np.uint64)
        assert L.adl_bloom_debug_stamps(buf.ctypes.data, buf.size) == 0
    for p in ((0, 1, 2) if varlen and buf.shape[0] == 3 else (0, 1)):
        rows = buf[p][buf[p].sum(axis=1) > 0]
        tot = rows.sum(axis=1).mean()
        print(f"pass {'ABH'[p]}: {len(rows)} workgroups, mean total {tot:.0f} cycles")
        for i in range(8):
            if NAMES[p][i] == "-":
                continue
            col = rows[:, i].astype(np.float64)
            print(f"  {NAMES[p][i]:22s} mean {col.mean():9.0f}  max {col.max():9.0f}  ({100 * col.mean() / tot:5.1f} %)")
    if os.environ.get("DETAIL"):
        for p in (0, 1):
            rows = buf[p][:256]
            tot = rows.sum(axis=1).astype(np.float64)
            xcd = [tot[x::8].mean() for x in range(8)]
            print(f"pass {'AB'[p]} per-XCD mean total (blockIdx % 8):", " ".join(f"{v:.0f}" for v in xcd))
            order = np.argsort(tot)[::-1][:8]
            print(f"pass {'AB'[p]} slowest workgroups:", " ".join(f"{b}:{tot[b]:.0f}" for b in order))
            print(f"pass {'AB'[p]} fastest workgroups:", " ".join(f"{b}:{tot[b]:.0f}" for b in np.argsort(tot)[:8]))
    del bm


if __name__ == "__main__":
    main()
