"""Register budget and spills of the built gfx950 kernels, read
from the code-object metadata of adlsm-tree_amd/lib/libadlbloom.so (no GPU).

* pass A (bloom_bin16 / bloom_bin) is capped at 120 VGPRs and the probe
  server at 32: four pass-A waves per SIMD plus the server's wave fill the
  512-entry register file, which is how a Get is served beside a build;
* no kernel on the headline build, the binned/direct probe or the var-len
  hashing path spills;
* the two kernels that do spill are pinned at their current amount: the
  resident server (kernel arguments and loop state, see probe_server.hip) and
  the generic var-len pass A (bloom_bin_kernel<KeysVar>, used only with
  ADL_BLOOM_SKIP_ADJACENT_DUPLICATES or k != 6)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "adlsm-tree_amd", "lib", "libadlbloom.so")

pytestmark = pytest.mark.skipif(
    not (os.path.exists(LIB) and shutil.which("llvm-readelf", path="/opt/rocm/lib/llvm/bin")),
    reason="needs the built library and ROCm's llvm tools")

ALLOWED_SCRATCH = {  # kernel substring -> max scratch bytes per lane
    "probe_server_kernel": 52,
    "bloom_bin_kernelILi1024ELi6ELi6EN7adl_dev7KeysVar": 40,
    "bloom_bin_kernelILi1024ELi0ELi8EN7adl_dev7KeysVar": 8,
}


@pytest.fixture(scope="module")
def res():
    import kernel_resources
    return kernel_resources.kernel_resources(LIB)


def test_every_kernel_found(res):
    for frag in ("bloom_bin16_kernel", "bloom_tile_kernel", "hash_var_kernel", "pb_tile_kernel", "pb_bin_kernel",
                 "pb_scatter_kernel", "bloom_probe_multi_kernel", "probe_server_kernel", "filter_block_pack_kernel"):
        assert any(frag in k for k in res), frag


def test_register_caps(res):
    for name, r in res.items():
        if "bloom_bin16_kernel" in name or "bloom_bin_kernel" in name:
            assert r["vgpr"] <= 120, (name, r)
        if "probe_server_kernel" in name:
            assert r["vgpr"] <= 32, (name, r)


def test_no_unexpected_spills(res):
    for name, r in res.items():
        cap = next((v for frag, v in ALLOWED_SCRATCH.items() if frag in name), 0)
        assert r["scratch"] <= cap, (name, r)
