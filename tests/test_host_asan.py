"""CPU: the host sanitizer build (make -C adlsm-tree_amd asan).

The reference builds every target with -fsanitize=address by default
(CMakeLists.txt:5,13).  Here the code that parses and frames
untrusted bytes -- the filter-block trailer walk behind FilterBlockReader::Init
and the device filter cache, FilterBlockWriter::Final's framing, the
SSTableWriter's blocks and footer -- is compiled with
-fsanitize=address,undefined and run over truncated, corrupted and hostile
blocks (csrc/asan_test.cpp).  Nothing in it reaches the GPU.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "adlsm-tree_amd")


def test_asan_parse_and_framing():
    subprocess.run(["make", "-s", "-C", PKG, "asan"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(PKG, "bin_asan", "asan_test")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed checks" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
