"""CPU: Level::Get's candidate tables for a batch of lookups (the selection
half of LevelMultiGetFilter, adlsm-tree_amd/csrc/level_filter.cpp) against the
oracle's restatement of src/revision.cpp:278-287 (oracle.level_candidates),
on random levels with overlapping ranges, shared user keys and ties.  Host
code only: no compute call reaches the GPU."""
import ctypes
import os
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "adlsm-tree_amd", "lib", "libadlfilterblock.so")


@pytest.fixture(scope="module")
def lvl():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} is missing: run __graft_entry__.build()")
    L = ctypes.CDLL(LIB)
    f = L.adl_level_candidates
    pp = ctypes.POINTER(ctypes.c_char_p)
    f.restype = ctypes.c_int64
    f.argtypes = [pp, ctypes.c_void_p, pp, ctypes.c_void_p, ctypes.c_uint32, pp, ctypes.c_void_p, ctypes.c_uint32,
                  ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    return f


def inner(user: bytes, seq: int, op: int) -> bytes:
    return user + struct.pack("<q", seq) + bytes([op])


def candidates(f, tables, keys, seq):
    def arr(bs):
        return (ctypes.c_char_p * max(len(bs), 1))(*bs), np.array([len(b) for b in bs] or [0], dtype=np.uint64)

    mins, ml = arr([t[0] for t in tables])
    maxs, xl = arr([t[1] for t in tables])
    ks, kl = arr(keys)
    cap = len(tables) * len(keys) + 1
    begin = np.zeros(len(keys) + 1, dtype=np.uint32)
    table = np.zeros(cap, dtype=np.uint32)
    n = f(mins, ml.ctypes.data, maxs, xl.ctypes.data, len(tables), ks, kl.ctypes.data, len(keys), seq,
          begin.ctypes.data, table.ctypes.data, cap)
    assert n >= 0
    return [list(table[begin[i]:begin[i + 1]]) for i in range(len(keys))]


@pytest.mark.parametrize("seed", range(32))
def test_level_candidates_vs_oracle(lvl, oracle, seed):
    rng = np.random.default_rng(seed)
    users = sorted({bytes(rng.integers(97, 101, int(rng.integers(1, 4))).astype(np.uint8)) for _ in range(30)})
    T = int(rng.integers(0, 40))
    tables = []
    for _ in range(T):
        a, b = sorted(rng.integers(0, len(users), 2))
        s1, s2 = int(rng.integers(0, 50)), int(rng.integers(0, 50))
        mn, mx = inner(users[a], s1, int(rng.integers(0, 2))), inner(users[b], s2, int(rng.integers(0, 2)))
        if a == b and oracle._memkey_less(oracle._decode_inner(mx), oracle._decode_inner(mn)):
            mn, mx = mx, mn
        tables.append((mn, mx))
    if T > 3:  # ties: equal min keys, and a range repeated
        tables[1] = (tables[0][0], tables[1][1])
        tables[3] = tables[2]
    keys = [users[int(i)] for i in rng.integers(0, len(users), 60)]
    keys += [b"", b"a", b"zzz", users[0] + b"\x00", users[-1] + b"\xff"]
    seq = int(rng.choice([2**63 - 1, 25, 0]))
    got = candidates(lvl, tables, keys, seq)
    for i, k in enumerate(keys):
        assert got[i] == oracle.level_candidates(tables, k, seq), (i, k)


@pytest.mark.parametrize("seed,K", [(0, 1), (1, 3), (2, 40), (3, 400)])
def test_level_candidates_overlapping_direct_scan(lvl, oracle, seed, K):
    """An L0-shaped level: 300 tables whose ranges nearly all overlap, so the
    region lists would hold O(T^2) entries; with few lookups LevelCandidates
    scans the tables directly instead (same predicate, same visiting order).
    K = 400 takes the region sweep again; both must equal the oracle."""
    rng = np.random.default_rng(100 + seed)
    users = sorted({b"u%05d" % int(x) for x in rng.integers(0, 5000, 600)})
    tables = []
    for _ in range(300):
        a = int(rng.integers(0, 40))
        b = int(rng.integers(len(users) - 40, len(users)))
        tables.append((inner(users[a], int(rng.integers(0, 50)), 1), inner(users[b], int(rng.integers(0, 50)), 1)))
    keys = [users[int(i)] for i in rng.integers(0, len(users), K)]
    seq = 25
    got = candidates(lvl, tables, keys, seq)
    for i, k in enumerate(keys):
        assert got[i] == oracle.level_candidates(tables, k, seq), (i, k)


def test_level_candidates_disjoint_level_scales(lvl, oracle):
    """An L1-shaped level (disjoint ranges, 2 000 tables) and 20 000 lookups:
    at most one candidate each, the right one."""
    T, K = 2000, 20000
    tables = [(inner(b"k%08d" % (10 * t), 99, 1), inner(b"k%08d" % (10 * t + 9), 1, 1)) for t in range(T)]
    rng = np.random.default_rng(3)
    q = rng.integers(0, 10 * T + 50, K)
    keys = [b"k%08d" % v for v in q]
    got = candidates(lvl, tables, keys, 2**63 - 1)
    for i, v in enumerate(q):
        assert got[i] == ([int(v) // 10] if v < 10 * T else []), (i, v)
