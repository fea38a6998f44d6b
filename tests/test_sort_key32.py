"""CPU: the HIP batch sort's 32-bit keys (dofs_kernels.h key32_of / key32_etop, compiled into the emulator).

The packed MST sort orders (u32 key, value) pairs and the fix-up (dofs_sortfix.h) re-sorts runs of equal
32-bit keys by the full weight. That is exact only if the 32-bit key is monotone non-decreasing in the
64-bit weight key read as unsigned (segment.cpp:68's order of dbits(weight)), and useful only if weights
of the window keep their top 27 mantissa bits and the window's top bounds every weight of the frame.
"""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L(emu):
    lib = C.CDLL(os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so"))
    lib.emu_key32.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_void_p]
    lib.emu_key32_etop.argtypes = [C.c_int]
    lib.emu_key32_etop.restype = C.c_int
    lib.emu_key32b.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p]
    return lib


def _key32(L, k64, etop, m):
    k64 = np.ascontiguousarray(k64, dtype=np.uint64)
    out = np.empty(len(k64), np.uint32)
    L.emu_key32(k64.ctypes.data, len(k64), etop, m, out.ctypes.data)
    return out


def _etop(L, M):
    return L.emu_key32_etop(int(np.float32(M).view(np.int32)))


def _weights(rng, n, M):
    """KMstEmit's weights of random blurred components in [-M, M]: float subtraction, double squares."""
    b = rng.uniform(-M, M, size=(n, 4)).astype(np.float32)
    dx = (b[:, 0] - b[:, 2]).astype(np.float64)
    dy = (b[:, 1] - b[:, 3]).astype(np.float64)
    return np.sqrt(dx * dx + dy * dy)


@pytest.mark.parametrize("m", [27, 20, 8])
def test_key32_monotone_in_the_unsigned_key(L, m):
    rng = np.random.default_rng(5 + m)
    M = 37.5
    w = np.concatenate([
        _weights(rng, 20000, M),
        np.array([0.0, 5e-324, 1e-300, 1e-12, 2.0 ** -40, 1.0, 150.0, 1e30, np.inf, np.nan, -np.nan]),
        np.exp(rng.uniform(-60, 8, 20000)),  # far below the window too
    ])
    k64 = np.sort(w.view(np.uint64))  # unsigned order: a set sign bit sorts last
    k32 = _key32(L, k64, _etop(L, M), m)
    assert np.all(np.diff(k32.astype(np.int64)) >= 0)
    assert k32[-1] == 0xFFFFFFFF  # the sign-bit NaN at the top
    if m == 27:  # a window of 31 binades: zero (and the far smaller weights) at the bottom key
        assert k32[0] == 0


def test_key32_window_bounds_every_weight(L):
    """Every weight of components within [-M, M] lies at or below the window's top exponent."""
    rng = np.random.default_rng(9)
    for M in (1e-3, 0.7, 1.0, 3.9999, 4.0, 117.0, 3e4):
        etop = _etop(L, M)
        w = _weights(rng, 50000, M)
        extreme = np.array([np.sqrt(2.0) * 2 * np.float64(np.float32(M))])  # dx = dy = 2M
        e = (np.concatenate([w, extreme]).view(np.uint64) >> np.uint64(52)) & np.uint64(0x7FF)
        assert int(e.max()) <= etop, M


def test_key32_keeps_27_mantissa_bits_in_the_window(L):
    """Two weights of the window whose 64-bit keys differ above bit 25 get different 32-bit keys; the
    window spans 31 binades below the bound."""
    rng = np.random.default_rng(3)
    M = 20.0
    etop = _etop(L, M)
    w = np.exp(rng.uniform(np.log(2.0 ** (etop - 1023 - 30)), np.log(4 * M), 40000))
    k64 = np.unique(w.view(np.uint64))
    k32 = _key32(L, k64, etop, 27)
    top = k64 >> np.uint64(25)
    same32 = k32[1:] == k32[:-1]
    assert not np.any(same32 & (top[1:] != top[:-1]))
    assert k32.min() > 0  # nothing of the window collapses to the bottom key


@pytest.mark.parametrize("m,e", [(19, 5), (21, 3), (16, 8)])
def test_narrow_keys_monotone_and_capped(L, m, e):
    """Keys of m + e < 32 bits (dofs_debug_sort_k32e: three sort digits at 24 bits) stay monotone and below 2^(m+e),
    the sign-bit NaN and weights above the window at the largest one."""
    rng = np.random.default_rng(31 + m)
    M = 9.25
    w = np.concatenate([_weights(rng, 20000, M), np.exp(rng.uniform(-40, 6, 20000)),
                        np.array([0.0, 1e-300, 1.0, 1e30, np.inf, -np.nan])])
    k64 = np.sort(w.view(np.uint64))
    tb = m + e
    out = np.empty(len(k64), np.uint32)
    L.emu_key32b(k64.ctypes.data, len(k64), _etop(L, M), m, tb, out.ctypes.data)
    assert np.all(np.diff(out.astype(np.int64)) >= 0)
    assert int(out.max()) == (1 << tb) - 1 and out[-1] == (1 << tb) - 1 and out[0] == 0
    wide = np.empty(len(k64), np.uint32)  # inside the window the mantissa bits are the 32-bit key's
    L.emu_key32b(k64.ctypes.data, len(k64), _etop(L, M), m, 32, wide.ctypes.data)
    inw = (out > 0) & (out < (1 << tb) - 1)
    assert np.array_equal(out[inw] & np.uint32((1 << m) - 1), wide[inw] & np.uint32((1 << m) - 1))
