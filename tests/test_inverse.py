"""Binary-GCD field inversion (csrc/bingcd.h, Pornin's optimized binary GCD)
through qg_selftest_inverse: host path on the CPU, device path on the GPU,
against Python's pow(x, -1, m) on random values, powers of two, values next
to the modulus and zero (-> 0, like ark's inverse() returning None)."""
import ctypes as C
import random

import numpy as np
import pytest

import quill_oracle as o
from quill_amd._lib import lib

MODS = [(0, o.R_MOD), (1, o.P_MOD)]


def _vals(m, seed, nrand):
    rnd = random.Random(seed)
    v = [0, 1, 2, 3, m - 1, m - 2, (m - 1) // 2]
    v += [1 << k for k in range(m.bit_length() - 1)]
    v += [m - (1 << k) for k in range(m.bit_length() - 1)]
    v += [rnd.randrange(m) for _ in range(nrand)]
    v += [rnd.randrange(1 << rnd.randrange(1, m.bit_length() - 1)) for _ in range(nrand // 4)]
    return v


def _run(ctx, field, dev, vals):
    n = len(vals)
    a = np.zeros((n, 4), dtype=np.uint64)
    for i, x in enumerate(vals):
        for limb in range(4):
            a[i, limb] = (x >> (64 * limb)) & (2**64 - 1)
    out = np.zeros((n, 4), dtype=np.uint64)
    rc = lib().qg_selftest_inverse(ctx, field, dev, a.ctypes.data_as(C.POINTER(C.c_uint64)),
                                   out.ctypes.data_as(C.POINTER(C.c_uint64)), C.c_size_t(n))
    assert rc == 0, rc
    return [sum(int(out[i, limb]) << (64 * limb) for limb in range(4)) for i in range(n)]


@pytest.mark.parametrize("field,m", MODS)
def test_bingcd_inverse_host(field, m):
    vals = _vals(m, field + 1, 4000)
    got = _run(None, field, 0, vals)
    for x, y in zip(vals, got):
        assert y == (pow(x, -1, m) if x else 0), x


def test_bingcd_rejects_noncanonical():
    a = np.array([[2**64 - 1] * 4], dtype=np.uint64)  # >= r
    out = np.zeros((1, 4), dtype=np.uint64)
    rc = lib().qg_selftest_inverse(None, 0, 0, a.ctypes.data_as(C.POINTER(C.c_uint64)),
                                   out.ctypes.data_as(C.POINTER(C.c_uint64)), C.c_size_t(1))
    assert rc != 0


@pytest.mark.gpu
@pytest.mark.parametrize("field,m", MODS)
def test_bingcd_inverse_device(dev, field, m):
    vals = _vals(m, field + 7, 20000)
    got = _run(dev.h, field, 1, vals)
    for x, y in zip(vals, got):
        assert y == (pow(x, -1, m) if x else 0), x
