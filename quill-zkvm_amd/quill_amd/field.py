"""Conversions between canonical Python ints and the ABI's limb layout
(4 x u64 little-endian Montgomery limbs, R = 2^256 — arkworks' in-memory form)."""
from __future__ import annotations

import ctypes as C

import numpy as np

R_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617
P_MOD = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_R = 1 << 256
_M64 = (1 << 64) - 1
_RINV_R = pow(_R, -1, R_MOD)
_RINV_P = pow(_R, -1, P_MOD)


def _limbs(v: int):
    return [(v >> (64 * i)) & _M64 for i in range(4)]


def fr_to_mont_limbs(x: int):
    return _limbs((x % R_MOD) * _R % R_MOD)


def fr_from_mont_limbs(l) -> int:
    v = int(l[0]) | (int(l[1]) << 64) | (int(l[2]) << 128) | (int(l[3]) << 192)
    return v * _RINV_R % R_MOD


def fq_from_mont_limbs(l) -> int:
    v = int(l[0]) | (int(l[1]) << 64) | (int(l[2]) << 128) | (int(l[3]) << 192)
    return v * _RINV_P % P_MOD


def fq_to_mont_limbs(x: int):
    return _limbs((x % P_MOD) * _R % P_MOD)


def fr_array(xs) -> np.ndarray:
    """list of ints -> (n, 4) uint64 Montgomery array (C-contiguous)."""
    out = np.empty((len(xs), 4), dtype=np.uint64)
    for i, x in enumerate(xs):
        m = (int(x) % R_MOD) * _R % R_MOD
        out[i, 0] = m & _M64
        out[i, 1] = (m >> 64) & _M64
        out[i, 2] = (m >> 128) & _M64
        out[i, 3] = m >> 192
    return out


def fr_canonical_array(xs) -> np.ndarray:
    """list of ints -> (n, 4) uint64 canonical limbs (reduced mod r); the device
    converts to Montgomery form (DeviceVec.from_canonical)."""
    b = b"".join((int(x) % R_MOD).to_bytes(32, "little") for x in xs)
    return np.frombuffer(b, dtype="<u8").reshape(len(xs), 4).copy()


def fr_inv(x: int) -> int:
    x %= R_MOD
    if x == 0:
        raise ZeroDivisionError("inverse of zero in Fr")
    return pow(x, R_MOD - 2, R_MOD)


def eq_eval(x, y) -> int:
    """eq(x, y) = prod_i (x_i y_i + (1 - x_i)(1 - y_i))  (eq_eval.rs:33-43);
    unequal lengths raise like the reference's assert_eq! (eq_eval.rs:34)"""
    if len(x) != len(y):
        raise ValueError(f"eq_eval: point lengths differ ({len(x)} vs {len(y)})")
    acc = 1
    for a, b in zip(x, y):
        acc = acc * (a * b + (1 - a) * (1 - b)) % R_MOD
    return acc


def fr_list(arr) -> list:
    a = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    return [fr_from_mont_limbs(row) for row in a]


_U64_ARR = {}
_U32_ARR = {}


def _arr_type(cache, ct, n):
    t = cache.get(n)
    if t is None:
        t = cache[n] = ct * n
    return t


def u64p(arr: np.ndarray):
    """The array's memory as a u64* argument.  A writable array is wrapped as a
    ctypes array over the same buffer (~0.5 us; ndarray.ctypes.data_as costs
    ~4 us, which the per-call wrappers of the small provers paid several times)."""
    assert arr.dtype == np.uint64 and arr.flags["C_CONTIGUOUS"]
    if arr.flags.writeable and arr.size:
        return _arr_type(_U64_ARR, C.c_uint64, arr.size).from_buffer(arr)
    return arr.ctypes.data_as(C.POINTER(C.c_uint64))


def u32p(arr: np.ndarray):
    """u32 counterpart of u64p"""
    assert arr.dtype == np.uint32 and arr.flags["C_CONTIGUOUS"]
    if arr.flags.writeable and arr.size:
        return _arr_type(_U32_ARR, C.c_uint32, arr.size).from_buffer(arr)
    return arr.ctypes.data_as(C.POINTER(C.c_uint32))


_FR_C_SMALL = {}


def fr_c(x: int):
    if 0 <= x < 256:  # small constants (claims of 0, ones) recur in every call
        limbs = _FR_C_SMALL.get(x)
        if limbs is None:
            limbs = _FR_C_SMALL[x] = tuple(fr_to_mont_limbs(x))
        return (C.c_uint64 * 4)(*limbs)
    return (C.c_uint64 * 4)(*fr_to_mont_limbs(x))


def g1_from_abi(xy, inf):
    """ABI affine (Montgomery limbs + flag) -> canonical (x, y) or None."""
    if inf:
        return None
    return (fq_from_mont_limbs(list(xy)[:4]), fq_from_mont_limbs(list(xy)[4:8]))


def g1_to_abi(P):
    xy = (C.c_uint64 * 8)()
    if P is None:
        return xy, 1
    lx, ly = fq_to_mont_limbs(P[0]), fq_to_mont_limbs(P[1])
    for i in range(4):
        xy[i] = lx[i]
        xy[4 + i] = ly[i]
    return xy, 0


def g2_from_abi(xy, inf):
    """ABI G2 (x.c0, x.c1, y.c0, y.c1 Montgomery limbs) -> ((x0, x1), (y0, y1)) or None"""
    if inf:
        return None
    v = [fq_from_mont_limbs(list(xy)[4 * k:4 * k + 4]) for k in range(4)]
    return ((v[0], v[1]), (v[2], v[3]))


def g2_to_abi(Q):
    xy = (C.c_uint64 * 16)()
    if Q is None:
        return xy, 1
    for k, c in enumerate((Q[0][0], Q[0][1], Q[1][0], Q[1][1])):
        for i, limb in enumerate(fq_to_mont_limbs(c)):
            xy[4 * k + i] = limb
    return xy, 0
