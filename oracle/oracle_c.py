"""ctypes wrapper of the oracle's C restatement (oracle/oracle_c.c) —
TEST INFRASTRUCTURE ONLY (checker + bench.py's cpu_baseline leg)."""
from __future__ import annotations

import ctypes as C
import os
import platform

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle_c.so")
_lib = None

R_MOD = 21888242871839275222246405745257275088548364400416034343698204186575808495617
P_MOD = 21888242871839275222246405745257275088696311157297823662689037894645226208583
_M64 = (1 << 64) - 1
U64P = C.POINTER(C.c_uint64)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise FileNotFoundError(f"{LIB} missing (make -C oracle)")
        L = C.CDLL(LIB)
        U64P = C.POINTER(C.c_uint64)
        L.oc_msm.argtypes = [U64P, C.POINTER(C.c_uint8), U64P, C.c_size_t, U64P,
                             C.POINTER(C.c_uint8)]
        L.oc_bench_msm.argtypes = [C.c_int, C.c_uint64, C.POINTER(C.c_double),
                                   C.POINTER(C.c_double), U64P]
        L.oc_sumcheck_prod.argtypes = [C.c_int, C.c_int, U64P, U64P, C.POINTER(C.c_uint8), U64P,
                                       C.POINTER(C.c_uint32), U64P, U64P]
        L.oc_bench_msm_arrays.argtypes = [U64P, C.POINTER(C.c_uint8), U64P, C.c_size_t,
                                          C.POINTER(C.c_double), C.POINTER(C.c_double), U64P,
                                          C.POINTER(C.c_uint8)]
        L.oc_bench_sumcheck.argtypes = [C.c_int, C.c_uint64, C.POINTER(C.c_double)]
        L.oc_logup_column.argtypes = [U64P, U64P, U64P, C.c_size_t, U64P, U64P, U64P,
                                      C.POINTER(C.c_double)]
        L.oc_fr_horner.argtypes = [U64P, C.c_size_t, U64P, U64P]
        L.oc_fr_mle_eval.argtypes = [U64P, C.c_int, U64P, U64P]
        L.oc_fr_sum_prod.argtypes = [C.POINTER(U64P), C.c_int, C.c_size_t, U64P]
        L.oc_g1_mul.argtypes = [U64P, C.c_uint8, U64P, U64P, C.POINTER(C.c_uint8)]
        L.oc_bench_msm_arrays_mt.argtypes = [U64P, C.POINTER(C.c_uint8), U64P, C.c_size_t,
                                             C.c_int, C.POINTER(C.c_double), U64P,
                                             C.POINTER(C.c_uint8)]
        L.oc_sumcheck_prod_mt.argtypes = [C.c_int, C.c_int, U64P, U64P, C.POINTER(C.c_uint8),
                                          U64P, C.POINTER(C.c_uint32), U64P, U64P, C.c_int]
        L.oc_sumcheck_ref_prod.argtypes = [C.c_int, C.c_int, U64P, U64P, C.POINTER(C.c_uint8),
                                           U64P, C.POINTER(C.c_uint32), U64P, U64P]
        L.oc_bench_sumcheck_ref.argtypes = [C.c_int, C.c_uint64, C.POINTER(C.c_double)]
        L.oc_bench_sumcheck_mt.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
        U8P, U32P = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)
        L.oc_srs_set.argtypes = [U64P, C.c_size_t]
        L.oc_commit.argtypes = [U64P, C.c_size_t, U64P, U8P]
        L.oc_mle_open.argtypes = [U64P, C.c_size_t, U64P, C.c_int, U8P, U64P, U64P, U8P, U64P,
                                  U64P, U8P, U64P]
        L.oc_sumcheck_ref_expr.argtypes = [C.c_int, C.c_int, U64P, U32P, C.c_int, U64P, C.c_int,
                                           U64P, U8P, C.c_int, U64P, U32P, U64P, U64P]
        L.oc_logup_expr.argtypes = [C.c_int, C.c_size_t, U64P, U32P, C.c_int, U64P, C.c_int,
                                    U32P, C.c_int, U64P, C.c_int, U64P, U64P]
        L.oc_eq_table.argtypes = [U64P, C.c_int, U64P]
        _lib = L
    return _lib


def _mont(x, m):
    v = (x % m) * (1 << 256) % m
    return [(v >> (64 * i)) & _M64 for i in range(4)]


def _unmont(l, m):
    v = sum(int(l[i]) << (64 * i) for i in range(4))
    return v * pow(1 << 256, -1, m) % m


def msm(bases, scalars):
    """sum scalars[i] * bases[i] (affine canonical tuples / None) via the C Pippenger."""
    n = min(len(bases), len(scalars))
    xy = (C.c_uint64 * (8 * max(n, 1)))()
    inf = (C.c_uint8 * max(n, 1))()
    sc = (C.c_uint64 * (4 * max(n, 1)))()
    for i in range(n):
        P = bases[i]
        if P is None:
            inf[i] = 1
        else:
            for k, v in enumerate(_mont(P[0], P_MOD) + _mont(P[1], P_MOD)):
                xy[8 * i + k] = v
        for k, v in enumerate(_mont(scalars[i], R_MOD)):
            sc[4 * i + k] = v
    out = (C.c_uint64 * 8)()
    oinf = C.c_uint8()
    lib().oc_msm(xy, inf, sc, n, out, C.byref(oinf))
    if oinf.value:
        return None
    return (_unmont(out[:4], P_MOD), _unmont(out[4:8], P_MOD))


def sumcheck_prod(nvars, tables, claimed, state: bytes, variant="eval", nthreads=4):
    """h = prod tables; returns (r_polys, point, evaluation, new_state).
    variant: "eval" (evaluation form, 1 thread), "mt" (evaluation form,
    nthreads), "ref" (the reference's DensePolynomial / FFT-product structure)."""
    k = len(tables)
    N = 1 << nvars
    t = (C.c_uint64 * (4 * N * k))()
    for i, tb in enumerate(tables):
        for j, x in enumerate(tb):
            for q, v in enumerate(_mont(x, R_MOD)):
                t[4 * (i * N + j) + q] = v
    st = (C.c_uint8 * 32).from_buffer_copy(state)
    co = (C.c_uint64 * (4 * nvars * (k + 1)))()
    lens = (C.c_uint32 * nvars)()
    pt = (C.c_uint64 * (4 * nvars))()
    ev = (C.c_uint64 * 4)()
    cl = (C.c_uint64 * 4)(*_mont(claimed, R_MOD))
    if variant == "mt":
        lib().oc_sumcheck_prod_mt(nvars, k, t, cl, st, co, lens, pt, ev, nthreads)
    elif variant == "ref":
        lib().oc_sumcheck_ref_prod(nvars, k, t, cl, st, co, lens, pt, ev)
    else:
        lib().oc_sumcheck_prod(nvars, k, t, cl, st, co, lens, pt, ev)
    r_polys = [[_unmont(co[4 * (j * (k + 1) + i):4 * (j * (k + 1) + i) + 4], R_MOD)
                for i in range(lens[j])] for j in range(nvars)]
    point = [_unmont(pt[4 * j:4 * j + 4], R_MOD) for j in range(nvars)]
    return r_polys, point, _unmont(ev[:], R_MOD), bytes(st)


def sumcheck_prod_mont(nvars, mont_tables, claimed, state: bytes, variant="mt", nthreads=4):
    """sumcheck_prod on tables given as (2^nvars, 4) uint64 numpy arrays of
    Montgomery limbs (arkworks' in-memory Fr, as DeviceVec.to_numpy returns):
    no per-entry Python conversion, for the 2^20-variable parity test"""
    import numpy as np
    k = len(mont_tables)
    N = 1 << nvars
    flat = np.ascontiguousarray(np.concatenate([np.asarray(t, dtype=np.uint64).reshape(N, 4)
                                                for t in mont_tables]))
    t = flat.ctypes.data_as(C.POINTER(C.c_uint64))
    st = (C.c_uint8 * 32).from_buffer_copy(state)
    co = (C.c_uint64 * (4 * nvars * (k + 1)))()
    lens = (C.c_uint32 * nvars)()
    pt = (C.c_uint64 * (4 * nvars))()
    ev = (C.c_uint64 * 4)()
    cl = (C.c_uint64 * 4)(*_mont(claimed, R_MOD))
    if variant == "mt":
        lib().oc_sumcheck_prod_mt(nvars, k, t, cl, st, co, lens, pt, ev, nthreads)
    else:
        lib().oc_sumcheck_prod(nvars, k, t, cl, st, co, lens, pt, ev)
    r_polys = [[_unmont(co[4 * (j * (k + 1) + i):4 * (j * (k + 1) + i) + 4], R_MOD)
                for i in range(lens[j])] for j in range(nvars)]
    point = [_unmont(pt[4 * j:4 * j + 4], R_MOD) for j in range(nvars)]
    return r_polys, point, _unmont(ev[:], R_MOD), bytes(st)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def bench_msm_baseline(log_n: int = 18, seed: int = 0x5155494C4C):
    """Single-thread arkworks-faithful Pippenger on a 2^log_n sample (the
    reference has no rayon, so one core is the reference configuration)."""
    tm, tc = C.c_double(), C.c_double()
    out = (C.c_uint64 * 8)()
    lib().oc_bench_msm(log_n, seed, C.byref(tm), C.byref(tc), out)
    n = 1 << log_n
    return {"value": n / tm.value, "unit": "scalars/s", "cores": 1, "kind": "port",
            "sample": f"one MSM of 2^{log_n} uniform Fr scalars over [tau^i]g bases, "
                      f"msm_unchecked only ({tm.value:.2f} s); KZG::commit as written "
                      f"(+ into_affine of every SRS point) {n / tc.value:.4g} scalars/s",
            "seconds": tm.value, "kzg_commit_as_written_scalars_per_s": n / tc.value,
            "cpu_model": cpu_model()}


def bench_msm_arrays(xy, inf, scalars):
    """Single-thread arkworks-faithful Pippenger on caller arrays: xy (n, 8)
    uint64 affine Montgomery, inf (n,) uint8, scalars (n, 4) uint64 Montgomery.
    Returns (seconds_msm, seconds_commit_as_written, (xy limbs, inf))."""
    import numpy as np
    n = len(inf)
    xy = np.ascontiguousarray(xy, dtype=np.uint64)
    inf = np.ascontiguousarray(inf, dtype=np.uint8)
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    tm, tc = C.c_double(), C.c_double()
    out = (C.c_uint64 * 8)()
    oinf = C.c_uint8()
    P64, P8 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)
    lib().oc_bench_msm_arrays(xy.ctypes.data_as(P64), inf.ctypes.data_as(P8),
                              sc.ctypes.data_as(P64), C.c_size_t(n), C.byref(tm), C.byref(tc),
                              out, C.byref(oinf))
    return tm.value, tc.value, (list(out), oinf.value)


def usable_cores(cap: int = 16) -> int:
    """CPU threads for the all-cores baselines: this process's affinity, capped
    (the GPU box's share for one GPU is 16 threads)"""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


def bench_msm_arrays_mt(xy, inf, scalars, nthreads):
    """ark-ec's parallel window split on nthreads threads, same arrays and
    output as bench_msm_arrays.  Returns (seconds, (xy limbs, inf))."""
    import numpy as np
    n = len(inf)
    xy = np.ascontiguousarray(xy, dtype=np.uint64)
    inf = np.ascontiguousarray(inf, dtype=np.uint8)
    sc = np.ascontiguousarray(scalars, dtype=np.uint64)
    tm = C.c_double()
    out = (C.c_uint64 * 8)()
    oinf = C.c_uint8()
    P64, P8 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)
    lib().oc_bench_msm_arrays_mt(xy.ctypes.data_as(P64), inf.ctypes.data_as(P8),
                                 sc.ctypes.data_as(P64), C.c_size_t(n), nthreads, C.byref(tm),
                                 out, C.byref(oinf))
    return tm.value, (list(out), oinf.value)


def mle_open_ref(nvars: int, poly, point, tau: int, state: bytes):
    """C restatement of MLEvalProof::prove (mlpcs.rs:83-124) with the reference's
    data flow; bases [tau^i] g.  Returns (proof dict, new state, seconds)."""
    P64, P8 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)
    pa = np.array([_mont(x, R_MOD) for x in poly], dtype=np.uint64).reshape(-1, 4)
    pt = np.array([_mont(x, R_MOD) for x in point] or [[0, 0, 0, 0]],
                  dtype=np.uint64).reshape(-1, 4)
    st = (C.c_uint8 * 32)(*state)
    sec = C.c_double()
    ev, sc, y, pi = (C.c_uint64 * 4)(), (C.c_uint64 * 8)(), (C.c_uint64 * 16)(), (C.c_uint64 * 32)()
    sci, pii = C.c_uint8(), (C.c_uint8 * 4)()
    lib().oc_mle_open_ref(nvars, pa.ctypes.data_as(P64), pt.ctypes.data_as(P64),
                          (C.c_uint64 * 4)(*_mont(tau, R_MOD)), st, C.byref(sec), ev, sc,
                          C.byref(sci), y, pi, pii)
    g1 = lambda xy, inf: None if inf else (_unmont(list(xy)[:4], P_MOD), _unmont(list(xy)[4:8], P_MOD))
    out = {"evaluation": _unmont(list(ev), R_MOD), "s_comm": g1(sc, sci.value),
           "y": [_unmont(list(y)[4 * k:4 * k + 4], R_MOD) for k in range(4)],
           "proof": [g1(list(pi)[8 * k:8 * k + 8], pii[k]) for k in range(4)]}
    return out, bytes(st), sec.value


def bench_mle_open_ref(log_n: int, seed: int = 0x5155494C4C):
    """timed C MLEvalProof::prove at 2^log_n (random poly / point, fixed tau)"""
    import random
    rnd = random.Random(seed)
    poly = [rnd.randrange(R_MOD) for _ in range(1 << log_n)]
    point = [rnd.randrange(R_MOD) for _ in range(log_n)]
    _, _, sec = mle_open_ref(log_n, poly, point, 0x5155494C4C2D53525321, bytes(32))
    return sec


def bench_sumcheck_ref(log_n: int, seed: int = 0x5155494C4C):
    s = C.c_double()
    lib().oc_bench_sumcheck_ref(log_n, seed, C.byref(s))
    return s.value


def bench_sumcheck_mt(log_n: int, nthreads: int, seed: int = 0x5155494C4C):
    s = C.c_double()
    lib().oc_bench_sumcheck_mt(log_n, seed, nthreads, C.byref(s))
    return s.value


def bench_sumcheck_baseline(log_n: int = 16, seed: int = 0x5155494C4C):
    s = C.c_double()
    lib().oc_bench_sumcheck(log_n, seed, C.byref(s))
    return {"ms": s.value * 1e3, "cores": 1, "kind": "port",
            "sample": f"evaluation-form sumcheck prover, h = g1*g2*g3 at 2^{log_n} vars "
                      f"(lower bound on the reference's per-pair DensePolynomial structure)"}


def logup_column_arrays(t0, t1, t2, a_mont, beta_mont):
    """C restatement of the reference's per-row Logup loop on Montgomery-limb
    arrays (n x 4 uint64): out = t2 / (beta + t0 + a t1).  Returns (out, seconds);
    raises ZeroDivisionError on a zero denominator."""
    n = t0.shape[0]
    out = np.zeros((n, 4), dtype=np.uint64)
    s = C.c_double()
    arrs = [np.ascontiguousarray(x, dtype=np.uint64) for x in (t0, t1, t2)]
    av = np.array(a_mont, dtype=np.uint64)
    bv = np.array(beta_mont, dtype=np.uint64)
    p = [x.ctypes.data_as(U64P) for x in arrs]
    rc = lib().oc_logup_column(p[0], p[1], p[2], n, av.ctypes.data_as(U64P),
                               bv.ctypes.data_as(U64P), out.ctypes.data_as(U64P), C.byref(s))
    if rc:
        raise ZeroDivisionError("logup denominator is zero")
    return out, s.value


# ---------------------------------------------------------------- checkers
# Full-size checks of device results on Montgomery-limb numpy arrays (n x 4
# uint64, the layout DeviceVec.to_numpy returns): plain ints in and out.
def _limbs(x, m=R_MOD):
    return np.array(_mont(x, m), dtype=np.uint64)


def _arr(a):
    return np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 4)


def fr_horner(coeffs, x: int) -> int:
    """sum_i coeffs[i] x^i (kzg.rs:77-78); coeffs Montgomery limbs (n, 4)."""
    c = _arr(coeffs)
    xv, out = _limbs(x), np.zeros(4, dtype=np.uint64)
    lib().oc_fr_horner(c.ctypes.data_as(U64P), c.shape[0], xv.ctypes.data_as(U64P),
                       out.ctypes.data_as(U64P))
    return _unmont(out, R_MOD)


def fr_mle_eval(table, point) -> int:
    """MLE of the first 2^len(point) entries of table at point (bit j <-> point[j])."""
    t = _arr(table)
    nv = len(point)
    assert t.shape[0] >= 1 << nv
    pt = np.array([_mont(p, R_MOD) for p in point], dtype=np.uint64).reshape(-1)
    out = np.zeros(4, dtype=np.uint64)
    lib().oc_fr_mle_eval(t.ctypes.data_as(U64P), nv, pt.ctypes.data_as(U64P),
                         out.ctypes.data_as(U64P))
    return _unmont(out, R_MOD)


def fr_sum_prod(tables) -> int:
    """sum_i prod_j tables[j][i]"""
    ts = [_arr(t) for t in tables]
    n = min(t.shape[0] for t in ts)
    ptrs = (U64P * len(ts))(*[t.ctypes.data_as(U64P) for t in ts])
    out = np.zeros(4, dtype=np.uint64)
    lib().oc_fr_sum_prod(ptrs, len(ts), n, out.ctypes.data_as(U64P))
    return _unmont(out, R_MOD)


def g1_mul(P, s: int):
    """[s] P for an affine canonical point P = (x, y) or None (infinity)."""
    xy = np.zeros(8, dtype=np.uint64)
    if P is not None:
        xy[:4] = _mont(P[0], P_MOD)
        xy[4:] = _mont(P[1], P_MOD)
    sv, out, oinf = _limbs(s), np.zeros(8, dtype=np.uint64), C.c_uint8()
    lib().oc_g1_mul(xy.ctypes.data_as(U64P), 1 if P is None else 0, sv.ctypes.data_as(U64P),
                    out.ctypes.data_as(U64P), C.byref(oinf))
    if oinf.value:
        return None
    return (_unmont(out[:4], P_MOD), _unmont(out[4:], P_MOD))
