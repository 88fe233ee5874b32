"""TEST INFRASTRUCTURE / CPU BASELINE ONLY (never the product): HyperPlonk::prove
(proof.rs:145-301) with its heavy steps in C and the reference's data flow —
the C5 CPU baseline.  The orchestration (transcript order, expressions, store
mutations) is hyperplonk_oracle's; inside `c_backend()` the oracle's
  * KZG::commit           -> oc_commit (single-thread ark-style Pippenger over [tau^i] g)
  * MLEvalProof::prove    -> oc_mle_open (oracle_c.c: compute_pr + IFFT, FFT S polynomial,
                             long division + FFT assert, Pippenger; mlpcs.rs:83-124)
  * SumcheckProof::prove  -> oc_sumcheck_ref_expr (per-pair evaluate_expr_poly with ark-style
                             FFT products and allocations; sumcheck.rs:28-114)
  * logup_column          -> oc_logup_expr (multiset_check.rs:43-95)
  * fast_eq_eval_hypercube-> oc_eq_table (eq_eval.rs:6-31)
are swapped for C.  Checked bit-exact against the pure-Python restatement
(tests/test_oracle_c.py).  The Python glue (expression building, O(N) list
conversions, check_constraints) stays in the timed region, as a Rust caller's
equivalent work would."""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

import oracle_c as oc
import quill_oracle as qo

R = qo.R_MOD
P64, P8, P32 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)


def _arr(xs):
    b = b"".join((int(x) % R).to_bytes(32, "little") for x in xs)
    return np.frombuffer(b, dtype="<u8").reshape(-1, 4).copy() if xs else np.zeros((1, 4), "<u8")


def _ints(a, n):
    b = np.ascontiguousarray(a[:n]).tobytes()
    return [int.from_bytes(b[32 * i:32 * i + 32], "little") for i in range(n)]


def _g1(xy, inf):
    if inf:
        return None
    return (oc._unmont(list(xy)[:4], oc.P_MOD), oc._unmont(list(xy)[4:8], oc.P_MOD))


def _postfix(expr):
    """Expr -> (op, arg) pairs + constants (stack depth < 64 checked)"""
    ops, consts, depth, maxd = [], [], [0], [0]

    def rec(e):
        if e.kind == "in":
            ops.append((0, e.args[0]))
            depth[0] += 1
        elif e.kind == "const":
            ops.append((1, len(consts)))
            consts.append(e.args[0] % R)
            depth[0] += 1
        else:
            rec(e.args[0])
            rec(e.args[1])
            ops.append((2 if e.kind == "add" else 3, 0))
            depth[0] -= 1
        maxd[0] = max(maxd[0], depth[0])

    rec(expr)
    assert maxd[0] < 64, "expression stack too deep for the C evaluator"
    prog = np.array([v for op in ops for v in op], dtype=np.uint32)
    return prog, len(ops), _arr(consts), len(consts)


def _tables(polys, n):
    b = b"".join((int(x) % R).to_bytes(32, "little") for p in polys for x in p)
    return np.frombuffer(b, dtype="<u8").reshape(-1, 4).copy() if polys else np.zeros((1, 4), "<u8")


def _commit(self, poly):
    a = _arr(poly)
    xy, inf = (C.c_uint64 * 8)(), C.c_uint8()
    if oc.lib().oc_commit(a.ctypes.data_as(P64), C.c_size_t(len(poly)), xy, C.byref(inf)):
        raise ValueError("Polynomial degree exceeds max degree")
    return _g1(xy, inf.value)


def _mle_prove(poly, eval_point, kzg, t, trace=None):
    nv = len(eval_point)
    a, pt = _arr(poly), _arr(eval_point)
    st = (C.c_uint8 * 32)(*t.state)
    ev, sc, y, pi, x = ((C.c_uint64 * 4)(), (C.c_uint64 * 8)(), (C.c_uint64 * 16)(),
                        (C.c_uint64 * 32)(), (C.c_uint64 * 4)())
    sci, pii = C.c_uint8(), (C.c_uint8 * 4)()
    if oc.lib().oc_mle_open(a.ctypes.data_as(P64), C.c_size_t(len(poly)), pt.ctypes.data_as(P64),
                            nv, st, ev, sc, C.byref(sci), y, pi, pii, x):
        raise ValueError("Polynomial degree exceeds max degree")
    t.state = bytes(st)
    r = _ints(np.array(list(x), dtype=np.uint64).reshape(1, 4), 1)[0]
    ri = pow(r, R - 2, R)
    ys = _ints(np.array(list(y), dtype=np.uint64).reshape(4, 4), 4)
    pis = [_g1(list(pi)[8 * k:8 * k + 8], pii[k]) for k in range(4)]
    xs = (r, ri, r, ri)
    ev_i = _ints(np.array(list(ev), dtype=np.uint64).reshape(1, 4), 1)[0]
    return qo.MLEvalProof(list(eval_point), ev_i, _g1(sc, sci.value),
                          *[(xs[k], ys[k], pis[k]) for k in range(4)])


def _sumcheck(num_vars, store, h, claimed_sum, t):
    expr = store.virtual_polys[h]
    prog, plen, cs, nc = _postfix(expr)
    maxw = expr.degree() + 1
    tabs = _tables(store.polynomials, 1 << num_vars)
    st = (C.c_uint8 * 32)(*t.state)
    co = np.zeros((max(num_vars, 1) * maxw, 4), dtype=np.uint64)
    lens = np.zeros(max(num_vars, 1), dtype=np.uint32)
    pt = np.zeros((max(num_vars, 1), 4), dtype=np.uint64)
    ev = (C.c_uint64 * 4)()
    rc = oc.lib().oc_sumcheck_ref_expr(
        num_vars, len(store.polynomials), tabs.ctypes.data_as(P64), prog.ctypes.data_as(P32), plen,
        cs.ctypes.data_as(P64), nc, _arr([claimed_sum]).ctypes.data_as(P64), st, maxw,
        co.ctypes.data_as(P64), lens.ctypes.data_as(P32), pt.ctypes.data_as(P64), ev)
    assert rc == 0, "sumcheck message longer than the degree bound"
    t.state = bytes(st)
    allc = _ints(co, num_vars * maxw)
    r_polys = [allc[j * maxw:j * maxw + int(lens[j])] for j in range(num_vars)]
    final = _ints(np.array(list(ev), dtype=np.uint64).reshape(1, 4), 1)[0]
    return qo.SumcheckProof(num_vars, claimed_sum, r_polys), (_ints(pt, num_vars), final)


def _logup(store, h, beta, m=None):
    n = 1 << store.num_vars
    hp, hl, hc, hn = _postfix(store.virtual_polys[h])
    if m is not None:
        mp, ml, mc, mn = _postfix(store.virtual_polys[m])
    else:
        mp, ml, mc, mn = None, 0, _arr([]), 0
    tabs = _tables(store.polynomials, n)
    out = np.zeros((n, 4), dtype=np.uint64)
    rc = oc.lib().oc_logup_expr(
        len(store.polynomials), C.c_size_t(n), tabs.ctypes.data_as(P64), hp.ctypes.data_as(P32), hl,
        hc.ctypes.data_as(P64), hn, mp.ctypes.data_as(P32) if mp is not None else None, ml,
        mc.ctypes.data_as(P64), mn, _arr([beta]).ctypes.data_as(P64), out.ctypes.data_as(P64))
    if rc:
        raise ZeroDivisionError("logup denominator is zero (inverse().unwrap())")
    return _ints(out, n)


def _eq(n, point):
    out = np.zeros((1 << n, 4), dtype=np.uint64)
    oc.lib().oc_eq_table(_arr(point).ctypes.data_as(P64), n, out.ctypes.data_as(P64))
    return _ints(out, 1 << n)


@contextlib.contextmanager
def c_backend(tau: int, srs_len: int):
    """swap the oracle's heavy steps for the C restatement (SRS [tau^i] g, i < srs_len)"""
    lib = oc.lib()
    lib.oc_srs_set(_arr([tau]).ctypes.data_as(P64), C.c_size_t(srs_len))
    saved = (qo.KZG.commit, qo.MLEvalProof.prove, qo.SumcheckProof.prove,
             qo.SumcheckProof.prove_fast, qo.logup_column, qo.fast_eq_eval_hypercube)
    qo.KZG.commit = _commit
    qo.MLEvalProof.prove = staticmethod(_mle_prove)
    qo.SumcheckProof.prove = staticmethod(_sumcheck)
    qo.SumcheckProof.prove_fast = staticmethod(_sumcheck)
    qo.logup_column = _logup
    qo.fast_eq_eval_hypercube = _eq
    try:
        yield
    finally:
        (qo.KZG.commit, mp, sp, sf, qo.logup_column, qo.fast_eq_eval_hypercube) = saved
        qo.MLEvalProof.prove = staticmethod(mp)
        qo.SumcheckProof.prove = staticmethod(sp)
        qo.SumcheckProof.prove_fast = staticmethod(sf)
