"""hyperplonk mirror: VirtualPolyExpr / VirtualPolynomialStore
(hyperplonk/src/utils/virtual_polynomial.rs), SumcheckProof
(hyperplonk/src/piops/sumcheck.rs) and ZeroCheckProof
(hyperplonk/src/piops/zerocheck.rs), proving on the gfx950 kernels through the
C-ABI.  Canonical Python ints for field elements."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import ExprOp, check, lib
from .device import Device, DeviceVec
from .field import R_MOD, eq_eval, fr_array, fr_c, fr_canonical_array, fr_inv, fr_list, u32p, u64p
from .pcs import EvaluationClaim
from .transcript import Transcript

OP_INPUT, OP_CONST, OP_ADD, OP_MUL = 0, 1, 2, 3


class VirtualPolyExpr:
    """virtual_polynomial.rs:9-18 (Input / Const / Add / Mul); Sub is
    Add(a, Mul(Const(-1), b)) as at :67-77."""

    def __init__(self, kind, *args):
        self.kind, self.args = kind, args

    @staticmethod
    def Input(i):
        return VirtualPolyExpr("in", i)

    @staticmethod
    def Const(c):
        return VirtualPolyExpr("const", c % R_MOD)

    def __add__(self, o):
        return VirtualPolyExpr("add", self, o)

    def __mul__(self, o):
        return VirtualPolyExpr("mul", self, o)

    def __sub__(self, o):
        return VirtualPolyExpr("add", self, VirtualPolyExpr("mul", VirtualPolyExpr.Const(-1), o))

    def evaluate(self, g):
        """virtual_polynomial.rs:22-37"""
        if self.kind == "in":
            return g[self.args[0]] % R_MOD
        if self.kind == "const":
            return self.args[0]
        a, b = self.args[0].evaluate(g), self.args[1].evaluate(g)
        return (a + b) % R_MOD if self.kind == "add" else a * b % R_MOD

    def to_program(self):
        """postfix program (qg_expr_op[]) + constant pool"""
        ops, consts = [], []

        def rec(e):
            if e.kind == "in":
                ops.append((OP_INPUT, e.args[0]))
            elif e.kind == "const":
                ops.append((OP_CONST, len(consts)))
                consts.append(e.args[0])
            else:
                rec(e.args[0])
                rec(e.args[1])
                ops.append((OP_ADD if e.kind == "add" else OP_MUL, 0))

        rec(self)
        return ops, consts


def _program_c(expr: VirtualPolyExpr):
    # expressions are immutable once built: the compiled program (read-only for
    # the library) is kept on the object, so a prover called in a loop does not
    # recompile it per call
    c = expr.__dict__.get("_qg_prog")
    if c is None:
        ops, consts = expr.to_program()
        prog = (ExprOp * len(ops))(*[ExprOp(o, a) for o, a in ops])
        carr = fr_array(consts) if consts else np.zeros((1, 4), dtype=np.uint64)
        c = expr._qg_prog = (prog, len(ops), carr, len(consts))
    return c


def expr_degree(expr: VirtualPolyExpr) -> int:
    d = expr.__dict__.get("_qg_deg")
    if d is None:
        prog, n, _, _ = _program_c(expr)
        dd = C.c_uint32()
        check(lib().qg_expr_degree(prog, n, C.byref(dd)))
        d = expr._qg_deg = dd.value
    return d


class VirtualPolynomialStore:
    """virtual_polynomial.rs:142-331.

    Host store (dev=None): tables are lists of canonical ints, uploaded per call.
    Device store (dev given): tables are DeviceVec (HBM-resident; host lists are
    uploaded once at allocation) and every prover below runs on them in place.
    The reference clones each table into the store (:161-171); tables are never
    mutated here, so the device store keeps a reference instead of a copy."""

    def __init__(self, num_vars: int, dev: Device = None):
        self.num_vars = num_vars
        self.dev = dev
        self.polynomials = []
        self.virtual_polys = []

    @property
    def on_device(self) -> bool:
        return self.dev is not None

    @property
    def local_len(self) -> int:
        """entries per table held here: 2^num_vars, or this rank's block of
        2^num_vars / world with a communicator attached"""
        return (1 << self.num_vars) // (self.dev.world if self.dev is not None else 1)

    def allocate_polynomial(self, evals):
        assert len(evals) == self.local_len, \
            "Input polynomial evaluations length does not match number of variables"
        if self.dev is not None:
            if not isinstance(evals, DeviceVec):
                evals = DeviceVec.from_canonical(self.dev, fr_canonical_array(evals))
            self.polynomials.append(evals)
        else:
            if isinstance(evals, DeviceVec):
                evals = evals.to_list()
            self.polynomials.append([int(e) % R_MOD for e in evals])
        return len(self.polynomials) - 1

    def new_virtual_from_input(self, g):
        self.virtual_polys.append(VirtualPolyExpr.Input(g))
        return len(self.virtual_polys) - 1

    def new_virtual_from_virtual(self, v):
        self.virtual_polys.append(self.virtual_polys[v])
        return len(self.virtual_polys) - 1

    def new_virtual_from_expr(self, e):
        self.virtual_polys.append(e)
        return len(self.virtual_polys) - 1

    def add_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] + VirtualPolyExpr.Input(g)

    def add_const_in_place(self, f, c):
        self.virtual_polys[f] = self.virtual_polys[f] + VirtualPolyExpr.Const(c)

    def sub_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] + (
            VirtualPolyExpr.Const(-1) * VirtualPolyExpr.Input(g))

    def mul_in_place(self, f, g):
        self.virtual_polys[f] = self.virtual_polys[f] * VirtualPolyExpr.Input(g)

    def mul_const_in_place(self, f, c):
        self.virtual_polys[f] = self.virtual_polys[f] * VirtualPolyExpr.Const(c)

    def evaluate_point(self, g_evals, h):
        return self.virtual_polys[h].evaluate(g_evals)


def _tables_c(tables):
    arrs = [fr_array(t) for t in tables]
    ptrs = (C.POINTER(C.c_uint64) * max(len(arrs), 1))(*[u64p(a) for a in arrs])
    return arrs, ptrs


def _unpack(nvars, width, coeffs, lens, point, ev):
    from .field import fr_from_mont_limbs
    r_polys = []
    c = coeffs.reshape(nvars, width, 4)
    for j in range(nvars):
        r_polys.append([fr_from_mont_limbs(c[j, i]) for i in range(lens[j])])
    pt = fr_list(point)
    return r_polys, pt, fr_from_mont_limbs(list(ev))


@dataclass
class SumcheckProof:
    """sumcheck.rs:15-19"""
    num_vars: int
    claimed_sum: int
    r_polys: list

    @staticmethod
    def prove(num_vars, store: VirtualPolynomialStore, h, claimed_sum, transcript: Transcript,
              dev: Device = None):
        """sumcheck.rs:28-114 on the device; returns (proof, EvaluationClaim)."""
        if store.on_device:
            r_polys, pt, e = _unpack_dev(num_vars, store.virtual_polys[h], *sumcheck_prove_device(
                store.dev, num_vars, store.polynomials, store.virtual_polys[h], claimed_sum,
                transcript))
            return SumcheckProof(num_vars, claimed_sum % R_MOD, r_polys), EvaluationClaim(pt, e)
        dev = dev or _default_device()
        expr = store.virtual_polys[h]
        prog, plen, carr, nc = _program_c(expr)
        width = expr_degree(expr) + 1
        arrs, ptrs = _tables_c(store.polynomials)
        coeffs = np.zeros((num_vars * width, 4), dtype=np.uint64)
        lens = np.zeros(num_vars, dtype=np.uint32)
        point = np.zeros((num_vars, 4), dtype=np.uint64)
        ev = (C.c_uint64 * 4)()
        check(lib().qg_sumcheck_prove(
            dev.h, num_vars, len(arrs), ptrs, prog, plen, u64p(carr), nc, fr_c(claimed_sum),
            transcript.c_state(), u64p(coeffs), lens.ctypes.data_as(C.POINTER(C.c_uint32)),
            u64p(point), ev), dev.h)
        r_polys, pt, e = _unpack(num_vars, width, coeffs, lens, point, ev)
        return SumcheckProof(num_vars, claimed_sum % R_MOD, r_polys), EvaluationClaim(pt, e)


def _poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R_MOD
    return acc


def _sumcheck_verify(self, transcript: Transcript) -> EvaluationClaim:
    """sumcheck.rs:116-150: r_i(0) + r_i(1) == v per round; raises ValueError
    with the reference's Err message"""
    transcript.append_u64(self.num_vars)
    transcript.append_fr(self.claimed_sum)
    v = self.claimed_sum % R_MOD
    point = []
    for rp in self.r_polys:
        if (_poly_eval(rp, 0) + _poly_eval(rp, 1)) % R_MOD != v:
            raise ValueError("Sumcheck polynomial does not sum to previous value")
        transcript.append_poly(rp)
        r = transcript.draw_field_element()
        point.append(r)
        v = _poly_eval(rp, r)
    return EvaluationClaim(point, v)


SumcheckProof.verify = _sumcheck_verify


@dataclass
class ZeroCheckProof:
    """zerocheck.rs:8-11"""
    num_vars: int
    sumcheck_proof: SumcheckProof

    def verify(self, transcript: Transcript) -> EvaluationClaim:
        """zerocheck.rs:51-75"""
        z = [transcript.draw_field_element() for _ in range(self.num_vars)]
        if self.sumcheck_proof.claimed_sum % R_MOD != 0:
            raise ValueError("Sumcheck claimed sum is not zero")
        if self.sumcheck_proof.num_vars != self.num_vars:
            raise ValueError("Sumcheck proof num_vars does not match zerocheck num_vars")
        claim = self.sumcheck_proof.verify(transcript)
        # division by eq_eval: ark's `/` panics on zero, like fr_inv here
        e = eq_eval(z, claim.point)
        return EvaluationClaim(claim.point, claim.evaluation * fr_inv(e) % R_MOD)

    @staticmethod
    def prove(store: VirtualPolynomialStore, h, transcript: Transcript, dev: Device = None):
        """zerocheck.rs:14-49 on the device.  Mutates `store` exactly like the
        reference: appends the eq table and the virtual polynomial h * eq."""
        if store.on_device:
            return ZeroCheckProof._prove_dev(store, h, transcript)
        dev = dev or _default_device()
        n = store.num_vars
        expr = store.virtual_polys[h]
        prog, plen, carr, nc = _program_c(expr)
        width = expr_degree(expr) + 2
        arrs, ptrs = _tables_c(store.polynomials)
        coeffs = np.zeros((n * width, 4), dtype=np.uint64)
        lens = np.zeros(n, dtype=np.uint32)
        point = np.zeros((n, 4), dtype=np.uint64)
        eq = np.zeros((1 << n, 4), dtype=np.uint64)
        ev = (C.c_uint64 * 4)()
        check(lib().qg_zerocheck_prove(
            dev.h, n, len(arrs), ptrs, prog, plen, u64p(carr), nc, transcript.c_state(),
            u64p(coeffs), lens.ctypes.data_as(C.POINTER(C.c_uint32)), u64p(point), ev,
            u64p(eq)), dev.h)
        # store mutation of zerocheck.rs:27-29
        eq_idx = store.allocate_polynomial(fr_list(eq))
        h_hat = store.new_virtual_from_virtual(h)
        store.mul_in_place(h_hat, eq_idx)
        r_polys, pt, e = _unpack(n, width, coeffs, lens, point, ev)
        return (ZeroCheckProof(n, SumcheckProof(n, 0, r_polys)), EvaluationClaim(pt, e))


def _prove_dev_zc(store, h, transcript):
    """zerocheck.rs:14-49 over a device store, step for step: draw z, eq table
    on the device, store mutation, sumcheck of h * eq with sum 0, claim / eq(z, pt)."""
    n = store.num_vars
    z = [transcript.draw_field_element() for _ in range(n)]
    eq_idx = store.allocate_polynomial(store.dev.eq_table_dev(z))
    h_hat = store.new_virtual_from_virtual(h)
    store.mul_in_place(h_hat, eq_idx)
    proof, claim = SumcheckProof.prove(n, store, h_hat, 0, transcript)
    ev = claim.evaluation * fr_inv(eq_eval(z, claim.point)) % R_MOD
    return ZeroCheckProof(n, proof), EvaluationClaim(claim.point, ev)


ZeroCheckProof._prove_dev = staticmethod(_prove_dev_zc)


def _unpack_dev(num_vars, expr, coeffs, lens, point, ev):
    return _unpack(num_vars, expr_degree(expr) + 1, coeffs, lens, point, ev)


def sumcheck_prove_tables(dev: Device, num_vars: int, tables, expr: VirtualPolyExpr,
                          claimed_sum: int, transcript: Transcript, zerocheck: bool = False):
    """qg_sumcheck_prove / qg_zerocheck_prove on host tables (lists of ints).
    With a communicator attached, `num_vars` is global and `tables` are this
    rank's blocks.  Returns (r_polys, point, evaluation)."""
    prog, plen, carr, nc = _program_c(expr)
    width = expr_degree(expr) + (2 if zerocheck else 1)
    arrs, ptrs = _tables_c(tables)
    coeffs = np.zeros((num_vars * width, 4), dtype=np.uint64)
    lens = np.zeros(num_vars, dtype=np.uint32)
    point = np.zeros((num_vars, 4), dtype=np.uint64)
    ev = (C.c_uint64 * 4)()
    L = lib()
    if zerocheck:
        rc = L.qg_zerocheck_prove(dev.h, num_vars, len(arrs), ptrs, prog, plen, u64p(carr), nc,
                                  transcript.c_state(), u64p(coeffs),
                                  lens.ctypes.data_as(C.POINTER(C.c_uint32)), u64p(point), ev, None)
    else:
        rc = L.qg_sumcheck_prove(dev.h, num_vars, len(arrs), ptrs, prog, plen, u64p(carr), nc,
                                 fr_c(claimed_sum), transcript.c_state(), u64p(coeffs),
                                 lens.ctypes.data_as(C.POINTER(C.c_uint32)), u64p(point), ev)
    check(rc, dev.h)
    return _unpack(num_vars, width, coeffs, lens, point, ev)


def sumcheck_prove_device(dev: Device, num_vars: int, tables, expr: VirtualPolyExpr,
                          claimed_sum: int, transcript: Transcript):
    """Device-resident variant (tables are DeviceVec): the bench entry point."""
    prog, plen, carr, nc = _program_c(expr)
    width = expr_degree(expr) + 1
    ptrs = (C.c_void_p * len(tables))(*[t.h for t in tables])
    coeffs = np.zeros((num_vars * width, 4), dtype=np.uint64)
    lens = np.zeros(num_vars, dtype=np.uint32)
    point = np.zeros((num_vars, 4), dtype=np.uint64)
    ev = (C.c_uint64 * 4)()
    check(lib().qg_sumcheck_prove_dev(
        dev.h, num_vars, len(tables), ptrs, prog, plen, u64p(carr), nc, fr_c(claimed_sum),
        transcript.c_state(), u64p(coeffs), u32p(lens), u64p(point), ev), dev.h)
    return coeffs, lens, point, ev


def zerocheck_prove_device(dev: Device, num_vars: int, tables, expr: VirtualPolyExpr,
                           transcript: Transcript):
    """qg_zerocheck_prove_dev on DeviceVec tables (the bench's zero-check
    variant): returns the raw (coeffs, lens, point, ev) like
    sumcheck_prove_device, round messages of degree(expr) + 1."""
    prog, plen, carr, nc = _program_c(expr)
    width = expr_degree(expr) + 2
    ptrs = (C.c_void_p * len(tables))(*[t.h for t in tables])
    coeffs = np.zeros((num_vars * width, 4), dtype=np.uint64)
    lens = np.zeros(num_vars, dtype=np.uint32)
    point = np.zeros((num_vars, 4), dtype=np.uint64)
    ev = (C.c_uint64 * 4)()
    check(lib().qg_zerocheck_prove_dev(
        dev.h, num_vars, len(tables), ptrs, prog, plen, u64p(carr), nc, transcript.c_state(),
        u64p(coeffs), u32p(lens), u64p(point), ev), dev.h)
    return coeffs, lens, point, ev


def sumcheck_prove_callback(dev: Device, num_vars: int, tables, expr: VirtualPolyExpr,
                            challenge):
    """qg_sumcheck_prove_cb: the caller's transcript stays authoritative.
    `challenge(coeffs) -> r` gets each round's trimmed message (list of Fr
    ints) and returns r_j; the caller has absorbed num_vars and the claimed
    sum beforehand (sumcheck.rs:35-36).  Tables are DeviceVec.  Returns
    (r_polys, point, evaluation)."""
    from ._lib import CHALLENGE_FN
    from .field import fr_from_mont_limbs, fr_to_mont_limbs
    prog, plen, carr, nc = _program_c(expr)
    width = expr_degree(expr) + 1
    ptrs = (C.c_void_p * len(tables))(*[t.h for t in tables])
    coeffs = np.zeros((num_vars * width, 4), dtype=np.uint64)
    lens = np.zeros(num_vars, dtype=np.uint32)
    point = np.zeros((num_vars, 4), dtype=np.uint64)
    ev = (C.c_uint64 * 4)()
    errors = []

    def _cb(_user, cptr, n, out):
        try:
            msg = [fr_from_mont_limbs([cptr[4 * i + k] for k in range(4)]) for i in range(n)]
            limbs = fr_to_mont_limbs(int(challenge(msg)))
            for k in range(4):
                out[k] = limbs[k]
            return 0
        except Exception as e:  # reported after the call
            errors.append(e)
            return 1
    fn = CHALLENGE_FN(_cb)
    rc = lib().qg_sumcheck_prove_cb(dev.h, num_vars, len(tables), ptrs, prog, plen, u64p(carr),
                                    nc, fn, None, u64p(coeffs), u32p(lens), u64p(point), ev)
    if errors:
        raise errors[0]
    check(rc, dev.h)
    return _unpack(num_vars, width, coeffs, lens, point, ev)


_DEV = None


def _default_device():
    global _DEV
    if _DEV is None:
        _DEV = Device(0)
    return _DEV
