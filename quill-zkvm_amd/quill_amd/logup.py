"""Logup PIOP mirror: MultisetEqualityProof (hyperplonk/src/piops/multiset_check.rs),
SetInclusionProof (set_inclusion.rs), PermutationCheckProof
(permutation_check.rs) and LookupProof (lookup.rs), proving on the gfx950
kernels through the C-ABI: the log-derivative columns (qg_logup_column), the
commitments (MSM), the eq table, the sumchecks and the ML-PCS openings all run
on the device; this module only sequences the transcript the way the
reference does.  Canonical Python ints for field elements."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import check, lib
from .device import Device, DeviceVec
from .field import R_MOD, eq_eval, fr_c, fr_from_mont_limbs, fr_list, u64p
from .hyperplonk import (SumcheckProof, VirtualPolyExpr, VirtualPolynomialStore, _default_device,
                         _program_c, _tables_c)
from .pcs import EvaluationClaim
from .transcript import Transcript


class LookupMode:
    """multiset_check.rs:11-16"""
    Subset = "subset"
    Equality = "equality"


def _expr_args(expr):
    if expr is None:
        return None, 0, None, 0, []
    prog, plen, carr, nc = _program_c(expr)
    return prog, plen, u64p(carr), nc, [carr]


def logup_column(store: VirtualPolynomialStore, h, beta: int, m=None, dev: Device = None):
    """m(x) / (beta + h(x)) for every row (multiset_check.rs:43-95,
    set_inclusion.rs:93-131); `h`, `m` are virtual-polynomial indices of
    `store` (m = None: 1).  Returns (column, sum of the column).  Raises
    QuillGpuError(QG_ERR_ASSERT) on a zero denominator, where the reference
    panics in inverse().unwrap()."""
    if store.on_device:
        out = DeviceVec(store.dev, store.local_len, pooled=True)
        s = logup_column_device(store.dev, store.num_vars, store.polynomials,
                                store.virtual_polys[h], beta, out,
                                store.virtual_polys[m] if m is not None else None)
        return out, s
    dev = dev or _default_device()
    n = store.num_vars
    hp = _expr_args(store.virtual_polys[h])
    mp = _expr_args(store.virtual_polys[m] if m is not None else None)
    arrs, ptrs = _tables_c(store.polynomials)
    out = np.zeros((1 << n, 4), dtype=np.uint64)
    s = (C.c_uint64 * 4)()
    check(lib().qg_logup_column(dev.h, n, len(arrs), ptrs, hp[0], hp[1], hp[2], hp[3], mp[0],
                                mp[1], mp[2], mp[3], fr_c(beta), u64p(out), s), dev.h)
    return fr_list(out), fr_from_mont_limbs(list(s))


def logup_column_device(dev: Device, num_vars: int, tables, h_expr: VirtualPolyExpr, beta: int,
                        out: DeviceVec, m_expr: VirtualPolyExpr = None) -> int:
    """Device-resident variant (tables and out are DeviceVec); returns the
    column sum.  With a communicator attached `num_vars` is global."""
    hp = _expr_args(h_expr)
    mp = _expr_args(m_expr)
    ptrs = (C.c_void_p * max(len(tables), 1))(*[t.h for t in tables])
    s = (C.c_uint64 * 4)()
    check(lib().qg_logup_column_dev(dev.h, num_vars, len(tables), ptrs, hp[0], hp[1], hp[2],
                                    hp[3], mp[0], mp[1], mp[2], mp[3], fr_c(beta), out.h, s),
          dev.h)
    return fr_from_mont_limbs(list(s))


def _eq_for(store: VirtualPolynomialStore, dev: Device, z):
    """eq(., z) table in the store's residency (device vector or host list)"""
    return store.dev.eq_table_dev(z) if store.on_device else dev.eq_table(z)


@dataclass
class MultisetEqualityProof:
    """multiset_check.rs:18-24"""
    denom_left_commitment: object
    denom_right_commitment: object
    sumcheck_proof: SumcheckProof
    opening_proof_denom_left: object
    opening_proof_denom_right: object

    @staticmethod
    def prove(store: VirtualPolynomialStore, h_left, h_right, transcript: Transcript, pcs,
              mode=LookupMode.Equality, multiplicities=None):
        """multiset_check.rs:28-181; mutates `store` like the reference
        (+denominator tables, +eq table, +the batched virtual polynomial).
        Returns (proof, evaluation point)."""
        dev = pcs.dev
        n = store.num_vars
        beta = transcript.draw_field_element()
        left, _ = logup_column(store, h_left, beta, None, dev)
        if mode == LookupMode.Subset:
            assert multiplicities is not None, \
                "Multiplicities polynomial must be provided in subset mode"
            right, _ = logup_column(store, h_right, beta, multiplicities, dev)
        else:
            assert multiplicities is None, \
                "Multiplicities polynomial must not be provided in equality mode"
            right, _ = logup_column(store, h_right, beta, None, dev)
        cl, cr = pcs.commit_batch([left, right])
        transcript.append_g1(cl)
        transcript.append_g1(cr)
        lam = transcript.draw_field_element()
        alpha = transcript.draw_field_element()
        dl = store.allocate_polynomial(left)
        dr = store.allocate_polynomial(right)
        E = VirtualPolyExpr
        m = store.virtual_polys[multiplicities] if mode == LookupMode.Subset else E.Const(1)
        zc = (E.Input(dl) * (E.Const(beta) + store.virtual_polys[h_left]) - E.Const(1)
              + E.Const(lam) * (E.Input(dr) * (E.Const(beta) + store.virtual_polys[h_right]) - m))
        z = [transcript.draw_field_element() for _ in range(n)]
        eq_idx = store.allocate_polynomial(_eq_for(store, dev, z))
        h_hat = store.new_virtual_from_expr(zc)
        store.mul_in_place(h_hat, eq_idx)
        store.mul_const_in_place(h_hat, alpha)
        store.add_in_place(h_hat, dl)
        store.sub_in_place(h_hat, dr)
        sc, claim = SumcheckProof.prove(n, store, h_hat, 0, transcript, dev)
        ol = pcs.open(left, claim.point, transcript)
        orr = pcs.open(right, claim.point, transcript)
        return MultisetEqualityProof(cl, cr, sc, ol, orr), claim.point

    def verify(self, transcript: Transcript, pcs, left_h_eval: EvaluationClaim,
               right_h_eval: EvaluationClaim, mode=LookupMode.Equality,
               multiplicities_eval: EvaluationClaim = None):
        """multiset_check.rs:185-292; raises ValueError with the reference's Err"""
        beta = transcript.draw_field_element()
        transcript.append_g1(self.denom_left_commitment)
        transcript.append_g1(self.denom_right_commitment)
        lam = transcript.draw_field_element()
        alpha = transcript.draw_field_element()
        z = [transcript.draw_field_element() for _ in range(len(left_h_eval.point))]
        if self.sumcheck_proof.claimed_sum % R_MOD != 0:
            raise ValueError("Multiset equality sumcheck claimed sum is not zero")
        claim = self.sumcheck_proof.verify(transcript)
        ok_l = pcs.verify(self.denom_left_commitment, self.opening_proof_denom_left, transcript)
        ok_r = pcs.verify(self.denom_right_commitment, self.opening_proof_denom_right, transcript)
        if not ok_l or not ok_r:
            raise ValueError("Multiset equality opening proof verification failed")
        if self.opening_proof_denom_left.point() != claim.point or \
                self.opening_proof_denom_right.point() != claim.point:
            raise ValueError("Multiset equality opening proof evaluation point does not match "
                             "sumcheck")
        if left_h_eval.point != claim.point or right_h_eval.point != claim.point:
            raise ValueError("Multiset equality h evaluation point does not match sumcheck")
        m = 1
        if mode == LookupMode.Subset:
            assert multiplicities_eval is not None, \
                "Multiplicities evaluation must be provided in subset mode"
            if multiplicities_eval.point != claim.point:
                raise ValueError("Multiset equality multiplicities evaluation point does not "
                                 "match sumcheck")
            m = multiplicities_eval.evaluation
        else:
            assert multiplicities_eval is None, \
                "Multiplicities evaluation must not be provided in equality mode"
        dl = self.opening_proof_denom_left.evaluation
        dr = self.opening_proof_denom_right.evaluation
        zc = (dl * (beta + left_h_eval.evaluation) - 1
              + lam * (dr * (beta + right_h_eval.evaluation) - m)) % R_MOD
        final = (zc * eq_eval(z, left_h_eval.point) % R_MOD * alpha + dl - dr) % R_MOD
        if final != claim.evaluation % R_MOD:
            raise ValueError("Multiset equality final evaluation does not match sumcheck")


@dataclass
class SetInclusionProof:
    """set_inclusion.rs:52-61"""
    denom_left_commitment: object
    denom_right_commitment: object
    sumcheck_proof_left: SumcheckProof
    sumcheck_proof_right: SumcheckProof
    opening_proof_denom_left: object
    opening_proof_denom_right: object

    @staticmethod
    def prove(store_left: VirtualPolynomialStore, h_left, store_right: VirtualPolynomialStore,
              h_right, multiplicities, transcript: Transcript, pcs):
        """set_inclusion.rs:74-235 -> (proof, (left point, right point))."""
        dev = pcs.dev
        nl, nr = store_left.num_vars, store_right.num_vars
        gamma = transcript.draw_field_element()  # logup_eval_point
        left, sum_left = logup_column(store_left, h_left, gamma, None, dev)
        right, sum_right = logup_column(store_right, h_right, gamma, multiplicities, dev)
        cl, cr = pcs.commit_batch([left, right])
        transcript.append_g1(cl)
        transcript.append_g1(cr)
        z1 = [transcript.draw_field_element() for _ in range(nl)]
        alpha = transcript.draw_field_element()
        dl = store_left.allocate_polynomial(left)
        dr = store_right.allocate_polynomial(right)
        E = VirtualPolyExpr
        m_expr = store_right.virtual_polys[multiplicities]
        hl = store_left.virtual_polys[h_left]
        hr = store_right.virtual_polys[h_right]
        eq1 = store_left.allocate_polynomial(_eq_for(store_left, dev, z1))
        el = E.Input(dl) * (E.Const(gamma) + hl) - E.Const(1)
        el = el * E.Input(eq1) + E.Input(dl) * E.Const(alpha)
        vl = store_left.new_virtual_from_expr(el)
        scl, cll = SumcheckProof.prove(nl, store_left, vl, sum_left * alpha % R_MOD, transcript,
                                       dev)
        z2 = [transcript.draw_field_element() for _ in range(nr)]
        beta = transcript.draw_field_element()
        eq2 = store_right.allocate_polynomial(_eq_for(store_right, dev, z2))
        er = E.Input(dr) * (E.Const(gamma) + hr) - m_expr
        er = er * E.Input(eq2) + E.Input(dr) * E.Const(beta)
        vr = store_right.new_virtual_from_expr(er)
        scr, clr = SumcheckProof.prove(nr, store_right, vr, sum_right * beta % R_MOD, transcript,
                                       dev)
        ol = pcs.open(left, cll.point, transcript)
        orr = pcs.open(right, clr.point, transcript)
        return SetInclusionProof(cl, cr, scl, scr, ol, orr), (cll.point, clr.point)


@dataclass
class PermutationCheckProof:
    """permutation_check.rs:8-10"""
    multiset_equality_proof: MultisetEqualityProof

    @staticmethod
    def prove(store: VirtualPolynomialStore, h_left, h_right, id_indices, permutation_indices,
              transcript: Transcript, pcs):
        """permutation_check.rs:13-59 -> (proof, evaluation point)."""
        n = store.num_vars
        assert len(id_indices) == store.local_len and len(permutation_indices) == store.local_len
        id_ref = store.allocate_polynomial(id_indices)
        perm_ref = store.allocate_polynomial(permutation_indices)
        alpha = transcript.draw_field_element()
        lh = store.new_virtual_from_virtual(h_left)
        store.mul_const_in_place(lh, alpha)
        store.add_in_place(lh, id_ref)
        rh = store.new_virtual_from_virtual(h_right)
        store.mul_const_in_place(rh, alpha)
        store.add_in_place(rh, perm_ref)
        proof, point = MultisetEqualityProof.prove(store, lh, rh, transcript, pcs,
                                                   LookupMode.Equality, None)
        return PermutationCheckProof(proof), point

    def verify(self, transcript: Transcript, pcs, left_h_eval: EvaluationClaim,
               right_h_eval: EvaluationClaim, id_eval: EvaluationClaim,
               perm_eval: EvaluationClaim):
        """permutation_check.rs:61-92"""
        alpha = transcript.draw_field_element()
        lhat = EvaluationClaim(list(left_h_eval.point),
                               (id_eval.evaluation + alpha * left_h_eval.evaluation) % R_MOD)
        rhat = EvaluationClaim(list(right_h_eval.point),
                               (perm_eval.evaluation + alpha * right_h_eval.evaluation) % R_MOD)
        self.multiset_equality_proof.verify(transcript, pcs, lhat, rhat, LookupMode.Equality,
                                            None)


@dataclass
class LookupProof:
    """lookup.rs:14-16"""
    set_inclusion_proof: SetInclusionProof

    @staticmethod
    def prove(source_store: VirtualPolynomialStore, source_cols, dest_store: VirtualPolynomialStore,
              dest_cols, multiplicities, transcript: Transcript, pcs):
        """lookup.rs:28-84 -> (proof, (source point, dest point))."""
        assert len(source_cols) == len(dest_cols), \
            "The number of source and destination columns must be equal"
        n = len(source_cols)
        transcript.append_u64(n)
        assert n > 0, "Lookup must be applied to at least one column"
        alpha = transcript.draw_field_element()
        ap = [pow(alpha, i, R_MOD) for i in range(n)]
        E = VirtualPolyExpr
        bl = source_store.virtual_polys[source_cols[0]]
        br = dest_store.virtual_polys[dest_cols[0]]
        for i in range(1, n):
            bl = bl + E.Const(ap[i]) * source_store.virtual_polys[source_cols[i]]
            br = br + E.Const(ap[i]) * dest_store.virtual_polys[dest_cols[i]]
        vl = source_store.new_virtual_from_expr(bl)
        vr = dest_store.new_virtual_from_expr(br)
        proof, pts = SetInclusionProof.prove(source_store, vl, dest_store, vr, multiplicities,
                                             transcript, pcs)
        return LookupProof(proof), pts


__all__ = ["LookupMode", "logup_column", "logup_column_device", "MultisetEqualityProof",
           "SetInclusionProof", "PermutationCheckProof", "LookupProof", "EvaluationClaim"]
