"""PCS mirror: KZG (pcs/src/kzg.rs), MLEvalProof (pcs/src/mlpcs.rs) and the
MultilinearPCS trait surface (pcs/src/lib.rs:26-41), backed by the gfx950
kernels through the C-ABI.  Field elements are canonical Python ints; G1 points
are affine (x, y) tuples or None (infinity)."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from ._lib import KzgOpening, KzgVk, MleOpenItem, MleProof, QuillGpuError, check, lib
from .device import Device, DeviceVec, Srs
from .field import (fq_from_mont_limbs, fr_array, fr_c, fr_from_mont_limbs, g1_from_abi,
                    g1_to_abi, g2_from_abi, g2_to_abi, u64p)
from .transcript import Transcript


@dataclass
class EvaluationClaim:
    """pcs/src/lib.rs:10-13"""
    point: list
    evaluation: int


@dataclass
class KZGOpeningProof:
    """pcs/src/kzg.rs:25-32"""
    x: int
    y: int
    proof: object


def _opening_c(o: KZGOpeningProof) -> KzgOpening:
    c = KzgOpening()
    C.memmove(c.x, fr_c(o.x), 32)
    C.memmove(c.y, fr_c(o.y), 32)
    xy, inf = g1_to_abi(o.proof)
    C.memmove(c.proof_xy, xy, 64)
    c.proof_inf = inf
    return c


def _mle_proof_c(p: "MLEvalProof") -> MleProof:
    c = MleProof()
    C.memmove(c.evaluation, fr_c(p.evaluation), 32)
    xy, inf = g1_to_abi(p.s_comm)
    C.memmove(c.s_comm_xy, xy, 64)
    c.s_comm_inf = inf
    c.poly_opening = _opening_c(p.poly_opening)
    c.poly_opening_inv = _opening_c(p.poly_opening_inv)
    c.s_opening = _opening_c(p.s_opening)
    c.s_opening_inv = _opening_c(p.s_opening_inv)
    return c


# ---------------------------------------------------------------- pairing group G2
G1_GENERATOR = (1, 2)


def g2_generator():
    """ark-bn254 G2Affine::generator() as ((x0, x1), (y0, y1))"""
    xy = (C.c_uint64 * 16)()
    check(lib().qg_g2_generator(xy))
    return g2_from_abi(xy, 0)


def g2_mul(Q, k: int):
    xy, inf = g2_to_abi(Q)
    out, oinf = (C.c_uint64 * 16)(), C.c_uint8()
    check(lib().qg_g2_mul(xy, inf, fr_c(k), out, C.byref(oinf)))
    return g2_from_abi(out, oinf.value)


def pairing(P, Q):
    """E::pairing(P, Q) (ark-bn254 optimal ate) in the tower layout of
    qg_pairing: 12 canonical Fq ints (c0.c0.re, c0.c0.im, c0.c1.re, ...)"""
    pxy, pinf = g1_to_abi(P)
    qxy, qinf = g2_to_abi(Q)
    out = (C.c_uint64 * 48)()
    check(lib().qg_pairing(pxy, pinf, qxy, qinf, out))
    return [fq_from_mont_limbs(list(out)[4 * k:4 * k + 4]) for k in range(12)]


def _opening(o: KzgOpening) -> KZGOpeningProof:
    return KZGOpeningProof(fr_from_mont_limbs(list(o.x)), fr_from_mont_limbs(list(o.y)),
                           g1_from_abi(o.proof_xy, o.proof_inf))


@dataclass
class MLEvalProof:
    """pcs/src/mlpcs.rs:32-44"""
    evaluation_point: list
    evaluation: int
    s_comm: object
    poly_opening: KZGOpeningProof
    poly_opening_inv: KZGOpeningProof
    s_opening: KZGOpeningProof
    s_opening_inv: KZGOpeningProof

    def verify(self, commitment, kzg: "KZG", transcript: Transcript) -> bool:
        """mlpcs.rs:126-161 (host pairing check, qg_mle_verify)"""
        return kzg.verify(commitment, self, transcript)

    # MultilinearPCSProof (pcs/src/lib.rs:15-24)
    def point(self):
        return list(self.evaluation_point)

    def evaluation_claim(self):
        return EvaluationClaim(self.point(), self.evaluation)


class KZG:
    """KZG<Bn254> with a device-resident SRS.

    trusted_setup(max_degree, tau) builds g1_points = [tau^i] g on the device
    (kzg.rs:35-59 with an explicit tau instead of an rng; MultilinearPCS's
    thread_rng setup (mlpcs.rs:178-182) is not reproducible and is not offered)."""

    def __init__(self, dev: Device, srs: Srs, max_degree: int, tau: int = None, g=None,
                 g2_points=None):
        self.dev = dev
        self.srs = srs
        self._max_degree = max_degree
        self._tau, self._g = tau, g
        self._shards = {}
        # the verifier's part of the CRS (kzg.rs:14-22): g1, g2 = g2_points[0],
        # g2_points[1] = tau g2 (kzg.rs:52-53)
        self.g1 = g if g is not None else G1_GENERATOR
        if g2_points is None and tau is not None:
            g2 = g2_generator()
            g2_points = [g2, g2_mul(g2, tau)]
        self.g2_points = g2_points

    @classmethod
    def trusted_setup(cls, max_degree: int, tau: int, dev: Device = None, g=None):
        """With a communicator attached (dev.world > 1) the SRS is held as shards:
        a polynomial of global length L is split over the ranks (rank r owns
        entries [r L/world, (r+1) L/world)) and each rank keeps the matching
        slice [tau^(r L/world + i)] g of the bases, generated on first use per L."""
        dev = dev or Device(0)
        if dev.world > 1:
            return cls(dev, None, max_degree, tau, g)
        return cls(dev, Srs.generate(dev, tau, max_degree + 1, g), max_degree, tau, g)

    def srs_for(self, n_local: int) -> Srs:
        """the bases a local vector of n_local entries is committed against"""
        if self.dev.world == 1:
            return self.srs
        if self.srs is not None and len(self.srs) == n_local:
            return self.srs  # a caller-provided shard of this length
        L = n_local * self.dev.world
        if L > self._max_degree + 1:
            raise QuillGpuError(-1, "Polynomial degree exceeds max degree")
        if self._tau is None:
            raise QuillGpuError(-4, "sharded commitments need a generated (tau) SRS")
        if n_local not in self._shards:
            self._shards[n_local] = Srs.generate(self.dev, self._tau, n_local, self._g,
                                                 offset=self.dev.rank * n_local)
        return self._shards[n_local]

    def close(self):
        for s in [self.srs] + list(self._shards.values()):
            if s is not None:
                s.close()
        self._shards = {}

    @classmethod
    def from_points(cls, g1_points, dev: Device = None, g2_points=None):
        """an uploaded CRS; verification needs g2_points = [g2, tau g2] and
        takes g1 = g1_points[0]"""
        dev = dev or Device(0)
        return cls(dev, Srs.upload(dev, g1_points), len(g1_points) - 1, None, g1_points[0],
                   g2_points)

    @classmethod
    def verifier(cls, tau: int = None, g1=None, g2_points=None):
        """the verifier's view only (g1, g2_points; no device SRS): built from
        tau like trusted_setup, or from published points"""
        if tau is None and g2_points is None:
            raise QuillGpuError(-1, "verifier needs tau or g2_points")
        return cls(None, None, -1, tau, g1, g2_points)

    def _vk(self) -> KzgVk:
        if self.g2_points is None:
            raise QuillGpuError(-1, "no G2 points: verification needs g2 and tau g2")
        vk = KzgVk()
        xy, inf = g1_to_abi(self.g1)
        if inf:
            raise QuillGpuError(-1, "g1 generator is the identity")
        C.memmove(vk.g1_xy, xy, 64)
        for fld, Q in (("g2_xy", self.g2_points[0]), ("g2_tau_xy", self.g2_points[1])):
            qxy, qinf = g2_to_abi(Q)
            if qinf:
                raise QuillGpuError(-1, "G2 point is the identity")
            C.memmove(getattr(vk, fld), qxy, 128)
        return vk

    # KZG::verify (kzg.rs:98-108)
    def verify_univariate(self, commitment, opening: KZGOpeningProof) -> bool:
        xy, inf = g1_to_abi(commitment)
        ok = C.c_int()
        check(lib().qg_kzg_verify(C.byref(self._vk()), xy, inf, C.byref(_opening_c(opening)),
                                  C.byref(ok)))
        return bool(ok.value)

    # MultilinearPCS::verify == MLEvalProof::verify (lib.rs:35-40, mlpcs.rs:126-161)
    def verify(self, commitment, proof: MLEvalProof, transcript: Transcript) -> bool:
        xy, inf = g1_to_abi(commitment)
        pt = proof.evaluation_point
        arr = fr_array(pt) if len(pt) else np.zeros((1, 4), dtype=np.uint64)
        ok = C.c_int()
        check(lib().qg_mle_verify(C.byref(self._vk()), xy, inf, u64p(arr), len(pt),
                                  C.byref(_mle_proof_c(proof)), transcript.c_state(),
                                  C.byref(ok)))
        return bool(ok.value)

    # MultilinearPCS::max_degree (lib.rs:32)
    def max_degree(self) -> int:
        return self._max_degree

    # KZG::commit (kzg.rs:61-73) == MultilinearPCS::commit (mlpcs.rs:187-189)
    def commit(self, poly):
        if len(poly) > self._max_degree + 1:
            raise QuillGpuError(-1, "Polynomial degree exceeds max degree")
        if isinstance(poly, DeviceVec):
            return self.srs_for(len(poly)).msm_dev(poly, len(poly))
        arr = fr_array(poly) if len(poly) else np.zeros((1, 4), dtype=np.uint64)
        xy = (C.c_uint64 * 8)()
        inf = C.c_uint8()
        check(lib().qg_kzg_commit(self.dev.h, self.srs.h, u64p(arr), len(poly), xy,
                                  C.byref(inf)), self.dev.h)
        return g1_from_abi(xy, inf.value)

    def commit_batch(self, polys) -> list:
        """[commit(p) for p in polys], device vectors of one SRS shard as one MSM
        batch (qg_msm_g1_dev_batch); the same points"""
        if (len(polys) < 2 or not all(isinstance(p, DeviceVec) for p in polys)
                or (self.dev.world > 1 and len({len(p) for p in polys}) != 1)
                or os.environ.get("QUILL_COMMIT_BATCH", "1") == "0"):  # A/B runs
            return [self.commit(p) for p in polys]
        for p in polys:
            if len(p) > self._max_degree + 1:
                raise QuillGpuError(-1, "Polynomial degree exceeds max degree")
        return self.srs_for(len(polys[0])).msm_dev_batch(polys)

    # KZG::open (kzg.rs:75-96)
    def open_univariate(self, poly, x: int) -> KZGOpeningProof:
        arr = fr_array(poly) if len(poly) else np.zeros((1, 4), dtype=np.uint64)
        out = KzgOpening()
        check(lib().qg_kzg_open(self.dev.h, self.srs.h, u64p(arr), len(poly), fr_c(x),
                                C.byref(out)), self.dev.h)
        return _opening(out)

    # MultilinearPCS::open == MLEvalProof::prove (mlpcs.rs:83-124, 191-198)
    def open_dev(self, vec, n, eval_point, transcript: Transcript,
                 unchanged: bool = False) -> MLEvalProof:
        """open() on the first n entries of a device-resident DeviceVec.
        unchanged=True: vec has not changed since an earlier open of it on this
        device (qg_mle_open_dev_ex QG_OPEN_UNCHANGED: its transform is reused)"""
        pt = fr_array(eval_point) if len(eval_point) else np.zeros((1, 4), dtype=np.uint64)
        out = MleProof()
        check(lib().qg_mle_open_dev_ex(self.dev.h, self.srs_for(n).h, vec.h, n, u64p(pt),
                                       len(eval_point), transcript.c_state(),
                                       1 if unchanged else 0, C.byref(out)), self.dev.h)
        return MLEvalProof(list(eval_point), fr_from_mont_limbs(list(out.evaluation)),
                           g1_from_abi(out.s_comm_xy, out.s_comm_inf),
                           _opening(out.poly_opening), _opening(out.poly_opening_inv),
                           _opening(out.s_opening), _opening(out.s_opening_inv))

    def open_batch_dev(self, items, transcript: Transcript) -> list:
        """K openings [(vec, n, eval_point, unchanged), ...] in one call
        (qg_mle_open_batch_dev): the same proofs and transcript as K successive
        open_dev calls, with the S and quotient commitments as two MSM batches.
        Sharded devices batch each run of consecutive items of one local length
        (they commit against one SRS shard; mle_open_batch_sharded): the runs
        keep the item order, so the transcript is the same."""
        if len(items) <= 1:
            return [self.open_dev(v, n, pt, transcript, unch) for v, n, pt, unch in items]
        if self.dev.world > 1:
            out, i = [], 0
            while i < len(items):
                j = i
                while j < len(items) and items[j][1] == items[i][1]:
                    j += 1
                out += self._open_batch(items[i:j], transcript, self.srs_for(items[i][1]))
                i = j
            return out
        return self._open_batch(items, transcript, self.srs)

    def _open_batch(self, items, transcript: Transcript, srs) -> list:
        if len(items) == 1:
            v, n, pt, unch = items[0]
            return [self.open_dev(v, n, pt, transcript, unch)]
        k = len(items)
        arr = (MleOpenItem * k)()
        pts = []
        for i, (vec, n, pt, unch) in enumerate(items):
            a = fr_array(pt) if len(pt) else np.zeros((1, 4), dtype=np.uint64)
            pts.append(a)  # kept alive through the call
            arr[i] = MleOpenItem(vec.h.value, n, a.ctypes.data_as(C.POINTER(C.c_uint64)), len(pt),
                                 1 if unch else 0, 0)
        outs = (MleProof * k)()
        check(lib().qg_mle_open_batch_dev(self.dev.h, srs.h, arr, k, transcript.c_state(),
                                          outs), self.dev.h)
        return [MLEvalProof(list(pt), fr_from_mont_limbs(list(o.evaluation)),
                            g1_from_abi(o.s_comm_xy, o.s_comm_inf),
                            _opening(o.poly_opening), _opening(o.poly_opening_inv),
                            _opening(o.s_opening), _opening(o.s_opening_inv))
                for (_, _, pt, _), o in zip(items, outs)]

    def open(self, poly, eval_point, transcript: Transcript,
             unchanged: bool = False) -> MLEvalProof:
        if isinstance(poly, DeviceVec):
            return self.open_dev(poly, len(poly), eval_point, transcript, unchanged)
        arr = fr_array(poly) if len(poly) else np.zeros((1, 4), dtype=np.uint64)
        pt = fr_array(eval_point) if len(eval_point) else np.zeros((1, 4), dtype=np.uint64)
        out = MleProof()
        check(lib().qg_mle_open(self.dev.h, self.srs.h, u64p(arr), len(poly), u64p(pt),
                                len(eval_point), transcript.c_state(), C.byref(out)), self.dev.h)
        return MLEvalProof(list(eval_point), fr_from_mont_limbs(list(out.evaluation)),
                           g1_from_abi(out.s_comm_xy, out.s_comm_inf),
                           _opening(out.poly_opening), _opening(out.poly_opening_inv),
                           _opening(out.s_opening), _opening(out.s_opening_inv))
