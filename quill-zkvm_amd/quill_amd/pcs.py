"""PCS mirror: KZG (pcs/src/kzg.rs), MLEvalProof (pcs/src/mlpcs.rs) and the
MultilinearPCS trait surface (pcs/src/lib.rs:26-41), backed by the gfx950
kernels through the C-ABI.  Field elements are canonical Python ints; G1 points
are affine (x, y) tuples or None (infinity)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ._lib import KzgOpening, MleProof, QuillGpuError, check, lib
from .device import Device, DeviceVec, Srs
from .field import fr_array, fr_c, fr_from_mont_limbs, g1_from_abi, u64p
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

    def __init__(self, dev: Device, srs: Srs, max_degree: int, tau: int = None, g=None):
        self.dev = dev
        self.srs = srs
        self._max_degree = max_degree
        self._tau, self._g = tau, g
        self._shards = {}

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
    def from_points(cls, g1_points, dev: Device = None):
        dev = dev or Device(0)
        return cls(dev, Srs.upload(dev, g1_points), len(g1_points) - 1)

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

    # KZG::open (kzg.rs:75-96)
    def open_univariate(self, poly, x: int) -> KZGOpeningProof:
        arr = fr_array(poly) if len(poly) else np.zeros((1, 4), dtype=np.uint64)
        out = KzgOpening()
        check(lib().qg_kzg_open(self.dev.h, self.srs.h, u64p(arr), len(poly), fr_c(x),
                                C.byref(out)), self.dev.h)
        return _opening(out)

    # MultilinearPCS::open == MLEvalProof::prove (mlpcs.rs:83-124, 191-198)
    def open_dev(self, vec, n, eval_point, transcript: Transcript) -> MLEvalProof:
        """open() on the first n entries of a device-resident DeviceVec"""
        pt = fr_array(eval_point) if len(eval_point) else np.zeros((1, 4), dtype=np.uint64)
        out = MleProof()
        check(lib().qg_mle_open_dev(self.dev.h, self.srs_for(n).h, vec.h, n, u64p(pt),
                                    len(eval_point),
                                    transcript.c_state(), C.byref(out)), self.dev.h)
        return MLEvalProof(list(eval_point), fr_from_mont_limbs(list(out.evaluation)),
                           g1_from_abi(out.s_comm_xy, out.s_comm_inf),
                           _opening(out.poly_opening), _opening(out.poly_opening_inv),
                           _opening(out.s_opening), _opening(out.s_opening_inv))

    def open(self, poly, eval_point, transcript: Transcript) -> MLEvalProof:
        if isinstance(poly, DeviceVec):
            return self.open_dev(poly, len(poly), eval_point, transcript)
        arr = fr_array(poly) if len(poly) else np.zeros((1, 4), dtype=np.uint64)
        pt = fr_array(eval_point) if len(eval_point) else np.zeros((1, 4), dtype=np.uint64)
        out = MleProof()
        check(lib().qg_mle_open(self.dev.h, self.srs.h, u64p(arr), len(poly), u64p(pt),
                                len(eval_point), transcript.c_state(), C.byref(out)), self.dev.h)
        return MLEvalProof(list(eval_point), fr_from_mont_limbs(list(out.evaluation)),
                           g1_from_abi(out.s_comm_xy, out.s_comm_inf),
                           _opening(out.poly_opening), _opening(out.poly_opening_inv),
                           _opening(out.s_opening), _opening(out.s_opening_inv))
