"""Proof wire format: ark-serialize `CanonicalSerialize` (uncompressed,
little-endian) of the reference's proof structs, field by field in
declaration order — what `#[derive(CanonicalSerialize)]` on them would emit:

  Fr                 32 bytes, canonical LE
  G1 (Bn254)         x || y, 32 bytes each LE; y's top byte carries the flags
                     (bit 6: point at infinity, coordinates zero; bit 7: y is
                     the larger root) — the same bytes the transcript absorbs
                     (transcript.rs:33-37, qg_g1_serialize)
  usize              u64 LE
  Vec<T>             u64 LE length, then the items
  DensePolynomial    its `coeffs: Vec<Fr>`

Structs (field order of the reference):
  KZGOpeningProof        x, y, proof                      (kzg.rs:25-32)
  MLEvalProof            evaluation_point, evaluation, s_comm, poly_opening,
                         poly_opening_inv, s_opening, s_opening_inv (mlpcs.rs:32-44)
  SumcheckProof          num_vars, claimed_sum, r_polys   (sumcheck.rs:15-19)
  ZeroCheckProof         num_vars, sumcheck_proof         (zerocheck.rs:8-11)
  MultisetEqualityProof  denom_left_commitment, denom_right_commitment,
                         sumcheck_proof, opening_proof_denom_left,
                         opening_proof_denom_right        (multiset_check.rs:18-24)
  PermutationCheckProof  multiset_equality_proof          (permutation_check.rs:8-10)
  TraceProof             zero_check_proof, permutation_check_proof,
                         openings_zero_check, openings_public, opening_id,
                         opening_permutation, opening_permutation_trace (proof.rs:17-25)
  HyperPlonkProof        witness_commitment, trace_proofs (proof.rs:27-30)

Decoding validates like `CanonicalDeserialize` with `Validate::Yes`:
canonical field encodings, points on the curve (G1 has cofactor 1), no
trailing bytes; a malformed encoding raises ValueError."""
from __future__ import annotations

import struct

from .field import P_MOD, R_MOD
from .hyperplonk import SumcheckProof, ZeroCheckProof
from .logup import MultisetEqualityProof, PermutationCheckProof
from .pcs import KZGOpeningProof, MLEvalProof
from .proof import HyperPlonkProof, TraceProof

_INF, _NEG = 0x40, 0x80


# ---------------------------------------------------------------- writers
def _fr(x: int) -> bytes:
    return (int(x) % R_MOD).to_bytes(32, "little")


def _g1(pt) -> bytes:
    if pt is None:
        return bytes(63) + bytes([_INF])
    x, y = int(pt[0]) % P_MOD, int(pt[1]) % P_MOD
    b = bytearray(x.to_bytes(32, "little") + y.to_bytes(32, "little"))
    if y > P_MOD - y:
        b[63] |= _NEG
    return bytes(b)


def _u64(v: int) -> bytes:
    return struct.pack("<Q", int(v))


def _vec(items, enc) -> bytes:
    return _u64(len(items)) + b"".join(enc(i) for i in items)


def _poly(coeffs) -> bytes:
    return _vec(list(coeffs), _fr)


def _kzg_opening(o: KZGOpeningProof) -> bytes:
    return _fr(o.x) + _fr(o.y) + _g1(o.proof)


def _mle(p: MLEvalProof) -> bytes:
    return (_vec(list(p.evaluation_point), _fr) + _fr(p.evaluation) + _g1(p.s_comm)
            + _kzg_opening(p.poly_opening) + _kzg_opening(p.poly_opening_inv)
            + _kzg_opening(p.s_opening) + _kzg_opening(p.s_opening_inv))


def _sumcheck(p: SumcheckProof) -> bytes:
    return _u64(p.num_vars) + _fr(p.claimed_sum) + _vec(list(p.r_polys), _poly)


def _zerocheck(p: ZeroCheckProof) -> bytes:
    return _u64(p.num_vars) + _sumcheck(p.sumcheck_proof)


def _multiset(p: MultisetEqualityProof) -> bytes:
    return (_g1(p.denom_left_commitment) + _g1(p.denom_right_commitment)
            + _sumcheck(p.sumcheck_proof) + _mle(p.opening_proof_denom_left)
            + _mle(p.opening_proof_denom_right))


def _trace(p: TraceProof) -> bytes:
    return (_zerocheck(p.zero_check_proof)
            + _multiset(p.permutation_check_proof.multiset_equality_proof)
            + _vec(list(p.openings_zero_check), _mle) + _vec(list(p.openings_public), _mle)
            + _mle(p.opening_id) + _mle(p.opening_permutation) + _mle(p.opening_permutation_trace))


def _hyperplonk(p: HyperPlonkProof) -> bytes:
    return _vec(list(p.witness_commitment), _g1) + _vec(list(p.trace_proofs), _trace)


_ENCODERS = [(HyperPlonkProof, _hyperplonk), (TraceProof, _trace), (MLEvalProof, _mle),
             (SumcheckProof, _sumcheck), (ZeroCheckProof, _zerocheck),
             (MultisetEqualityProof, _multiset),
             (PermutationCheckProof, lambda p: _multiset(p.multiset_equality_proof)),
             (KZGOpeningProof, _kzg_opening)]


def serialize(obj) -> bytes:
    """CanonicalSerialize::serialize_uncompressed of a proof object"""
    for cls, enc in _ENCODERS:
        if isinstance(obj, cls):
            return enc(obj)
    raise TypeError(f"no wire format for {type(obj).__name__}")


# ---------------------------------------------------------------- readers
class _Reader:
    def __init__(self, b: bytes):
        self.b, self.o = memoryview(bytes(b)), 0

    def take(self, n: int) -> bytes:
        if self.o + n > len(self.b):
            raise ValueError("truncated proof encoding")
        out = bytes(self.b[self.o:self.o + n])
        self.o += n
        return out

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def fr(self) -> int:
        v = int.from_bytes(self.take(32), "little")
        if v >= R_MOD:
            raise ValueError("non-canonical field element")
        return v

    def g1(self):
        b = bytearray(self.take(64))
        flags = b[63] & 0xC0
        b[63] &= 0x3F
        x, y = int.from_bytes(b[:32], "little"), int.from_bytes(b[32:], "little")
        if flags & _INF:
            if x or y or flags & _NEG:
                raise ValueError("malformed point at infinity")
            return None
        if x >= P_MOD or y >= P_MOD:
            raise ValueError("non-canonical coordinate")
        if (y * y - x * x * x - 3) % P_MOD:
            raise ValueError("point not on the curve")
        if bool(flags & _NEG) != (y > P_MOD - y):
            raise ValueError("y-sign flag inconsistent with the point")
        return (x, y)

    def vec(self, dec):
        n = self.u64()
        if n > len(self.b) - self.o:  # every item takes at least one byte
            raise ValueError("vector length exceeds the encoding")
        return [dec() for _ in range(n)]

    def kzg_opening(self):
        return KZGOpeningProof(self.fr(), self.fr(), self.g1())

    def mle(self):
        pt = self.vec(self.fr)
        ev, s = self.fr(), self.g1()
        return MLEvalProof(pt, ev, s, self.kzg_opening(), self.kzg_opening(),
                           self.kzg_opening(), self.kzg_opening())

    def sumcheck(self):
        nv, cs = self.u64(), self.fr()
        return SumcheckProof(nv, cs, self.vec(lambda: self.vec(self.fr)))

    def zerocheck(self):
        nv = self.u64()
        return ZeroCheckProof(nv, self.sumcheck())

    def multiset(self):
        cl, cr = self.g1(), self.g1()
        sc = self.sumcheck()
        return MultisetEqualityProof(cl, cr, sc, self.mle(), self.mle())

    def trace(self):
        zc = self.zerocheck()
        pc = PermutationCheckProof(self.multiset())
        ozc, opub = self.vec(self.mle), self.vec(self.mle)
        return TraceProof(zc, pc, ozc, opub, self.mle(), self.mle(), self.mle())

    def hyperplonk(self):
        comms = self.vec(self.g1)
        return HyperPlonkProof(comms, self.vec(self.trace))


_DECODERS = {HyperPlonkProof: "hyperplonk", TraceProof: "trace", MLEvalProof: "mle",
             SumcheckProof: "sumcheck", ZeroCheckProof: "zerocheck",
             MultisetEqualityProof: "multiset", KZGOpeningProof: "kzg_opening"}


def deserialize(cls, data: bytes):
    """CanonicalDeserialize::deserialize_uncompressed (Validate::Yes)"""
    if cls is PermutationCheckProof:
        r = _Reader(data)
        out = PermutationCheckProof(r.multiset())
    else:
        if cls not in _DECODERS:
            raise TypeError(f"no wire format for {cls.__name__}")
        r = _Reader(data)
        out = getattr(r, _DECODERS[cls])()
    if r.o != len(r.b):
        raise ValueError("trailing bytes after the proof")
    return out
