"""HyperPlonk prover mirror (hyperplonk/src/proof/proof.rs:12-302) on device-resident
traces.

Every table lives in HBM for the whole proof: the full witness of a trace is
ONE device vector (column-major, index col * rows + row, proof.rs:270) and the
zero-check store's witness columns are views into it, so nothing is copied or
re-uploaded between the zero-check, the permutation check and the openings.
The transcript is the only host-side state; each step is one C-ABI call
(MSM, Logup column, eq table, sumcheck, ML-PCS opening) on the trace's
device vectors.  The verifier is not mirrored (CPU-only in the reference's
model; the oracle's restatement checks these proofs in tests)."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .device import Device, DeviceVec
from .field import R_MOD
from .frontend import TransitionCircuit
from .hyperplonk import VirtualPolyExpr, VirtualPolynomialStore, ZeroCheckProof
from .logup import PermutationCheckProof
from .pcs import KZG, MLEvalProof
from .transcript import Transcript


@dataclass
class TraceProof:
    """proof.rs:17-25"""
    zero_check_proof: ZeroCheckProof
    permutation_check_proof: PermutationCheckProof
    openings_zero_check: list
    openings_public: list
    opening_id: MLEvalProof
    opening_permutation: MLEvalProof
    opening_permutation_trace: MLEvalProof


@dataclass
class HyperPlonkProof:
    """proof.rs:27-30"""
    witness_commitment: list
    trace_proofs: list


@dataclass
class TraceVK:
    """proof.rs:32-37"""
    circuit: TransitionCircuit
    public_columns_commitments: list
    id_commitment: object
    permutation_commitment: object


@dataclass
class TracePK:
    """proof.rs:50-54 (device vectors of 2^trace_num_vars entries)"""
    id_poly: DeviceVec
    permutation_poly: DeviceVec
    public_values: list = field(default_factory=list)


class TraceWitness:
    """proof.rs:60: the trace's columns.  Accepted column forms: DeviceVec,
    (rows, 4) uint64 numpy arrays of canonical limbs, or lists of ints."""

    def __init__(self, columns):
        self.columns = list(columns)
        self.full = None

    @classmethod
    def from_full(cls, full: DeviceVec, num_cols: int) -> "TraceWitness":
        """A trace already resident in HBM as its full witness (column-major,
        num_cols x rows): proving reads it in place."""
        rows = full.n // num_cols
        tw = cls([full.view(c * rows, rows) for c in range(num_cols)])
        tw.full = full
        return tw

    def __len__(self):
        return len(self.columns)

    def to_device(self, dev: Device, rows: int) -> DeviceVec:
        """full witness (proof.rs:270) as one device vector"""
        from .field import fr_canonical_array
        if self.full is not None:
            assert self.full.n == rows * len(self.columns), "Padded witness length mismatch"
            return self.full
        full = DeviceVec(dev, rows * len(self.columns))
        for c, col in enumerate(self.columns):
            assert len(col) == rows, "Witness column row length mismatch"
            if isinstance(col, DeviceVec):
                full.copy_from(col, c * rows, 0, rows)
            else:
                arr = col if isinstance(col, np.ndarray) else fr_canonical_array(col)
                DeviceVec.from_canonical(dev, arr, out=full, offset=c * rows)
        return full


def _log2(n: int) -> int:
    return n.bit_length() - 1


class HyperPlonk:
    """proof.rs:12-15"""

    def __init__(self, trace_vks, trace_pks):
        self.trace_vks, self.trace_pks = trace_vks, trace_pks

    @staticmethod
    def preprocess_trace(circuit: TransitionCircuit, pcs: KZG):
        """proof.rs:63-122"""
        rows, cols = circuit.num_rows(), circuit.num_cols()
        assert rows & (rows - 1) == 0, "Number of rows must be a power of two"
        assert cols & (cols - 1) == 0, "Number of columns must be a power of two"
        N = rows * cols
        pub = circuit.public_values_dev(pcs.dev, N)  # padded with zeros (:76-85)
        pub_comms = [pcs.commit(p) for p in pub]
        ids, perm = circuit.permutation_u64()
        assert len(ids) == N, "ID polynomial length mismatch"
        assert len(perm) == N, "Permutation polynomial length mismatch"
        id_dev = DeviceVec.from_u64(pcs.dev, ids)
        perm_dev = DeviceVec.from_u64(pcs.dev, perm)
        vk = TraceVK(circuit, pub_comms, pcs.commit(id_dev), pcs.commit(perm_dev))
        return TracePK(id_dev, perm_dev, pub), vk

    @staticmethod
    def preprocess(circuits, pcs: KZG) -> "HyperPlonk":
        """proof.rs:124-137"""
        pks, vks = [], []
        for c in circuits:
            pk, vk = HyperPlonk.preprocess_trace(c, pcs)
            pks.append(pk)
            vks.append(vk)
        return HyperPlonk(vks, pks)

    def to_vk(self):
        """proof.rs:139-143"""
        return list(self.trace_vks)

    def prove_trace(self, pcs: KZG, full: DeviceVec, transcript: Transcript, pk: TracePK,
                    circuit: TransitionCircuit) -> TraceProof:
        """proof.rs:145-237"""
        dev = pcs.dev
        rows, cols = circuit.num_rows(), circuit.num_cols()
        log2_rows, log2_cols = _log2(rows), _log2(cols)
        store = VirtualPolynomialStore(log2_rows, dev)
        for c in range(cols):
            store.allocate_polynomial(full.view(c * rows, rows))
        for p in pk.public_values:  # circuit.public_values(): the first `rows` entries
            store.allocate_polynomial(p.view(0, rows))
        exprs = circuit.zero_check_expressions()
        alpha = transcript.draw_field_element()
        E = VirtualPolyExpr
        zc = E.Const(0)
        for i, e in enumerate(exprs):
            zc = zc + E.Const(pow(alpha, i, R_MOD)) * e
        zv = store.new_virtual_from_expr(zc)
        zproof, zclaim = ZeroCheckProof.prove(store, zv, transcript)

        store2 = VirtualPolynomialStore(log2_rows + log2_cols, dev)
        widx = store2.allocate_polynomial(full)
        wv = store2.new_virtual_from_input(widx)
        pproof, ppoint = PermutationCheckProof.prove(store2, wv, wv, pk.id_poly,
                                                     pk.permutation_poly, transcript, pcs)

        open_zc = []
        for col in range(cols):
            point = list(zclaim.point) + [(col >> i) & 1 for i in range(log2_cols)]
            open_zc.append(pcs.open(full, point, transcript))
        open_pub = [pcs.open(p.view(0, rows), zclaim.point, transcript)
                    for p in pk.public_values]
        o_id = pcs.open(pk.id_poly, ppoint, transcript)
        o_perm = pcs.open(pk.permutation_poly, ppoint, transcript)
        o_pt = pcs.open(full, ppoint, transcript)
        for p in store.polynomials[cols + len(pk.public_values):]:
            p.close()  # eq table (zero-check)
        for p in store2.polynomials[3:]:
            p.close()  # Logup columns + eq table (permutation check)
        return TraceProof(zproof, pproof, open_zc, open_pub, o_id, o_perm, o_pt)

    def prove(self, pcs: KZG, witness_traces, transcript: Transcript = None,
              check_constraints: bool = True) -> HyperPlonkProof:
        """proof.rs:239-301.  `witness_traces`: TraceWitness (or column lists),
        one per circuit."""
        t = transcript if transcript is not None else Transcript(b"hyperplonk_proof")
        comms, fulls = [], []
        for tw, vk in zip(witness_traces, self.trace_vks):
            tw = tw if isinstance(tw, TraceWitness) else TraceWitness(tw)
            circuit = vk.circuit
            assert len(tw) == circuit.num_cols(), "Witness columns length mismatch"
            rows = circuit.num_rows()
            full = tw.to_device(pcs.dev, rows)
            if check_constraints:
                circuit.check_constraints([full.view(c * rows, rows)
                                           for c in range(circuit.num_cols())])
            C = pcs.commit(full)
            t.append_g1(C)
            comms.append(C)
            fulls.append(full)
        proofs = []
        for full, vk, pk in zip(fulls, self.trace_vks, self.trace_pks):
            proofs.append(self.prove_trace(pcs, full, t, pk, vk.circuit))
        for tw, full in zip(witness_traces, fulls):
            if not (isinstance(tw, TraceWitness) and tw.full is full):
                full.close()  # uploaded here; a caller-resident trace stays
        self.last_transcript = t
        return HyperPlonkProof(comms, proofs)
