"""HyperPlonk prover mirror (hyperplonk/src/proof/proof.rs:12-302) on device-resident
traces.

Every table lives in HBM for the whole proof: the full witness of a trace is
ONE device vector (column-major, index col * rows + row, proof.rs:270) and the
zero-check store's witness columns are views into it, so nothing is copied or
re-uploaded between the zero-check, the permutation check and the openings.
The transcript is the only host-side state; each step is one C-ABI call
(MSM, Logup column, eq table, sumcheck, ML-PCS opening) on the trace's
device vectors.  The verifier (proof.rs:303-522) runs on the host: field
arithmetic on Python ints, the transcript and the KZG pairing checks through
the C-ABI (qg_mle_verify)."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from ._lib import check, lib
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


def _verify_opening(comm, proof: MLEvalProof, expected_point, expected_nv, pcs,
                    transcript: Transcript) -> bool:
    """proof.rs:304-323"""
    if len(proof.point()) != expected_nv:
        return False
    if expected_point is not None and proof.point() != list(expected_point):
        return False
    return pcs.verify(comm, proof, transcript)


def _verify_trace_proof(witness_commitment, vk: "TraceVK", pcs, proof: TraceProof,
                        transcript: Transcript):
    """proof.rs:396-492 (with get_and_verify_column_evaluations :325-381 and
    recover_zerocheck_expr_evaluation :383-394); raises ValueError"""
    alpha = transcript.draw_field_element()
    zclaim = proof.zero_check_proof.verify(transcript)
    circuit = vk.circuit
    log2_cols, log2_rows = _log2(circuit.num_cols()), _log2(circuit.num_rows())
    if len(zclaim.point) != log2_rows:
        raise ValueError("Zero check evaluation claim point length mismatch")
    pt_claim = proof.opening_permutation_trace.evaluation_claim()
    proof.permutation_check_proof.verify(transcript, pcs, pt_claim, pt_claim,
                                         proof.opening_id.evaluation_claim(),
                                         proof.opening_permutation.evaluation_claim())
    # column evaluations
    points = [list(zclaim.point) + [(col >> i) & 1 for i in range(log2_cols)]
              for col in range(circuit.num_cols())]
    evals = []
    for i, op in enumerate(proof.openings_zero_check):
        if i >= len(points) or op.point() != points[i]:
            raise ValueError("Zero check opening point mismatch")
        if not pcs.verify(witness_commitment, op, transcript):
            raise ValueError("Zero check opening verification failed")
        evals.append(op.evaluation)
    for i, op in enumerate(proof.openings_public):
        if not _verify_opening(vk.public_columns_commitments[i], op, zclaim.point, log2_rows, pcs,
                               transcript):
            raise ValueError("Public opening verification failed")
        evals.append(op.evaluation)
    acc = 0
    for i, e in enumerate(circuit.zero_check_expressions()):
        acc = (acc + pow(alpha, i, R_MOD) * e.evaluate(evals)) % R_MOD
    if acc != zclaim.evaluation % R_MOD:
        raise ValueError("Zero check evaluation mismatch")
    nv = log2_rows + log2_cols
    if not _verify_opening(vk.id_commitment, proof.opening_id, None, nv, pcs, transcript):
        raise ValueError("ID commitment opening verification failed")
    if not _verify_opening(vk.permutation_commitment, proof.opening_permutation, None, nv, pcs,
                           transcript):
        raise ValueError("Permutation commitment opening verification failed")
    if not _verify_opening(witness_commitment, proof.opening_permutation_trace, None, nv, pcs,
                           transcript):
        raise ValueError("Permutation trace commitment opening verification failed")


def _hyperplonk_verify(self, vk, pcs) -> Transcript:
    """proof.rs:494-521: raises ValueError on rejection; returns the final
    transcript (equal to the prover's when the proof verifies)"""
    t = Transcript(b"hyperplonk_proof")
    for c in self.witness_commitment:
        t.append_g1(c)
    vks = vk.trace_vks if hasattr(vk, "trace_vks") else list(vk)
    if len(vks) != len(self.trace_proofs):
        raise ValueError("Number of trace VKS and proofs mismatch")
    for c, tvk, tp in zip(self.witness_commitment, vks, self.trace_proofs):
        _verify_trace_proof(c, tvk, pcs, tp, t)
    return t


HyperPlonkProof.verify = _hyperplonk_verify


@dataclass
class TraceVK:
    """proof.rs:32-37"""
    circuit: TransitionCircuit
    public_columns_commitments: list
    id_commitment: object
    permutation_commitment: object


@dataclass
class TracePK:
    """proof.rs:50-54 (device vectors of 2^trace_num_vars entries, or this
    rank's blocks of them).  `public_rows`: the unpadded public columns
    (circuit.public_values(), num_rows entries or this rank's row block) that
    the zero-check store and the public openings use."""
    id_poly: DeviceVec
    permutation_poly: DeviceVec
    public_values: list = field(default_factory=list)
    public_rows: list = field(default_factory=list)


class TraceWitness:
    """proof.rs:60: the trace's columns.  Host columns (all num_rows entries):
    (rows, 4) uint64 numpy arrays of canonical limbs or lists of ints.  Device
    columns: DeviceVec of num_rows entries, or with a communicator attached
    this rank's row block (rows / world entries) of each column."""

    def __init__(self, columns):
        self.columns = list(columns)
        self.full = None

    @classmethod
    def from_full(cls, full: DeviceVec, num_cols: int) -> "TraceWitness":
        """A single-GPU trace already resident in HBM as its full witness
        (column-major, num_cols x rows): proving reads it in place."""
        rows = full.n // num_cols
        tw = cls([full.view(c * rows, rows) for c in range(num_cols)])
        tw.full = full
        return tw

    def __len__(self):
        return len(self.columns)

    def to_device(self, dev: Device, rows: int):
        """-> (column blocks, full-witness block, owned buffers).  The full
        witness (proof.rs:270) is the column-major concatenation; sharded, each
        rank holds the row block of every column (zero-check) and its block of
        the flattening (permutation check, openings), exchanged by one
        all-to-all (qg_trace_full_witness)."""
        from .field import fr_canonical_array
        ncols = len(self.columns)
        if self.full is not None:
            assert dev.world == 1 and self.full.n == rows * ncols, "Padded witness length mismatch"
            return self.columns, self.full, []
        owned = []
        RL = rows // dev.world
        lo = dev.rank * RL
        if all(isinstance(c, DeviceVec) for c in self.columns):
            cols = self.columns
            for col in cols:
                assert len(col) == RL, "Witness column row length mismatch"
        else:
            store = DeviceVec(dev, RL * ncols)
            owned.append(store)
            cols = [store.view(c * RL, RL) for c in range(ncols)]
            for c, col in enumerate(self.columns):
                assert len(col) == rows, "Witness column row length mismatch"
                if isinstance(col, DeviceVec):
                    cols[c].copy_from(col, 0, lo if col.n == rows else 0, RL)
                else:
                    arr = col if isinstance(col, np.ndarray) else fr_canonical_array(col[lo:lo + RL])
                    if isinstance(col, np.ndarray):
                        arr = arr[lo:lo + RL]
                    DeviceVec.from_canonical(dev, arr, out=store, offset=c * RL)
        if dev.world == 1 and owned:
            return cols, owned[0], owned  # the column store IS the flattening
        full = DeviceVec(dev, rows * ncols // dev.world)
        owned.append(full)
        ptrs = (C.c_void_p * ncols)(*[c.h for c in cols])
        check(lib().qg_trace_full_witness(dev.h, ptrs, ncols, rows, full.h), dev.h)
        return cols, full, owned


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
        dev = pcs.dev
        if dev.world == 1:
            pub = circuit.public_values_dev(dev, N)  # padded with zeros (:76-85)
            pub_rows = [p.view(0, rows) for p in pub]
            pub_comms = [pcs.commit(p) for p in pub]
        else:
            # sharded: only the unpadded row blocks are kept; the commitment of
            # the zero-padded column is the same group element (zeros add nothing)
            pub = []
            pub_rows = circuit.public_values_dev(dev, rows)
            pub_comms = [pcs.commit(p) for p in pub_rows]
        ids, perm = circuit.permutation_u64()
        assert len(ids) == N, "ID polynomial length mismatch"
        assert len(perm) == N, "Permutation polynomial length mismatch"
        B = N // dev.world
        sl = slice(dev.rank * B, (dev.rank + 1) * B)
        id_dev = DeviceVec.from_u64(dev, ids[sl])
        perm_dev = DeviceVec.from_u64(dev, perm[sl])
        vk = TraceVK(circuit, pub_comms, pcs.commit(id_dev), pcs.commit(perm_dev))
        return TracePK(id_dev, perm_dev, pub, pub_rows), vk

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

    def prove_trace(self, pcs: KZG, columns, full: DeviceVec, transcript: Transcript,
                    pk: TracePK, circuit: TransitionCircuit) -> TraceProof:
        """proof.rs:145-237 (`columns`: the witness columns on the device, or
        this rank's row blocks; `full`: the full witness or this rank's block)"""
        dev = pcs.dev
        rows, cols = circuit.num_rows(), circuit.num_cols()
        log2_rows, log2_cols = _log2(rows), _log2(cols)
        store = VirtualPolynomialStore(log2_rows, dev)
        for c in range(cols):
            store.allocate_polynomial(columns[c])
        for p in pk.public_rows:  # circuit.public_values()
            store.allocate_polynomial(p)
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

        # `full` stays unchanged through these openings: its NTT transform is
        # computed once (unchanged=True, qg_mle_open_dev_ex), proofs identical.
        # They run as one batch (qg_mle_open_batch_dev: the same proofs and
        # transcript, the S and quotient commitments as two MSM batches; on a
        # sharded context four exchanges per trace instead of ~11 per opening);
        # QUILL_OPEN_BATCH=0 opens one by one.
        items = []
        for col in range(cols):
            point = list(zclaim.point) + [(col >> i) & 1 for i in range(log2_cols)]
            items.append((full, point, col > 0))
        items += [(p, list(zclaim.point), False) for p in pk.public_rows]
        items += [(pk.id_poly, list(ppoint), False), (pk.permutation_poly, list(ppoint), False),
                  (full, list(ppoint), True)]
        batch = (os.environ.get("QUILL_OPEN_BATCH", "1") != "0" and dev is not None
                 and all(isinstance(v, DeviceVec) for v, _, _ in items))
        if batch:
            opens = pcs.open_batch_dev([(v, len(v), pt, u) for v, pt, u in items], transcript)
        else:
            opens = [pcs.open(v, pt, transcript, unchanged=u) for v, pt, u in items]
        npub = len(pk.public_rows)
        open_zc = opens[:cols]
        open_pub = opens[cols:cols + npub]
        o_id, o_perm, o_pt = opens[cols + npub:]
        for p in store.polynomials[cols + len(pk.public_rows):]:
            p.close()  # eq table (zero-check)
        for p in store2.polynomials[3:]:
            p.close()  # Logup columns + eq table (permutation check)
        return TraceProof(zproof, pproof, open_zc, open_pub, o_id, o_perm, o_pt)

    def prove(self, pcs: KZG, witness_traces, transcript: Transcript = None,
              check_constraints: bool = True) -> HyperPlonkProof:
        """proof.rs:239-301.  `witness_traces`: TraceWitness (or column lists),
        one per circuit."""
        t = transcript if transcript is not None else Transcript(b"hyperplonk_proof")
        comms, layouts, owned = [], [], []
        for tw, vk in zip(witness_traces, self.trace_vks):
            tw = tw if isinstance(tw, TraceWitness) else TraceWitness(tw)
            circuit = vk.circuit
            assert len(tw) == circuit.num_cols(), "Witness columns length mismatch"
            cols, full, own = tw.to_device(pcs.dev, circuit.num_rows())
            owned += own
            if check_constraints:
                circuit.check_constraints(cols)
            layouts.append((cols, full))
        # the witness commitments (proof.rs:252-262) as one MSM batch, absorbed in
        # trace order: the same transcript as committing one by one
        comms = pcs.commit_batch([full for _, full in layouts])
        for Cm in comms:
            t.append_g1(Cm)
        proofs = []
        for (cols, full), vk, pk in zip(layouts, self.trace_vks, self.trace_pks):
            proofs.append(self.prove_trace(pcs, cols, full, t, pk, vk.circuit))
        for b in owned:
            b.close()  # built here; caller-resident traces stay
        self.last_transcript = t
        return HyperPlonkProof(comms, proofs)
