"""CPU restatement of the HyperPlonk prover/verifier and the transition-circuit
frontend — TEST INFRASTRUCTURE ONLY (see quill_oracle.py's header: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
use this module, as the checker).

Follows
  * hyperplonk/src/frontend/transition_circuit.rs:5-205  (TransitionCircuit)
  * hyperplonk/src/proof/circuit.rs:6-59                 (Circuit trait)
  * hyperplonk/src/proof/proof.rs:12-523                 (HyperPlonk prove / verify)
on top of quill_oracle's zero-check, permutation check and multilinear PCS.

Pinning: the reference's own end-to-end tests (hyperplonk/tests/
test_basic_proof.rs:17-196) only assert prove -> verify acceptance; the
restatement reproduces them (tests/test_oracle_hyperplonk.py), plus rejection of
tampered proofs and of unsatisfying witnesses.  Proof *bytes* inherit
quill_oracle's "transcript bytes parity-unpinned" status.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from quill_oracle import (KZG, R_MOD, Expr, MLEvalProof, MultisetEqualityProof, Transcript,
                          VirtualPolynomialStore, ZeroCheckProof, permutation_check_prove,
                          permutation_check_verify)


def next_power_of_two(n: int) -> int:
    """usize::next_power_of_two (0 -> 1)."""
    p = 1
    while p < n:
        p <<= 1
    return p


# ---------------------------------------------------------------------------
# frontend/transition_circuit.rs
# ---------------------------------------------------------------------------
class TransitionCircuit:
    """transition_circuit.rs:25-76.  Targets are plain column indices
    (TransitionCircuitTarget { col }); a state cell is (current, next)."""

    def __init__(self, num_rows: int):
        self.num_columns = 0
        self.num_rows_ = num_rows
        self.state_cells = []
        self.initial_state_values = []
        self.recurring_constraints = []
        self.boundary_constraints = []

    def allocate_witness_cell(self) -> int:
        idx = self.num_columns
        self.num_columns += 1
        return idx

    def allocate_state_cell(self):
        cur = self.allocate_witness_cell()
        nxt = self.allocate_witness_cell()
        self.state_cells.append((cur, nxt))
        return cur, nxt

    def enforce_constraint(self, c: Expr):
        self.recurring_constraints.append(c)

    def enforce_boundary_constraint(self, row: int, c: Expr):
        self.boundary_constraints.append((row, c))

    # Circuit impl (transition_circuit.rs:78-205)
    def num_rows(self) -> int:
        return self.num_rows_

    def num_cols(self) -> int:
        return next_power_of_two(self.num_columns)

    def num_public_columns(self) -> int:
        return len(self.boundary_constraints)

    def public_values(self):
        pub = [[0] * self.num_rows() for _ in range(self.num_public_columns())]
        for i, (row, _) in enumerate(self.boundary_constraints):
            pub[i][row] = 1
        return pub

    def zero_check_expressions(self):
        cs = list(self.recurring_constraints)
        pc = self.num_cols()
        for i, (_row, c) in enumerate(self.boundary_constraints):
            cs.append(Expr("mul", Expr.input(i + pc), c))
        return cs

    def permutation(self):
        """(id, permutation) index columns, +1 so no entry is zero (:120-151)."""
        rows = self.num_rows()
        ncells = rows * self.num_cols()
        perm = list(range(ncells))
        for cur, nxt in self.state_cells:
            for row in range(rows - 1):
                frm = nxt * rows + row
                to = cur * rows + row + 1
                perm[frm] = to
                perm[to] = frm
        return [i + 1 for i in range(ncells)], [p + 1 for p in perm]

    def check_constraints(self, witness):
        """:153-204 -> raises ValueError with the reference's message kind."""
        for row in range(self.num_rows()):
            vals = [col[row] for col in witness]
            for c in self.recurring_constraints:
                if c.evaluate(vals) != 0:
                    raise ValueError(f"Recurring constraint not satisfied at row {row}")
        for row, c in self.boundary_constraints:
            vals = [col[row] for col in witness]
            if c.evaluate(vals) != 0:
                raise ValueError(f"Boundary constraint not satisfied at row {row}")
        for cur, nxt in self.state_cells:
            for row in range(self.num_rows() - 1):
                if witness[nxt][row] % R_MOD != witness[cur][row + 1] % R_MOD:
                    raise ValueError(f"Permutation constraint not satisfied for state cell "
                                     f"at row {row}")


# ---------------------------------------------------------------------------
# proof/proof.rs
# ---------------------------------------------------------------------------
@dataclass
class TraceProof:
    """proof.rs:17-25"""
    zero_check_proof: ZeroCheckProof
    permutation_check_proof: MultisetEqualityProof  # PermutationCheckProof { multiset_equality_proof }
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
    """proof.rs:50-54"""
    id_poly: list
    permutation_poly: list
    public_values: list = field(default_factory=list)


def _log2(n: int) -> int:
    return n.bit_length() - 1


class HyperPlonk:
    """proof.rs:12-15, 62-302"""

    def __init__(self, trace_vks, trace_pks):
        self.trace_vks, self.trace_pks = trace_vks, trace_pks

    @staticmethod
    def preprocess_trace(circuit, pcs: KZG):
        """proof.rs:63-122"""
        rows, cols = circuit.num_rows(), circuit.num_cols()
        assert rows & (rows - 1) == 0, "Number of rows must be a power of two"
        assert cols & (cols - 1) == 0, "Number of columns must be a power of two"
        nv = _log2(rows) + _log2(cols)
        pub = circuit.public_values()
        for col in pub:
            assert len(col) == rows, "Public column length mismatch"
            col.extend([0] * ((1 << nv) - rows))
        pub_comms = [pcs.commit(c) for c in pub]
        ids, perm = circuit.permutation()
        assert len(ids) == 1 << nv, "ID polynomial length mismatch"
        assert len(perm) == 1 << nv, "Permutation polynomial length mismatch"
        vk = TraceVK(circuit, pub_comms, pcs.commit(ids), pcs.commit(perm))
        return TracePK(ids, perm, pub), vk

    @staticmethod
    def preprocess(circuits, pcs: KZG):
        """proof.rs:124-137"""
        pks, vks = [], []
        for c in circuits:
            pk, vk = HyperPlonk.preprocess_trace(c, pcs)
            pks.append(pk)
            vks.append(vk)
        return HyperPlonk(vks, pks)

    def prove_trace(self, pcs: KZG, witness, full_witness, t: Transcript, pk: TracePK, circuit):
        """proof.rs:145-237"""
        log2_rows, log2_cols = _log2(circuit.num_rows()), _log2(circuit.num_cols())
        store = VirtualPolynomialStore(log2_rows)
        for col in witness:
            store.allocate_polynomial(col)
        for pub in circuit.public_values():
            store.allocate_polynomial(pub)
        exprs = circuit.zero_check_expressions()
        alpha = t.draw_field_element()
        zc = Expr.const(0)
        for i, e in enumerate(exprs):
            zc = zc + Expr.const(pow(alpha, i, R_MOD)) * e
        zv = store.new_virtual_from_expr(zc)
        zproof, (zpoint, _zev) = ZeroCheckProof.prove(store, zv, t)

        store2 = VirtualPolynomialStore(log2_rows + log2_cols)
        widx = store2.allocate_polynomial(full_witness)
        wv = store2.new_virtual_from_input(widx)
        pproof, ppoint = permutation_check_prove(store2, wv, wv, pk.id_poly, pk.permutation_poly,
                                                 t, pcs)

        open_zc = []
        for col in range(circuit.num_cols()):
            point = list(zpoint) + [(col >> i) & 1 for i in range(log2_cols)]
            open_zc.append(MLEvalProof.prove(full_witness, point, pcs, t))
        open_pub = [MLEvalProof.prove(p, zpoint, pcs, t) for p in circuit.public_values()]
        o_id = MLEvalProof.prove(pk.id_poly, ppoint, pcs, t)
        o_perm = MLEvalProof.prove(pk.permutation_poly, ppoint, pcs, t)
        o_pt = MLEvalProof.prove(full_witness, ppoint, pcs, t)
        return TraceProof(zproof, pproof, open_zc, open_pub, o_id, o_perm, o_pt)

    def prove(self, pcs: KZG, witness_traces):
        """proof.rs:239-301; witness_traces = list of column lists."""
        t = Transcript(b"hyperplonk_proof")
        comms, fulls = [], []
        for witness, vk in zip(witness_traces, self.trace_vks):
            circuit = vk.circuit
            assert len(witness) == circuit.num_cols(), "Witness columns length mismatch"
            for col in witness:
                assert len(col) == circuit.num_rows(), "Witness column row length mismatch"
            circuit.check_constraints(witness)
            full = [v % R_MOD for col in witness for v in col]
            C = pcs.commit(full)
            t.append_g1(C)
            comms.append(C)
            fulls.append(full)
        proofs = []
        for i, witness in enumerate(witness_traces):
            proofs.append(self.prove_trace(pcs, witness, fulls[i], t, self.trace_pks[i],
                                           self.trace_vks[i].circuit))
        return HyperPlonkProof(comms, proofs), t

    def to_vk(self):
        return list(self.trace_vks)


def _verify_opening(comm, proof: MLEvalProof, expected_point, expected_nv, pcs, t) -> bool:
    """proof.rs:305-325"""
    if len(proof.evaluation_point) != expected_nv:
        return False
    if expected_point is not None and list(proof.evaluation_point) != list(expected_point):
        return False
    return proof.verify(comm, pcs, t)


def verify_trace_proof(witness_commitment, vk: TraceVK, pcs: KZG, proof: TraceProof,
                       t: Transcript):
    """proof.rs:404-491 (raises ValueError with the reference's messages)."""
    alpha = t.draw_field_element()
    zpoint, zev = proof.zero_check_proof.verify(t)
    circuit = vk.circuit
    log2_cols, log2_rows = _log2(circuit.num_cols()), _log2(circuit.num_rows())
    if len(zpoint) != log2_rows:
        raise ValueError("Zero check evaluation claim point length mismatch")
    oi, op, opt = proof.opening_id, proof.opening_permutation, proof.opening_permutation_trace
    permutation_check_verify(proof.permutation_check_proof, t, pcs,
                             (opt.evaluation_point, opt.evaluation),
                             (opt.evaluation_point, opt.evaluation),
                             (oi.evaluation_point, oi.evaluation),
                             (op.evaluation_point, op.evaluation))
    # get_and_verify_column_evaluations (proof.rs:330-385)
    col_evals = []
    for col, o in enumerate(proof.openings_zero_check):
        point = list(zpoint) + [(col >> i) & 1 for i in range(log2_cols)]
        if list(o.evaluation_point) != point:
            raise ValueError("Zero check opening point mismatch")
        if not o.verify(witness_commitment, pcs, t):
            raise ValueError("Zero check opening verification failed")
        col_evals.append(o.evaluation)
    for i, o in enumerate(proof.openings_public):
        if not _verify_opening(vk.public_columns_commitments[i], o, zpoint, log2_rows, pcs, t):
            raise ValueError("Public opening verification failed")
        col_evals.append(o.evaluation)
    # recover_zerocheck_expr_evaluation (proof.rs:387-402)
    acc = 0
    for i, e in enumerate(circuit.zero_check_expressions()):
        acc += pow(alpha, i, R_MOD) * e.evaluate(col_evals)
    if acc % R_MOD != zev % R_MOD:
        raise ValueError("Zero check evaluation mismatch")
    nv = log2_rows + log2_cols
    if not _verify_opening(vk.id_commitment, oi, None, nv, pcs, t):
        raise ValueError("ID commitment opening verification failed")
    if not _verify_opening(vk.permutation_commitment, op, None, nv, pcs, t):
        raise ValueError("Permutation commitment opening verification failed")
    if not _verify_opening(witness_commitment, opt, None, nv, pcs, t):
        raise ValueError("Permutation trace commitment opening verification failed")


def hyperplonk_verify(proof: HyperPlonkProof, trace_vks, pcs: KZG) -> Transcript:
    """HyperPlonkProof::verify (proof.rs:493-522); returns the final transcript."""
    t = Transcript(b"hyperplonk_proof")
    for C in proof.witness_commitment:
        t.append_g1(C)
    if len(trace_vks) != len(proof.trace_proofs):
        raise ValueError("Number of trace VKS and proofs mismatch")
    for C, vk, tp in zip(proof.witness_commitment, trace_vks, proof.trace_proofs):
        verify_trace_proof(C, vk, pcs, tp, t)
    return t


# ---------------------------------------------------------------------------
# the reference's test circuits (hyperplonk/tests/test_basic_proof.rs:17-105)
# ---------------------------------------------------------------------------
def fibonacci_circuit_and_trace(num_rows: int = 8):
    """test_basic_proof.rs:17-52 (num_rows = 8 there)."""
    c = TransitionCircuit(num_rows)
    s1 = c.allocate_state_cell()
    s2 = c.allocate_state_cell()
    c.enforce_boundary_constraint(0, Expr.input(s1[0]))
    c.enforce_boundary_constraint(0, Expr.input(s2[0]) - Expr.const(1))
    c.enforce_constraint(Expr.input(s2[1]) - (Expr.input(s1[0]) + Expr.input(s2[0])))
    c.enforce_constraint(Expr.input(s1[1]) - Expr.input(s2[0]))
    w = [[0] * num_rows for _ in range(c.num_cols())]
    for row in range(num_rows):
        if row == 0:
            w[s1[0]][0], w[s2[0]][0], w[s1[1]][0], w[s2[1]][0] = 0, 1, 1, 1
        else:
            w[s1[0]][row] = w[s1[1]][row - 1]
            w[s2[0]][row] = w[s2[1]][row - 1]
            w[s1[1]][row] = w[s2[0]][row]
            w[s2[1]][row] = (w[s2[0]][row] + w[s1[0]][row]) % R_MOD
    return c, w


def modified_fibonacci_circuit_and_trace(num_rows: int = 8):
    """test_basic_proof.rs:54-105: f(n) = f(n-1) + f(n-1) f(n-2)."""
    c = TransitionCircuit(num_rows)
    s1 = c.allocate_state_cell()
    s2 = c.allocate_state_cell()
    tmp = c.allocate_witness_cell()
    c.enforce_boundary_constraint(0, Expr.input(s1[0]) - Expr.const(1))
    c.enforce_boundary_constraint(0, Expr.input(s2[0]) - Expr.const(1))
    c.enforce_constraint(Expr.input(tmp) - Expr.input(s1[0]) * Expr.input(s2[0]))
    c.enforce_constraint(Expr.input(s2[1]) - (Expr.input(s1[0]) + Expr.input(tmp)))
    c.enforce_constraint(Expr.input(s1[1]) - Expr.input(s2[0]))
    w = [[0] * num_rows for _ in range(c.num_cols())]
    for row in range(num_rows):
        if row == 0:
            w[s1[0]][0], w[s2[0]][0] = 1, 1
        else:
            w[s1[0]][row] = w[s1[1]][row - 1]
            w[s2[0]][row] = w[s2[1]][row - 1]
        w[s1[1]][row] = w[s2[0]][row]
        w[tmp][row] = w[s1[0]][row] * w[s2[0]][row] % R_MOD
        w[s2[1]][row] = (w[s1[0]][row] + w[tmp][row]) % R_MOD
    return c, w
