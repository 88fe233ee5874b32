"""Transition-circuit frontend mirror (hyperplonk/src/frontend/transition_circuit.rs)
implementing the Circuit trait (hyperplonk/src/proof/circuit.rs:6-59).

Host-side circuit description only: the witness lives on the device, and the
per-row work of `check_constraints` (the reference's row loop at
transition_circuit.rs:153-204) runs as device kernels through the C-ABI
(qg_expr_first_nonzero_dev, qg_buf_first_mismatch).  The index columns of
`permutation()` and the selector columns of `public_values()` are built as
numpy arrays and converted on the device (F::from(u64)), so a 2^23-cell trace
never becomes a list of Python ints."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib
from .device import Device, DeviceVec
from .field import fr_from_mont_limbs
from .hyperplonk import VirtualPolyExpr, _program_c


def next_power_of_two(n: int) -> int:
    """usize::next_power_of_two (0 -> 1)"""
    p = 1
    while p < n:
        p <<= 1
    return p


class TransitionCircuitTarget:
    """transition_circuit.rs:5-15"""

    def __init__(self, col: int):
        self.col = col

    def to_expr(self) -> VirtualPolyExpr:
        return VirtualPolyExpr.Input(self.col)


class StateCell:
    """transition_circuit.rs:17-21"""

    def __init__(self, current: TransitionCircuitTarget, next_: TransitionCircuitTarget):
        self.current = current
        self.next = next_


class TransitionCircuit:
    """transition_circuit.rs:25-76 + the Circuit impl at :78-205"""

    def __init__(self, num_rows: int):
        self.num_columns = 0
        self._num_rows = num_rows
        self.state_cells = []
        self.initial_state_values = []
        self.recurring_constraints = []
        self.boundary_constraints = []

    def allocate_witness_cell(self) -> TransitionCircuitTarget:
        t = TransitionCircuitTarget(self.num_columns)
        self.num_columns += 1
        return t

    def allocate_state_cell(self) -> StateCell:
        cur = self.allocate_witness_cell()
        nxt = self.allocate_witness_cell()
        sc = StateCell(cur, nxt)
        self.state_cells.append(sc)
        return sc

    def enforce_constraint(self, constraint: VirtualPolyExpr):
        self.recurring_constraints.append(constraint)

    def enforce_boundary_constraint(self, row: int, constraint: VirtualPolyExpr):
        self.boundary_constraints.append((row, constraint))

    # ---- Circuit trait ----------------------------------------------------
    def num_rows(self) -> int:
        return self._num_rows

    def num_cols(self) -> int:
        return next_power_of_two(self.num_columns)

    def num_public_columns(self) -> int:
        # one selector per boundary constraint (:87-91)
        return len(self.boundary_constraints)

    def public_values(self):
        """:93-99 (host lists; see public_values_dev for the device form)"""
        pub = [[0] * self.num_rows() for _ in range(self.num_public_columns())]
        for i, (row, _) in enumerate(self.boundary_constraints):
            pub[i][row] = 1
        return pub

    def public_values_dev(self, dev: Device, length: int = None):
        """public_values() zero-padded to `length` rows, as device vectors
        (with a communicator attached: this rank's block of each)"""
        length = self.num_rows() if length is None else length
        B = length // dev.world
        lo = dev.rank * B
        out = []
        for row, _ in self.boundary_constraints:
            v = np.zeros(B, dtype=np.uint64)
            if lo <= row < lo + B:
                v[row - lo] = 1
            out.append(DeviceVec.from_u64(dev, v))
        return out

    def zero_check_expressions(self):
        """:101-118: recurring constraints, then selector_i * boundary_i"""
        cs = list(self.recurring_constraints)
        pc = self.num_cols()
        for i, (_row, c) in enumerate(self.boundary_constraints):
            cs.append(VirtualPolyExpr("mul", VirtualPolyExpr.Input(i + pc), c))
        return cs

    def permutation_u64(self):
        """:120-151 as u64 arrays (id, permutation), each entry + 1"""
        rows = self.num_rows()
        ncells = rows * self.num_cols()
        assert ncells & (ncells - 1) == 0
        ids = np.arange(ncells, dtype=np.uint64)
        perm = ids.copy()
        r = np.arange(rows - 1, dtype=np.uint64)
        for sc in self.state_cells:
            frm = sc.next.col * rows + r
            to = sc.current.col * rows + r + 1
            perm[frm] = to
            perm[to] = frm
        return ids + 1, perm + 1

    def permutation(self):
        ids, perm = self.permutation_u64()
        return [int(x) for x in ids], [int(x) for x in perm]

    def check_constraints(self, witness) -> None:
        """:153-204 on device-resident columns (list of DeviceVec: all num_rows
        entries, or with a communicator attached this rank's row block of each
        column); raises ValueError on the first violation, in the reference's
        order (recurring, boundary, permutation).  Sharded, every rank reaches
        the same verdict: first bad rows are allgathered, and the copy
        constraint across a block boundary uses the next rank's first row."""
        rows = self.num_rows()
        nv = rows.bit_length() - 1
        dev = witness[0].dev
        RL = rows // dev.world
        base = dev.rank * RL
        ptrs = (C.c_void_p * len(witness))(*[w.h for w in witness])

        def global_min(local):  # smallest non-negative over ranks, or -1
            vals = [int.from_bytes(b, "little", signed=True)
                    for b in dev.allgather_bytes(int(local).to_bytes(8, "little", signed=True))]
            vals = [v for v in vals if v >= 0]
            return min(vals) if vals else -1

        first = -1
        for c in self.recurring_constraints:
            prog, plen, carr, nc = _program_c(c)
            r = C.c_int64()
            check(lib().qg_expr_first_nonzero_dev(
                dev.h, nv, len(witness), ptrs, prog, plen,
                carr.ctypes.data_as(C.POINTER(C.c_uint64)), nc, C.byref(r)), dev.h)
            if r.value >= 0 and (first < 0 or base + r.value < first):
                first = base + r.value
        first = global_min(first)
        if first >= 0:
            raise ValueError(f"Recurring constraint not satisfied at row {first}")
        for i, (row, c) in enumerate(self.boundary_constraints):
            bad = 0
            if base <= row < base + RL:
                vals = [fr_from_mont_limbs(list(w.view(row - base, 1).to_numpy()[0]))
                        for w in witness]
                bad = 1 if c.evaluate(vals) != 0 else 0
            if global_min(row if bad else -1) >= 0:
                raise ValueError(f"Boundary constraint {c} not satisfied at row {row}")
        first = -1
        for sc in self.state_cells:
            cur, nxt = witness[sc.current.col], witness[sc.next.col]
            bad = nxt.first_mismatch(cur, 0, 1, RL - 1)
            if bad >= 0:
                bad += base
            if dev.world > 1:  # every rank joins the allgather
                # next(last row of this block) == current(first row of the next block)
                firsts = dev.allgather_bytes(cur.view(0, 1).to_numpy().tobytes())
                if bad < 0 and dev.rank + 1 < dev.world:
                    mine = nxt.view(RL - 1, 1).to_numpy().tobytes()
                    if mine != firsts[dev.rank + 1]:
                        bad = base + RL - 1
            if bad >= 0 and (first < 0 or bad < first):
                first = bad
        # (every rank runs the same allgathers above: the loop shape is rank-independent)
        first = global_min(first)
        if first >= 0:
            raise ValueError(f"Permutation constraint not satisfied for state cell at row "
                             f"{first}")
