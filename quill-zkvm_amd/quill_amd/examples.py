"""The reference's example circuits (hyperplonk/tests/test_basic_proof.rs:17-105)
on the frontend mirror, with their witnesses, at any power-of-two row count —
the config-5 workload ("Fibonacci (4 cols) + modified Fibonacci (5 -> 8 cols)
TransitionCircuits").  Witness columns are returned as
(rows, 4) uint64 arrays of canonical limbs (TraceWitness uploads them)."""
from __future__ import annotations

import numpy as np

from .field import R_MOD
from .frontend import TransitionCircuit
from .hyperplonk import VirtualPolyExpr as E


def _canon(col) -> np.ndarray:
    b = b"".join(int(x).to_bytes(32, "little") for x in col)
    return np.frombuffer(b, dtype="<u8").reshape(len(col), 4).copy()


def fibonacci_circuit_and_trace(num_rows: int = 8, as_lists: bool = False):
    """test_basic_proof.rs:17-52"""
    c = TransitionCircuit(num_rows)
    s1 = c.allocate_state_cell()
    s2 = c.allocate_state_cell()
    c.enforce_boundary_constraint(0, s1.current.to_expr())
    c.enforce_boundary_constraint(0, s2.current.to_expr() - E.Const(1))
    c.enforce_constraint(s2.next.to_expr() - (s1.current.to_expr() + s2.current.to_expr()))
    c.enforce_constraint(s1.next.to_expr() - s2.current.to_expr())
    a1, a2 = [0] * num_rows, [0] * num_rows  # state1.current, state2.current
    b1, b2 = [0] * num_rows, [0] * num_rows  # state1.next, state2.next
    x, y = 0, 1
    for row in range(num_rows):
        a1[row], a2[row] = x, y
        b1[row], b2[row] = y, (x + y) % R_MOD
        x, y = b1[row], b2[row]
    w = [None] * c.num_cols()
    w[s1.current.col], w[s2.current.col], w[s1.next.col], w[s2.next.col] = a1, a2, b1, b2
    for i in range(c.num_cols()):
        if w[i] is None:
            w[i] = [0] * num_rows
    return c, (w if as_lists else [_canon(col) for col in w])


def modified_fibonacci_circuit_and_trace(num_rows: int = 8, as_lists: bool = False):
    """test_basic_proof.rs:54-105: f(n) = f(n-1) + f(n-1) f(n-2)"""
    c = TransitionCircuit(num_rows)
    s1 = c.allocate_state_cell()
    s2 = c.allocate_state_cell()
    tmp = c.allocate_witness_cell()
    c.enforce_boundary_constraint(0, s1.current.to_expr() - E.Const(1))
    c.enforce_boundary_constraint(0, s2.current.to_expr() - E.Const(1))
    c.enforce_constraint(tmp.to_expr() - s1.current.to_expr() * s2.current.to_expr())
    c.enforce_constraint(s2.next.to_expr() - (s1.current.to_expr() + tmp.to_expr()))
    c.enforce_constraint(s1.next.to_expr() - s2.current.to_expr())
    cols = {k: [0] * num_rows for k in ("a1", "a2", "b1", "b2", "t")}
    x, y = 1, 1
    for row in range(num_rows):
        t = x * y % R_MOD
        cols["a1"][row], cols["a2"][row], cols["t"][row] = x, y, t
        cols["b1"][row], cols["b2"][row] = y, (x + t) % R_MOD
        x, y = y, (x + t) % R_MOD
    w = [None] * c.num_cols()
    w[s1.current.col], w[s2.current.col] = cols["a1"], cols["a2"]
    w[s1.next.col], w[s2.next.col], w[tmp.col] = cols["b1"], cols["b2"], cols["t"]
    for i in range(c.num_cols()):
        if w[i] is None:
            w[i] = [0] * num_rows
    return c, (w if as_lists else [_canon(col) for col in w])
