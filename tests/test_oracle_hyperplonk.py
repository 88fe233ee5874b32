"""CPU tests of the HyperPlonk restatement (oracle/hyperplonk_oracle.py) and of the
host-side frontend mirror (quill_amd.frontend / quill_amd.examples).

Pinning: the reference's end-to-end tests (hyperplonk/tests/test_basic_proof.rs:
137-196) assert prove -> verify acceptance for the fibonacci circuit alone and
for the fibonacci + modified-fibonacci multitrace; both are reproduced here, as
is rejection of tampered proofs (the reference's verifier error paths,
proof.rs:404-491) and of unsatisfying witnesses (transition_circuit.rs:153-204).
"""
import json
import os
import random

import pytest

import hyperplonk_oracle as ho
import quill_oracle as o

R = o.R_MOD
TAU = 0x48595045524C4F4E4B


def _prove(rows, which):
    b = {"fib": ho.fibonacci_circuit_and_trace, "mod": ho.modified_fibonacci_circuit_and_trace}
    cws = [b[w](rows) for w in which]
    pcs = o.KZG(max(c.num_cols() * c.num_rows() for c, _ in cws), TAU)
    hp = ho.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    proof, t = hp.prove(pcs, [w for _, w in cws])
    return pcs, hp, proof, t


def test_hyperplonk_proof():
    """test_basic_proof.rs:137-163"""
    pcs, hp, proof, t = _prove(8, ("fib",))
    assert ho.hyperplonk_verify(proof, hp.to_vk(), pcs).state == t.state


def test_hyperplonk_proof_multitrace():
    """test_basic_proof.rs:165-196"""
    pcs, hp, proof, t = _prove(8, ("fib", "mod"))
    assert ho.hyperplonk_verify(proof, hp.to_vk(), pcs).state == t.state


def test_golden_fixture_reproduces():
    with open(os.path.join(os.path.dirname(__file__), "golden", "hyperplonk.json")) as f:
        g = json.load(f)
    pcs, hp, proof, t = _prove(g["rows"], tuple(g["circuits"]))
    assert t.state.hex() == g["final_state"]
    assert [[str(x) for x in C] for C in proof.witness_commitment] == g["witness_commitments"]


@pytest.mark.parametrize("field", ["zc_eval", "pub_eval", "perm_trace_eval", "commitment",
                                   "zc_round", "vk"])
def test_tampered_proof_rejected(field):
    pcs, hp, proof, _ = _prove(8, ("fib", "mod"))
    vks = hp.to_vk()
    tp = proof.trace_proofs[1]
    if field == "zc_eval":
        tp.openings_zero_check[0].evaluation += 1
    elif field == "pub_eval":
        tp.openings_public[1].evaluation += 1
    elif field == "perm_trace_eval":
        tp.opening_permutation_trace.evaluation += 1
    elif field == "commitment":
        proof.witness_commitment[0] = o.g1_add(proof.witness_commitment[0], o.G1_GEN)
    elif field == "zc_round":
        tp.zero_check_proof.sumcheck_proof.r_polys[1][0] += 1
    else:
        vks[0].id_commitment = o.g1_add(vks[0].id_commitment, o.G1_GEN)
    with pytest.raises(ValueError):
        ho.hyperplonk_verify(proof, vks, pcs)


def test_unsatisfying_witness_rejected():
    c, w = ho.modified_fibonacci_circuit_and_trace(8)
    w[4][3] += 1
    with pytest.raises(ValueError, match="Recurring"):
        c.check_constraints(w)
    c, w = ho.fibonacci_circuit_and_trace(8)
    w[1][6] += 1  # s1n(6) != s2c(6): recurring; copy to s1c(7) too
    with pytest.raises(ValueError):
        c.check_constraints(w)


def test_permutation_mapping_is_involution():
    """transition_circuit.rs:120-151: the copy mapping swaps (next, i) <-> (current, i+1)."""
    c, _ = ho.modified_fibonacci_circuit_and_trace(16)
    ids, perm = c.permutation()
    p = [x - 1 for x in perm]
    assert ids == list(range(1, len(ids) + 1))
    assert all(p[p[i]] == i for i in range(len(p)))
    assert 0 not in perm


# ---- the product's host-side frontend mirror against the oracle (no GPU) -------
@pytest.mark.parametrize("rows", [8, 64, 1024])
@pytest.mark.parametrize("which", ["fib", "mod"])
def test_frontend_mirror_matches_oracle(rows, which):
    from quill_amd import examples as ex
    b = {"fib": (ex.fibonacci_circuit_and_trace, ho.fibonacci_circuit_and_trace),
         "mod": (ex.modified_fibonacci_circuit_and_trace, ho.modified_fibonacci_circuit_and_trace)}
    c, w = b[which][0](rows, as_lists=True)
    oc, ow = b[which][1](rows)
    assert (c.num_rows(), c.num_cols(), c.num_public_columns()) == \
        (oc.num_rows(), oc.num_cols(), oc.num_public_columns())
    assert w == ow
    assert c.public_values() == oc.public_values()
    assert c.permutation() == oc.permutation()
    rnd = random.Random(rows)
    for ce, oe in zip(c.zero_check_expressions(), oc.zero_check_expressions()):
        vals = [rnd.randrange(R) for _ in range(c.num_cols() + c.num_public_columns())]
        assert ce.evaluate(vals) == oe.evaluate(vals)
    # canonical-limb witness form used by TraceWitness
    _, wl = b[which][0](rows)
    for col_l, col_ints in zip(wl, w):
        back = [int(x[0]) | int(x[1]) << 64 | int(x[2]) << 128 | int(x[3]) << 192 for x in col_l]
        assert back == col_ints
