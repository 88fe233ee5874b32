"""Config 5 (HyperPlonk prove, hyperplonk/src/proof/proof.rs:239-301) on the
device against the oracle restatement (oracle/hyperplonk_oracle.py).

  * the reference's own circuits (hyperplonk/tests/test_basic_proof.rs:17-196)
    at 8 rows and at 64 rows: every proof field bit-exact (commitments, sumcheck
    messages, Logup commitments, all ML-PCS openings) and the same final
    transcript state; the oracle verifier accepts the device proof;
  * the committed golden fixture (tests/golden/hyperplonk.json);
  * at 2^14 rows (2^17-cell trace), where the oracle prover is too slow: the
    oracle VERIFIER (O(log N) per opening) accepts the device proof and ends in
    the same transcript state (size-independent property);
  * prover-side sanity checks: unsatisfying witnesses raise like the
    reference's check_constraints().unwrap()."""
import json
import os

import pytest

import hyperplonk_oracle as ho
import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD
TAU = 0x48595045524C4F4E4B  # fixed trapdoor
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "hyperplonk.json")


def _o_open(p):
    return o.MLEvalProof(p.evaluation_point, p.evaluation, p.s_comm,
                         (p.poly_opening.x, p.poly_opening.y, p.poly_opening.proof),
                         (p.poly_opening_inv.x, p.poly_opening_inv.y, p.poly_opening_inv.proof),
                         (p.s_opening.x, p.s_opening.y, p.s_opening.proof),
                         (p.s_opening_inv.x, p.s_opening_inv.y, p.s_opening_inv.proof))


def to_oracle(proof):
    """device HyperPlonkProof -> oracle objects (same field values)"""
    tps = []
    for tp in proof.trace_proofs:
        zc = tp.zero_check_proof
        zsc = zc.sumcheck_proof
        oz = o.ZeroCheckProof(zc.num_vars, o.SumcheckProof(zsc.num_vars, zsc.claimed_sum,
                                                           zsc.r_polys))
        me = tp.permutation_check_proof.multiset_equality_proof
        msc = me.sumcheck_proof
        om = o.MultisetEqualityProof(me.denom_left_commitment, me.denom_right_commitment,
                                     o.SumcheckProof(msc.num_vars, msc.claimed_sum, msc.r_polys),
                                     _o_open(me.opening_proof_denom_left),
                                     _o_open(me.opening_proof_denom_right))
        tps.append(ho.TraceProof(oz, om, [_o_open(p) for p in tp.openings_zero_check],
                                 [_o_open(p) for p in tp.openings_public], _o_open(tp.opening_id),
                                 _o_open(tp.opening_permutation),
                                 _o_open(tp.opening_permutation_trace)))
    return ho.HyperPlonkProof(list(proof.witness_commitment), tps)


def _open_fields(p):
    return (list(p.evaluation_point), p.evaluation, p.s_comm, tuple(p.poly_opening),
            tuple(p.poly_opening_inv), tuple(p.s_opening), tuple(p.s_opening_inv))


def assert_same_proof(dp, op):
    """field-by-field equality of a device proof (converted) and an oracle proof"""
    dp = to_oracle(dp)
    assert dp.witness_commitment == op.witness_commitment
    assert len(dp.trace_proofs) == len(op.trace_proofs)
    for a, b in zip(dp.trace_proofs, op.trace_proofs):
        assert a.zero_check_proof.num_vars == b.zero_check_proof.num_vars
        assert a.zero_check_proof.sumcheck_proof.r_polys == b.zero_check_proof.sumcheck_proof.r_polys
        ma, mb = a.permutation_check_proof, b.permutation_check_proof
        assert ma.denom_left_commitment == mb.denom_left_commitment
        assert ma.denom_right_commitment == mb.denom_right_commitment
        assert ma.sumcheck_proof.r_polys == mb.sumcheck_proof.r_polys
        assert _open_fields(ma.opening_proof_denom_left) == _open_fields(mb.opening_proof_denom_left)
        assert _open_fields(ma.opening_proof_denom_right) == _open_fields(mb.opening_proof_denom_right)
        for x, y in zip(a.openings_zero_check + a.openings_public,
                        b.openings_zero_check + b.openings_public):
            assert _open_fields(x) == _open_fields(y)
        assert len(a.openings_zero_check) == len(b.openings_zero_check)
        assert len(a.openings_public) == len(b.openings_public)
        for k in ("opening_id", "opening_permutation", "opening_permutation_trace"):
            assert _open_fields(getattr(a, k)) == _open_fields(getattr(b, k))


def _device_setup(dev, rows, which, as_lists=False):
    from quill_amd import KZG, HyperPlonk
    from quill_amd import examples as ex
    builders = {"fib": ex.fibonacci_circuit_and_trace,
                "mod": ex.modified_fibonacci_circuit_and_trace}
    cws = [builders[w](rows, as_lists=as_lists) for w in which]
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = KZG.trusted_setup(maxdeg, TAU, dev)
    hp = HyperPlonk.preprocess([c for c, _ in cws], pcs)
    return pcs, hp, [w for _, w in cws]


def _oracle_setup(rows, which):
    builders = {"fib": ho.fibonacci_circuit_and_trace,
                "mod": ho.modified_fibonacci_circuit_and_trace}
    cws = [builders[w](rows) for w in which]
    maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
    pcs = o.KZG(maxdeg, TAU)
    hp = ho.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    return pcs, hp, [w for _, w in cws]


@pytest.mark.parametrize("rows,which", [(8, ("fib",)), (8, ("fib", "mod")), (64, ("mod", "fib"))])
def test_hyperplonk_prove_vs_oracle(dev, rows, which):
    """test_basic_proof.rs:137-196 (8 rows) and a 64-row variant: bit-exact."""
    pcs, hp, ws = _device_setup(dev, rows, which)
    opcs, ohp, ows = _oracle_setup(rows, which)
    for a, b in zip(hp.trace_vks, ohp.trace_vks):
        assert a.public_columns_commitments == b.public_columns_commitments
        assert a.id_commitment == b.id_commitment
        assert a.permutation_commitment == b.permutation_commitment
    proof = hp.prove(pcs, ws)
    oproof, ot = ohp.prove(opcs, ows)
    assert_same_proof(proof, oproof)
    assert hp.last_transcript.state == ot.state
    vt = ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
    assert vt.state == ot.state


def test_hyperplonk_golden(dev):
    """the committed fixture (tests/golden/make_golden.py, multitrace at 8 rows)"""
    with open(GOLDEN) as f:
        g = json.load(f)
    pcs, hp, ws = _device_setup(dev, g["rows"], tuple(g["circuits"]))
    proof = hp.prove(pcs, ws)
    assert [list(c) for c in proof.witness_commitment] == [[int(x) for x in c]
                                                           for c in g["witness_commitments"]]
    assert hp.last_transcript.state.hex() == g["final_state"]
    assert [p.zero_check_proof.sumcheck_proof.r_polys for p in proof.trace_proofs] == \
        [[[int(x) for x in m] for m in rp] for rp in g["zerocheck_r_polys"]]


def test_hyperplonk_2p14_rows_oracle_verifies(dev):
    """2^14 rows (fib: 2^16 cells, mod-fib: 2^17 cells): the oracle verifier
    accepts and reproduces the prover's final transcript state."""
    rows = 1 << 14
    pcs, hp, ws = _device_setup(dev, rows, ("fib", "mod"))
    proof = hp.prove(pcs, ws)
    opcs, ohp, _ = _oracle_setup(rows, ("fib", "mod"))  # preprocessing only: cheap
    for a, b in zip(hp.trace_vks, ohp.trace_vks):
        assert (a.id_commitment, a.permutation_commitment) == (b.id_commitment,
                                                               b.permutation_commitment)
    vt = ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
    assert vt.state == hp.last_transcript.state


def test_hyperplonk_tampered_proof_rejected(dev):
    pcs, hp, ws = _device_setup(dev, 8, ("fib", "mod"))
    opcs, ohp, _ = _oracle_setup(8, ("fib", "mod"))
    proof = to_oracle(hp.prove(pcs, ws))
    proof.trace_proofs[1].openings_zero_check[2].evaluation += 1
    with pytest.raises(ValueError):
        ho.hyperplonk_verify(proof, ohp.to_vk(), opcs)


@pytest.mark.parametrize("kind", ["recurring", "boundary", "copy"])
def test_hyperplonk_bad_witness_raises(dev, kind):
    """check_constraints (transition_circuit.rs:153-204) on the device."""
    rows = 16
    pcs, hp, ws = _device_setup(dev, rows, ("mod",), as_lists=True)
    w = [list(c) for c in ws[0]]  # s1 = (0, 1), s2 = (2, 3), tmp = 4
    if kind == "recurring":   # tmp != s1c * s2c at row 5
        w[4][5] += 1
    elif kind == "boundary":  # s1c(0) = 2: row 0 self-consistent, boundary violated
        w[0][0] = 2
        w[4][0] = 2 * w[2][0] % R
        w[3][0] = (w[0][0] + w[4][0]) % R
    else:                     # last row recomputed from a new s1c: s1n(L-1) != s1c(L)
        L = rows - 1
        w[0][L] = (w[0][L] + 1) % R
        w[4][L] = w[0][L] * w[2][L] % R
        w[3][L] = (w[0][L] + w[4][L]) % R
    exp = {"recurring": "Recurring", "boundary": "Boundary", "copy": "Permutation"}[kind]
    with pytest.raises(ValueError, match=exp):
        hp.prove(pcs, [w])
