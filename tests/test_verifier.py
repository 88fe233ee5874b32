"""Product verifiers and proof wire format on the CPU (no GPU needed: the
pairing, the KZG / ML-PCS checks and the transcript are host code in
libquill_gpu.so; the HyperPlonk verifier is the host mirror of
proof.rs:303-522).

  * the tower pairing (csrc/pairing.hip) equals the oracle's independent
    w-basis pairing (oracle/pairing_oracle.py) value for value, and is
    bilinear and non-degenerate;
  * KZG::verify (kzg.rs:98-108) and MLEvalProof::verify (mlpcs.rs:126-161)
    accept the oracle prover's proofs (whose own check is the independent
    trapdoor identity), end in the oracle verifier's transcript state, and
    reject every tampered field;
  * the HyperPlonk verifier accepts the oracle's 8-row proofs of the
    reference's circuits (test_basic_proof.rs) in the oracle's final state and
    raises the reference's error for tampered ones;
  * serialize -> deserialize is the identity; malformed encodings raise."""
import random

import pytest

import hyperplonk_oracle as ho
import pairing_oracle as po
import quill_oracle as o

R = o.R_MOD
TAU = 0x48595045524C4F4E4B


def _q():
    import quill_amd
    return quill_amd


def test_g2_generator_and_mul_match_oracle():
    q = _q()
    g2 = q.g2_generator()
    assert g2 == po.G2_GEN
    assert po.g2_on_curve(g2)
    for k in (1, 2, 0xDEADBEEF, R - 1, TAU):
        assert q.g2_mul(g2, k) == po.g2_mul(po.G2_GEN, k)
    assert q.g2_mul(g2, R) is None and q.g2_mul(g2, 0) is None


def test_g2_rejects_point_off_curve():
    q = _q()
    (x0, x1), (y0, y1) = q.g2_generator()
    with pytest.raises(q.QuillGpuError):
        q.g2_mul(((x0, x1), (y0 + 1, y1)), 3)


def test_pairing_equals_oracle_value():
    """same reduced pairing, two representations (tower vs w-basis)"""
    q = _q()
    rnd = random.Random(7)
    a, b = rnd.randrange(1, R), rnd.randrange(1, R)
    P = po.g1_mul(po.G1_GEN, a)
    Q = po.g2_mul(po.G2_GEN, b)
    assert po.tower_to_w(q.pairing(P, Q)) == po.pairing(P, Q)


def test_pairing_bilinear_nondegenerate():
    q = _q()
    g2 = q.g2_generator()
    e = q.pairing((1, 2), g2)
    one = [1] + [0] * 11
    assert e != one
    a, b = 0x1234567, 0x89ABCDEF
    lhs = q.pairing(po.g1_mul(po.G1_GEN, a), q.g2_mul(g2, b))
    assert lhs == q.pairing(po.g1_mul(po.G1_GEN, a * b % R), g2)
    assert lhs == q.pairing((1, 2), q.g2_mul(g2, a * b % R))
    assert po.tower_to_w(lhs) == po.f12_pow(po.tower_to_w(e), a * b)
    # identity in either slot
    assert q.pairing(None, g2) == one and q.pairing((1, 2), None) == one
    # order r: e(-P, Q) e(P, Q) = 1
    assert po.f12_mul(po.tower_to_w(q.pairing(po.g1_neg(po.G1_GEN), g2)),
                      po.tower_to_w(e)) == po.f12(1)


def _kzg_pair(max_degree):
    q = _q()
    return o.KZG(max_degree, TAU), q.KZG.verifier(tau=TAU)


def test_kzg_verify_univariate():
    q = _q()
    okzg, vk = _kzg_pair(16)
    rnd = random.Random(3)
    poly = [rnd.randrange(R) for _ in range(17)]
    C = okzg.commit(poly)
    x = rnd.randrange(R)
    ox, oy, opi = okzg.open(poly, x)
    op = q.KZGOpeningProof(ox, oy, opi)
    assert vk.verify_univariate(C, op)
    assert po.kzg_verify(po.G1_GEN, po.G2_GEN, po.g2_mul(po.G2_GEN, TAU), C, ox, oy, opi)
    assert not vk.verify_univariate(C, q.KZGOpeningProof(ox, (oy + 1) % R, opi))
    assert not vk.verify_univariate(C, q.KZGOpeningProof((ox + 1) % R, oy, opi))
    assert not vk.verify_univariate(C, q.KZGOpeningProof(ox, oy, po.g1_add(opi, po.G1_GEN)))
    assert not vk.verify_univariate(po.g1_add(C, po.G1_GEN), op)
    # the zero polynomial: commitment and quotient are the identity
    zx, zy, zpi = okzg.open([0], x)
    assert vk.verify_univariate(None, q.KZGOpeningProof(zx, zy, zpi))
    with pytest.raises(q.QuillGpuError):  # point off the curve
        vk.verify_univariate((1, 3), op)


def _mle_from_oracle(p):
    q = _q()
    return q.MLEvalProof(list(p.evaluation_point), p.evaluation, p.s_comm,
                         *[q.KZGOpeningProof(*t) for t in (p.poly_opening, p.poly_opening_inv,
                                                          p.s_opening, p.s_opening_inv)])


@pytest.mark.parametrize("nv", [0, 1, 4, 7])
def test_mle_verify_oracle_proofs(nv):
    q = _q()
    okzg, vk = _kzg_pair(max(2, 2 << nv))
    rnd = random.Random(nv)
    poly = [rnd.randrange(R) for _ in range(1 << nv)]
    pt = [rnd.randrange(R) for _ in range(nv)]
    C = okzg.commit(poly)
    ot = o.Transcript(b"mle_verify")
    oproof = o.MLEvalProof.prove(poly, pt, okzg, ot)
    proof = _mle_from_oracle(oproof)
    t = q.Transcript(b"mle_verify")
    assert vk.verify(C, proof, t)
    assert t.state == ot.state
    # tampering: evaluation, each opening value, the s commitment, the commitment
    bad = _mle_from_oracle(oproof)
    bad.evaluation = (bad.evaluation + 1) % R
    assert not vk.verify(C, bad, q.Transcript(b"mle_verify"))
    for name in ("poly_opening", "poly_opening_inv", "s_opening", "s_opening_inv"):
        bad = _mle_from_oracle(oproof)
        op = getattr(bad, name)
        op.y = (op.y + 1) % R
        assert not vk.verify(C, bad, q.Transcript(b"mle_verify")), name
    bad = _mle_from_oracle(oproof)
    bad.s_comm = po.g1_add(bad.s_comm, po.G1_GEN)
    assert not vk.verify(C, bad, q.Transcript(b"mle_verify"))
    assert not vk.verify(po.g1_add(C, po.G1_GEN), proof, q.Transcript(b"mle_verify"))


# ---------------------------------------------------------------- HyperPlonk
def _to_product(op):
    """oracle HyperPlonkProof -> product dataclasses (same values)"""
    q = _q()
    tps = []
    for tp in op.trace_proofs:
        oz = tp.zero_check_proof
        zc = q.ZeroCheckProof(oz.num_vars, q.SumcheckProof(
            oz.sumcheck_proof.num_vars, oz.sumcheck_proof.claimed_sum,
            [list(p) for p in oz.sumcheck_proof.r_polys]))
        om = tp.permutation_check_proof
        me = q.MultisetEqualityProof(
            om.denom_left_commitment, om.denom_right_commitment,
            q.SumcheckProof(om.sumcheck_proof.num_vars, om.sumcheck_proof.claimed_sum,
                            [list(p) for p in om.sumcheck_proof.r_polys]),
            _mle_from_oracle(om.opening_proof_denom_left),
            _mle_from_oracle(om.opening_proof_denom_right))
        tps.append(q.TraceProof(zc, q.PermutationCheckProof(me),
                                [_mle_from_oracle(p) for p in tp.openings_zero_check],
                                [_mle_from_oracle(p) for p in tp.openings_public],
                                _mle_from_oracle(tp.opening_id),
                                _mle_from_oracle(tp.opening_permutation),
                                _mle_from_oracle(tp.opening_permutation_trace)))
    return q.HyperPlonkProof(list(op.witness_commitment), tps)


def _product_vk(rows, which, ohp):
    q = _q()
    from quill_amd import examples as ex
    builders = {"fib": ex.fibonacci_circuit_and_trace, "mod": ex.modified_fibonacci_circuit_and_trace}
    vks = []
    for w, ovk in zip(which, ohp.trace_vks):
        c, _ = builders[w](rows)
        vks.append(q.TraceVK(c, list(ovk.public_columns_commitments), ovk.id_commitment,
                             ovk.permutation_commitment))
    return vks


@pytest.fixture(scope="module")
def oracle_hyperplonk():
    rows, which = 8, ("fib", "mod")
    builders = {"fib": ho.fibonacci_circuit_and_trace, "mod": ho.modified_fibonacci_circuit_and_trace}
    cws = [builders[w](rows) for w in which]
    pcs = o.KZG(max(c.num_cols() * c.num_rows() for c, _ in cws), TAU)
    hp = ho.HyperPlonk.preprocess([c for c, _ in cws], pcs)
    proof, ot = hp.prove(pcs, [w for _, w in cws])
    return rows, which, hp, proof, ot


def test_hyperplonk_verifier_accepts_oracle_proof(oracle_hyperplonk):
    q = _q()
    rows, which, ohp, oproof, ot = oracle_hyperplonk
    proof = _to_product(oproof)
    vk = _product_vk(rows, which, ohp)
    t = proof.verify(vk, q.KZG.verifier(tau=TAU))
    assert t.state == ot.state


@pytest.mark.parametrize("where,msg", [
    ("zc_rpoly", "Sumcheck polynomial does not sum"),
    ("zc_opening_eval", "Zero check opening verification failed"),
    ("perm_denom", "Multiset equality opening proof verification failed"),
    ("public_eval", "Public opening verification failed"),
    ("witness_comm", "Sumcheck polynomial does not sum"),
])
def test_hyperplonk_verifier_rejects_tampering(oracle_hyperplonk, where, msg):
    q = _q()
    rows, which, ohp, oproof, _ = oracle_hyperplonk
    proof = _to_product(oproof)
    tp = proof.trace_proofs[1]
    if where == "zc_rpoly":
        tp.zero_check_proof.sumcheck_proof.r_polys[0][0] += 1
    elif where == "zc_opening_eval":
        tp.openings_zero_check[2].evaluation = (tp.openings_zero_check[2].evaluation + 1) % R
    elif where == "perm_denom":
        me = tp.permutation_check_proof.multiset_equality_proof
        me.opening_proof_denom_left.evaluation = (me.opening_proof_denom_left.evaluation + 1) % R
    elif where == "public_eval":
        tp.openings_public[0].evaluation = (tp.openings_public[0].evaluation + 1) % R
    else:
        # a different witness commitment changes every challenge: the
        # zero-check's second round no longer chains
        proof.witness_commitment[1] = po.g1_add(proof.witness_commitment[1], po.G1_GEN)
    with pytest.raises(ValueError, match=msg):
        proof.verify(_product_vk(rows, which, ohp), q.KZG.verifier(tau=TAU))


def test_serialize_roundtrip_and_verify(oracle_hyperplonk):
    q = _q()
    rows, which, ohp, oproof, ot = oracle_hyperplonk
    proof = _to_product(oproof)
    blob = q.serialize(proof)
    back = q.deserialize(q.HyperPlonkProof, blob)
    assert back == proof
    assert q.serialize(back) == blob
    t = back.verify(_product_vk(rows, which, ohp), q.KZG.verifier(tau=TAU))
    assert t.state == ot.state
    # component types
    mle = proof.trace_proofs[0].opening_id
    assert q.deserialize(q.MLEvalProof, q.serialize(mle)) == mle
    sc = proof.trace_proofs[0].zero_check_proof.sumcheck_proof
    assert q.deserialize(q.SumcheckProof, q.serialize(sc)) == sc


def test_serialize_layout_and_errors():
    q = _q()
    from quill_amd.serialize import deserialize, serialize
    sc = q.SumcheckProof(2, 5, [[1, 2], [3]])
    b = serialize(sc)
    # usize, Fr, Vec<DensePolynomial>: 8 + 32 + 8 + (8 + 64) + (8 + 32)
    assert len(b) == 8 + 32 + 8 + 72 + 40
    assert b[:8] == (2).to_bytes(8, "little") and b[8:40] == (5).to_bytes(32, "little")
    with pytest.raises(ValueError, match="truncated"):
        deserialize(q.SumcheckProof, b[:-1])
    with pytest.raises(ValueError, match="trailing"):
        deserialize(q.SumcheckProof, b + b"\0")
    bad = bytearray(b)
    bad[8:40] = R.to_bytes(32, "little")
    with pytest.raises(ValueError, match="non-canonical"):
        deserialize(q.SumcheckProof, bytes(bad))
    # G1: transcript bytes, infinity flag, off-curve rejection
    op = q.KZGOpeningProof(1, 2, (1, 2))
    ob = serialize(op)
    t = q.Transcript(b"x")
    t2 = q.Transcript(b"x")
    t.append_g1((1, 2))
    t2.append_bytes(ob[64:128])
    assert t.state == t2.state
    assert deserialize(q.KZGOpeningProof, ob) == op
    inf = serialize(q.KZGOpeningProof(1, 2, None))
    assert inf[-1] == 0x40 and deserialize(q.KZGOpeningProof, inf).proof is None
    off = bytearray(ob)
    off[96] ^= 1  # y += 1
    with pytest.raises(ValueError, match="not on the curve"):
        deserialize(q.KZGOpeningProof, bytes(off))


def test_zerocheck_verify_rejects_extra_num_vars():
    """ZeroCheckProof::verify draws num_vars challenges z and divides by
    eq_eval(z, point), which asserts equal lengths (eq_eval.rs:34).  A proof
    claiming one more variable than it has sumcheck rounds must raise, not be
    accepted on a silently truncated eq."""
    q = _q()
    nv = 3
    rnd = random.Random(11)
    st = o.VirtualPolynomialStore(nv)
    a = st.allocate_polynomial([rnd.randrange(R) for _ in range(1 << nv)])
    b = st.allocate_polynomial([rnd.randrange(R) for _ in range(1 << nv)])
    c = st.allocate_polynomial([0] * (1 << nv))
    h = st.new_virtual_from_expr(o.Expr("add", o.Expr("mul", o.Expr.input(a), o.Expr.input(b)),
                                        o.Expr("mul", o.Expr.const(R - 1), o.Expr.input(c))))
    # a * b - c vanishes only where a * b == c: make c = a * b
    st.polynomials[c] = [x * y % R for x, y in zip(st.polynomials[a], st.polynomials[b])]
    oz, _ = o.ZeroCheckProof.prove(st, h, o.Transcript(b"zc_tamper"))
    sp = oz.sumcheck_proof
    good = q.ZeroCheckProof(nv, q.SumcheckProof(nv, sp.claimed_sum, [list(p) for p in sp.r_polys]))
    good.verify(q.Transcript(b"zc_tamper"))
    # the forged proof: nv + 1 challenges z drawn and num_vars = nv + 1 absorbed
    # (so every sumcheck round checks out), but only nv rounds proved
    t = o.Transcript(b"zc_tamper")
    z = [t.draw_field_element() for _ in range(nv + 1)]
    e = st.allocate_polynomial(o.fast_eq_eval_hypercube(nv, z[:nv]))
    hh = st.new_virtual_from_virtual(h)
    st.mul_in_place(hh, e)

    class Forged(o.Transcript):
        def append_u64(self, v):
            super().append_u64(nv + 1 if v == nv else v)
    ft = Forged(b"")
    ft.state = t.state
    fsp, _ = o.SumcheckProof.prove_fast(nv, st, hh, 0, ft)
    bad = q.ZeroCheckProof(nv + 1, q.SumcheckProof(nv + 1, fsp.claimed_sum,
                                                   [list(p) for p in fsp.r_polys]))
    with pytest.raises(ValueError, match="lengths differ"):
        bad.verify(q.Transcript(b"zc_tamper"))
    with pytest.raises(ValueError):
        q.field.eq_eval([1, 2], [1])


def _twist_point_outside_subgroup():
    """a point of E'(Fq2) (y^2 = x^3 + 3/(9+u)) whose order is not r: x = k + u
    for the first k with x^3 + b' a square (Fq2 square root, p = 3 mod 4),
    kept when [r] Q != O (the twist's cofactor is ~p, so almost every point)"""
    Pm = po.P

    def fsqrt(v):
        s = pow(v, (Pm + 1) // 4, Pm)
        return s if s * s % Pm == v % Pm else None

    def f2sqrt(a):
        a0, a1 = a
        alpha = fsqrt((a0 * a0 + a1 * a1) % Pm)
        if alpha is None:
            return None
        half = (Pm + 1) // 2
        for d in ((a0 + alpha) * half % Pm, (a0 - alpha) * half % Pm):
            x0 = fsqrt(d)
            if x0:
                x1 = a1 * pow(2 * x0, Pm - 2, Pm) % Pm
                if po.f2_mul((x0, x1), (x0, x1)) == (a0 % Pm, a1 % Pm):
                    return (x0, x1)
        return None
    for k in range(1, 200):
        x = (k, 1)
        y = f2sqrt(po.f2_add(po.f2_mul(po.f2_mul(x, x), x), po.B2))
        if y is None:
            continue
        Q = (x, y)
        assert po.g2_on_curve(Q)
        acc = po.g2_add(po.g2_mul(Q, R - 1), Q)  # [r] Q
        if acc is not None:
            return Q
    raise AssertionError("no twist point found")


def test_g2_rejects_point_outside_subgroup():
    """G2 inputs are checked for the prime-order subgroup (ark's Validate::Yes),
    not only for the twist equation: qg_g2_mul, qg_pairing and a
    verifying key built from published points all refuse such a point."""
    q = _q()
    Q = _twist_point_outside_subgroup()
    with pytest.raises(q.QuillGpuError):
        q.g2_mul(Q, 3)
    with pytest.raises(q.QuillGpuError):
        q.pairing((1, 2), Q)
    okzg = o.KZG(4, TAU)
    poly = [1, 2, 3]
    ox, oy, opi = okzg.open(poly, 5)
    vk = q.KZG.verifier(g2_points=[q.g2_generator(), Q])
    with pytest.raises(q.QuillGpuError):
        vk.verify_univariate(okzg.commit(poly), q.KZGOpeningProof(ox, oy, opi))
    # subgroup points still pass (generator and a multiple)
    g2 = q.g2_generator()
    assert q.g2_mul(q.g2_mul(g2, 12345), 1) == q.g2_mul(g2, 12345)
