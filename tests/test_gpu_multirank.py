"""Sharded (multi-rank) paths on one GPU: `world` contexts in `world` host
threads joined by the library's in-process loopback communicator, which
replaces only the RCCL allgather.  Checks the sharded MSM, sumcheck and
zero-check against the single-process oracle, bit for bit."""
import random
import threading

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD


def run_ranks(world, fn):
    import quill_amd as q
    group = q.Device.loopback_group(world)
    out = [None] * world
    err = []

    def body(rank):
        try:
            dev = q.Device(0)
            dev.attach_loopback(group, rank)
            out[rank] = fn(dev, rank, world)
            dev.close()
        except Exception as e:  # surfaced below
            err.append(e)

    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=600)
    q.lib().qg_loopback_destroy(group)
    assert not err, err
    return out


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_msm(world):
    import quill_amd as q
    rnd = random.Random(world)
    L = 1 << 11
    tau = rnd.randrange(R)
    scal = [rnd.randrange(R) for _ in range(world * L)]
    exp = o.g1_mul(o.G1_GEN, o.poly_eval(scal, tau))

    def fn(dev, rank, world):
        srs = q.Srs.generate(dev, tau, L, offset=rank * L)
        r = srs.msm(scal[rank * L:(rank + 1) * L])
        srs.close()
        return r
    assert all(r == exp for r in run_ranks(world, fn))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_msm_oneshot_bases(world):
    """each rank's shard of the bases uploaded one-shot (qg_bases_upload): the
    window-by-window MSM's per-rank partials summed over the ranks"""
    import quill_amd as q
    rnd = random.Random(40 + world)
    L = 3000
    tau = rnd.randrange(R)
    scal = [rnd.randrange(R) for _ in range(world * L)]
    exp = o.g1_mul(o.G1_GEN, o.poly_eval(scal, tau))

    def fn(dev, rank, world):
        full = q.Srs.generate(dev, tau, L, offset=rank * L)
        xy, inf = full.download_raw()
        full.close()
        one = q.Srs.upload_raw(dev, xy, inf, oneshot=True)
        r = one.msm(scal[rank * L:(rank + 1) * L])
        one.close()
        return r
    assert all(r == exp for r in run_ranks(world, fn))


@pytest.mark.parametrize("world,nv_local", [(2, 9), (4, 6), (2, 1), (8, 5), (8, 1), (1, 9)])
def test_sharded_sumcheck(world, nv_local):
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    rnd = random.Random(world * 100 + nv_local)
    lw = world.bit_length() - 1
    nv = nv_local + lw
    N, NL = 1 << nv, 1 << nv_local
    tabs = [[rnd.randrange(R) for _ in range(N)] for _ in range(4)]
    me = E.Input(0) * E.Input(1) * E.Input(2) + E.Input(3) * E.Const(9)
    oe = o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2) + o.Expr.input(3) * o.Expr.const(9)
    claimed = rnd.randrange(R)
    st = o.VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
    h = st.new_virtual_from_expr(oe)
    ot = o.Transcript(b"shard")
    proof, (opt, oev) = o.SumcheckProof.prove_fast(nv, st, h, claimed, ot)

    def fn(dev, rank, world):
        t = q.Transcript(b"shard")
        rp, pt, ev = sumcheck_prove_tables(dev, nv, [tb[rank * NL:(rank + 1) * NL] for tb in tabs],
                                           me, claimed, t)
        return rp, pt, ev, t.state
    for rp, pt, ev, s in run_ranks(world, fn):
        assert rp == proof.r_polys and pt == opt and ev == oev and s == ot.state


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_zerocheck(world):
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    rnd = random.Random(5 + world)
    lw = world.bit_length() - 1
    nv = 7 + lw
    N, NL = 1 << nv, 1 << (nv - lw)
    g0 = [rnd.randrange(R) for _ in range(N)]
    g1 = [x * x % R for x in g0]
    me = E.Input(0) * E.Input(0) - E.Input(1)
    oe = o.Expr.input(0) * o.Expr.input(0) - o.Expr.input(1)
    st = o.VirtualPolynomialStore(nv)
    st.allocate_polynomial(g0)
    st.allocate_polynomial(g1)
    h = st.new_virtual_from_expr(oe)
    ot = o.Transcript(b"zshard")
    zp, (opt, oev) = o.ZeroCheckProof.prove(st, h, ot)

    def fn(dev, rank, world):
        t = q.Transcript(b"zshard")
        rp, pt, ev = sumcheck_prove_tables(
            dev, nv, [g0[rank * NL:(rank + 1) * NL], g1[rank * NL:(rank + 1) * NL]], me, 0, t,
            zerocheck=True)
        return rp, pt, ev, t.state
    for rp, pt, ev, s in run_ranks(world, fn):
        assert rp == zp.sumcheck_proof.r_polys and pt == opt and ev == oev and s == ot.state


@pytest.mark.parametrize("world,tail_zeros", [(2, 0), (4, 0), (4, 131), (2, 1), (8, 0), (8, 131),
                                              (8, 300), (1, 0), (1, 131)])
def test_sharded_mle_open(world, tail_zeros):
    """MLEvalProof::prove with the evaluations and the SRS sharded over ranks
    equals the single-context proof (and transcript state)."""
    import quill_amd as q
    from quill_amd import KZG, Transcript
    rnd = random.Random(40 + world)
    nv = 9
    N = 1 << nv
    L = N // world
    tau = rnd.randrange(R)
    poly = [rnd.randrange(R) for _ in range(N)]
    for i in range(tail_zeros):  # trimmed length ends inside a lower rank's slice
        poly[N - 1 - i] = 0
    point = [rnd.randrange(R) for _ in range(nv)]
    dev0 = q.Device(0)
    ref_kzg = KZG.trusted_setup(N, tau, dev0)
    t_ref = Transcript(b"shard-open")
    ref = ref_kzg.open(poly, point, t_ref)
    ref_kzg.srs.close()
    dev0.close()

    def fn(dev, rank, world):
        kzg = KZG(dev, q.Srs.generate(dev, tau, L, offset=rank * L), N - 1)
        vec = q.DeviceVec.from_list(dev, poly[rank * L:(rank + 1) * L])
        t = Transcript(b"shard-open")
        pr = kzg.open_dev(vec, L, point, t)
        vec.close()
        kzg.srs.close()
        return pr, t.state
    for pr, st in run_ranks(world, fn):
        assert pr == ref and st == t_ref.state


@pytest.mark.parametrize("world,rows,which", [(2, 64, ("fib", "mod")), (4, 64, ("mod", "fib")),
                                              (4, 16, ("fib",)), (2, 1024, ("mod",)),
                                              (8, 64, ("fib", "mod")), (8, 256, ("mod",))])
def test_sharded_hyperplonk(world, rows, which):
    """HyperPlonk::prove (proof.rs:239-301) sharded over `world` ranks: every
    rank holds its row block of each column, the full witness is exchanged by
    qg_trace_full_witness, all commitments / sumchecks / Logup columns /
    openings run sharded; every rank's proof equals the single-process oracle
    proof field by field (64 rows) or is accepted by the oracle verifier."""
    import hyperplonk_oracle as ho
    import quill_amd as q
    from quill_amd import examples as ex
    from test_gpu_hyperplonk import TAU, _oracle_setup, assert_same_proof, to_oracle
    b = {"fib": ex.fibonacci_circuit_and_trace, "mod": ex.modified_fibonacci_circuit_and_trace}
    opcs, ohp, ows = _oracle_setup(rows, which)
    oproof = ot = None
    if rows <= 64:
        oproof, ot = ohp.prove(opcs, ows)

    def fn(dev, rank, world):
        cws = [b[w](rows) for w in which]
        maxdeg = max(c.num_cols() * c.num_rows() for c, _ in cws)
        pcs = q.KZG.trusted_setup(maxdeg, TAU, dev)
        hp = q.HyperPlonk.preprocess([c for c, _ in cws], pcs)
        proof = hp.prove(pcs, [w for _, w in cws])
        vks = [(vk.public_columns_commitments, vk.id_commitment, vk.permutation_commitment)
               for vk in hp.trace_vks]
        pcs.close()
        return proof, hp.last_transcript.state, vks

    outs = run_ranks(world, fn)
    for proof, state, vks in outs:
        for (pc, ic, pm), ovk in zip(vks, ohp.trace_vks):
            assert (pc, ic, pm) == (ovk.public_columns_commitments, ovk.id_commitment,
                                    ovk.permutation_commitment)
        if oproof is not None:
            assert_same_proof(proof, oproof)
            assert state == ot.state
        vt = ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
        assert vt.state == state


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_hyperplonk_bad_copy_constraint_across_blocks(world):
    """the copy constraint next(row) == current(row + 1) at a block boundary is
    checked with the neighbour rank's first row; every rank raises."""
    import quill_amd as q
    from quill_amd import examples as ex
    from test_gpu_hyperplonk import TAU
    rows = 32
    RL = rows // world

    def fn(dev, rank, world):
        c, w = ex.modified_fibonacci_circuit_and_trace(rows, as_lists=True)
        L = RL  # first row of block 1: recompute row L from a new s1c (row stays consistent)
        w[0][L] = (w[0][L] + 1) % R
        w[4][L] = w[0][L] * w[2][L] % R
        w[3][L] = (w[0][L] + w[4][L]) % R
        pcs = q.KZG.trusted_setup(c.num_cols() * rows, TAU, dev)
        hp = q.HyperPlonk.preprocess([c], pcs)
        try:
            hp.prove(pcs, [w])
            return None
        except ValueError as e:
            return str(e)
        finally:
            pcs.close()

    outs = run_ranks(world, fn)
    assert all(o_ is not None and "Permutation" in o_ and f"row {RL - 1}" in o_ for o_ in outs), outs


@pytest.mark.parametrize("world,nv", [(2, 17), (4, 18), (2, 19), (8, 19), (8, 20)])
def test_sharded_sumcheck_early_gather_matches_single(world, nv):
    """nvars >= 17: the sharded prover runs nv - 15 rounds with per-round
    allgathers, then gathers the folded tables (2^16 global entries) and
    finishes redundantly on every rank.  Bit-exact against the single-context
    device prover (itself pinned to the oracle), for a sumcheck and a zero-check."""
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    lw = world.bit_length() - 1
    N, NL = 1 << nv, 1 << (nv - lw)
    dev0 = q.Device(0)
    tabs = [q.DeviceVec(dev0, N).fill_random(1000 + i) for i in range(3)]
    host = [t.to_list() for t in tabs]
    for t in tabs:
        t.close()
    me = E.Input(0) * E.Input(1) * E.Input(2) - E.Input(2) * E.Const(5)
    rnd = random.Random(nv)
    claimed = rnd.randrange(R)
    ref = sumcheck_prove_tables(dev0, nv, host, me, claimed, q.Transcript(b"eg"))
    zref = sumcheck_prove_tables(dev0, nv, host, me, 0, q.Transcript(b"egz"), zerocheck=True)
    dev0.close()

    def fn(dev, rank, world):
        blk = [tb[rank * NL:(rank + 1) * NL] for tb in host]
        a = sumcheck_prove_tables(dev, nv, blk, me, claimed, q.Transcript(b"eg"))
        b = sumcheck_prove_tables(dev, nv, blk, me, 0, q.Transcript(b"egz"), zerocheck=True)
        return a, b

    for a, b in run_ranks(world, fn):
        assert a == ref
        assert b == zref


@pytest.mark.parametrize("world,nv,kind", [(2, 6, "tables12"), (4, 7, "deg17"), (8, 8, "blowup"),
                                           (4, 3, "tables12"), (8, 4, "deg31"), (2, 9, "deg17")])
def test_sharded_sumcheck_generic(world, nv, kind):
    """The interpreted (generic-expression) sumcheck sharded by the high index
    bits (sumcheck_run_generic): per-round allgather of the local sums, then
    the one-value-per-slot gather and the last log2(world) rounds redundantly.
    Bit-exact against the oracle's reference-structured prover; nv = log2(world)
    + 1 leaves one local round (the API needs nvars > log2(world), like the
    compiled path)."""
    import quill_amd as q
    from quill_amd.hyperplonk import sumcheck_prove_tables
    from test_gpu_generic import _exprs
    rnd = random.Random(world * 1000 + nv)
    me, oe, k = _exprs(kind)
    lw = world.bit_length() - 1
    NL = 1 << (nv - lw)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(k)]
    ost = o.VirtualPolynomialStore(nv)
    for tb in tabs:
        ost.allocate_polynomial(tb)
    oh = ost.new_virtual_from_expr(oe)
    claimed = rnd.randrange(R)
    ot = o.Transcript(b"generic-shard")
    oproof, (opt, oev) = o.SumcheckProof.prove(nv, ost, oh, claimed, ot)

    def fn(dev, rank, world):
        t = q.Transcript(b"generic-shard")
        rp, pt, ev = sumcheck_prove_tables(dev, nv, [tb[rank * NL:(rank + 1) * NL] for tb in tabs],
                                           me, claimed, t)
        return rp, pt, ev, t.state
    for rp, pt, ev, s in run_ranks(world, fn):
        assert rp == oproof.r_polys and pt == opt and ev == oev and s == ot.state


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_zerocheck_generic(world):
    """9 inputs + eq = 10 tables: the sharded zero-check's h * eq runs interpreted"""
    import quill_amd as q
    from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables
    nv = 7
    lw = world.bit_length() - 1
    NL = 1 << (nv - lw)
    rnd = random.Random(77 + world)
    tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(8)]
    tabs.append([sum(tabs[2 * j][i] * tabs[2 * j + 1][i] for j in range(4)) % R
                 for i in range(1 << nv)])
    me = E.Input(0) * E.Input(1) + E.Input(2) * E.Input(3) + E.Input(4) * E.Input(5) + \
        E.Input(6) * E.Input(7) - E.Input(8)
    O = o.Expr
    oe = O.input(0) * O.input(1) + O.input(2) * O.input(3) + O.input(4) * O.input(5) + \
        O.input(6) * O.input(7) - O.input(8)
    ost = o.VirtualPolynomialStore(nv)
    for tb in tabs:
        ost.allocate_polynomial(tb)
    oh = ost.new_virtual_from_expr(oe)
    ot = o.Transcript(b"zc-generic-shard")
    ozp, (opt, oev) = o.ZeroCheckProof.prove(ost, oh, ot)

    def fn(dev, rank, world):
        t = q.Transcript(b"zc-generic-shard")
        rp, pt, ev = sumcheck_prove_tables(dev, nv, [tb[rank * NL:(rank + 1) * NL] for tb in tabs],
                                           me, 0, t, zerocheck=True)
        return rp, pt, ev, t.state
    for rp, pt, ev, s in run_ranks(world, fn):
        assert rp == ozp.sumcheck_proof.r_polys and pt == opt and ev == oev and s == ot.state


@pytest.mark.parametrize("world,rows", [(2, 32), (4, 32), (8, 64)])
def test_sharded_hyperplonk_16_column(world, rows):
    """The 16-column TransitionCircuit (23 tables, 330-term constraint: beyond
    the compiled sumcheck image) proved sharded over `world` ranks; every
    rank's proof equals the single-process oracle proof field by field."""
    import hyperplonk_oracle as ho
    import quill_amd as q
    from test_gpu_generic import TAU as GTAU, _wide_circuit_device, _wide_circuit_oracle, \
        _wide_witness
    from test_gpu_hyperplonk import assert_same_proof, to_oracle
    w = _wide_witness(rows)
    oc_ = _wide_circuit_oracle(rows)
    opcs = o.KZG(16 * rows, GTAU)
    ohp = ho.HyperPlonk.preprocess([oc_], opcs)
    oproof, ot = ohp.prove(opcs, [w])

    def fn(dev, rank, world):
        c = _wide_circuit_device(rows)
        pcs = q.KZG.trusted_setup(16 * rows, GTAU, dev)
        hp = q.HyperPlonk.preprocess([c], pcs)
        proof = hp.prove(pcs, [w])
        pcs.close()
        return proof, hp.last_transcript.state
    for proof, state in run_ranks(world, fn):
        assert_same_proof(proof, oproof)
        assert state == ot.state
        vt = ho.hyperplonk_verify(to_oracle(proof), ohp.to_vk(), opcs)
        assert vt.state == ot.state


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_mle_open_batch_matches_sequential(world):
    """qg_mle_open_batch_dev on a sharded context (mle_open_batch_sharded: four
    exchanges per batch) equals the item-by-item sharded openings
    (QG_OPEN_BATCH_SHARDED=0) and the single-context batch, proof for proof,
    with the same transcript state, at 2^14 evaluations: full vectors, a
    zero tail ending in a lower rank's slice, a vector trimming to one entry,
    a smaller variable count, and one vector opened twice."""
    import os
    import quill_amd as q
    from quill_amd import KZG, Transcript
    rnd = random.Random(7700 + world)
    tau = rnd.randrange(R)
    shapes = [(14, None), (14, (1 << 14) - 3000), (14, 1), (12, None), (13, None)]
    polys = []
    for nv, live in shapes:
        p = [rnd.randrange(R) for _ in range(1 << nv)]
        if live is not None:
            p = p[:live] + [0] * ((1 << nv) - live)
        polys.append(p)
    items = [(i, [rnd.randrange(R) for _ in range(shapes[i][0])]) for i in range(len(shapes))]
    items.append((0, [rnd.randrange(R) for _ in range(14)]))
    dev0 = q.Device(0)
    kz = KZG.trusted_setup(1 << 14, tau, dev0)
    vs = [q.DeviceVec.from_list(dev0, p) for p in polys]
    t_ref = Transcript(b"shard-batch")
    ref = kz.open_batch_dev([(vs[i], len(polys[i]), pt, False) for i, pt in items], t_ref)
    for v in vs:
        v.close()
    kz.srs.close()
    dev0.close()

    def fn(dev, rank, world):
        kzg = KZG.trusted_setup(1 << 14, tau, dev)  # one SRS shard per local length
        vecs = []
        for p in polys:
            L = len(p) // world
            vecs.append(q.DeviceVec.from_list(dev, p[rank * L:(rank + 1) * L]))
        batch = [(vecs[i], len(vecs[i]), pt, False) for i, pt in items]
        out = []
        for mode in ("1", "0"):
            bar.wait()  # every rank is between calls: one sets the mode for all
            if rank == 0:
                os.environ["QG_OPEN_BATCH_SHARDED"] = mode
            bar.wait()
            t = Transcript(b"shard-batch")
            out.append((kzg.open_batch_dev(batch, t), t.state))
        for v in vecs:
            v.close()
        kzg.close()
        return out

    bar = threading.Barrier(world)
    try:
        outs = run_ranks(world, fn)
    finally:
        os.environ.pop("QG_OPEN_BATCH_SHARDED", None)
    for (bat, sb), (seq, ss) in outs:
        assert bat == seq and sb == ss
        assert bat == ref and sb == t_ref.state
