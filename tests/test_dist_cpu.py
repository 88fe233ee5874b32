"""gloo tests (CPU, world 2 and 4) of the multi-GPU decompositions the HIP path
implements, each restated step for step from the
product code it mirrors:

* MSM sharded by base index: each rank's partial sum, allgathered and added,
  equals the full MSM (msm_device_batch).
* Sumcheck sharded by the high index bits (run_rounds_dist): per round every
  rank sums its local pairs, the (d+1) sums are allgathered, every rank runs
  the same transcript; once the global tables reach the gather size, every
  rank allgathers its block of that round's SOURCE tables and finishes
  redundantly.  Gather points before round 0, mid-way and after the last
  local round; bit-exact against the single-process proof.
* ML-PCS opening (mle_open_sharded / kzg_open_sharded): partial evaluations,
  replicated S, the suffix-Horner carry exchange and partial MSMs; bit-exact
  against the single-process MLEvalProof incl. trimmed lengths that end
  inside a lower rank's slice.
* HyperPlonk's full-witness exchange and the copy-constraint boundary check.

The per-rank arithmetic here is the oracle's (test infrastructure); the GPU
versions of the same protocols run in loopback (tests/test_gpu_multirank.py).
"""
import os
import random
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import quill_oracle as o

R = o.R_MOD


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _allgather_obj(x, world):
    out = [None] * world
    dist.all_gather_object(out, x)
    return out


def sharded_sumcheck(rank, world, nv, tabs, expr, claimed, domain, gather_log=16):
    """The sharded protocol of run_rounds_dist (csrc/sumcheck.hip), step for step:

    * rounds j < js (js = nv + 1 - gather_log, at most the local variable
      count m) pair local entries only; the fold by r_{j-1} is fused into round
      j's evaluation (k_sc_big), each round's (d+1) local sums are allgathered
      and every rank runs the identical transcript step (k_sc_finish);
    * then every rank allgathers its block of the round-js SOURCE tables
      (folded through r_{js-2}: S = NL >> (js - 1) entries per slot, the
      product's `scg_pack`), reassembles the global tables with the rank as
      the high index bits (k_sc_gather_tables) and runs rounds js.. nv-1
      redundantly (k_sc_persist), starting with the fold by r_{js-1}.
    The product uses gather_log = 16 (SC_GATHER_LOG); the tests scale it down."""
    lw = world.bit_length() - 1
    m = nv - lw
    NL = 1 << m
    d = expr.degree()
    js = nv + 1 - gather_log if nv + 1 > gather_log else 0
    js = min(js, m)
    gs = [t[rank * NL:(rank + 1) * NL] for t in tabs]
    t = o.Transcript(domain)
    t.append_u64(nv)
    t.append_fr(claimed)
    r_polys, point = [], []

    def round_msg(sums):
        msg = o.interpolate_consecutive([s % R for s in sums])
        t.append_poly(msg)
        r_polys.append(msg)
        r = t.draw_field_element()
        point.append(r)
        return r

    def fold(gs, r):
        return [[(g[2 * p] + r * (g[2 * p + 1] - g[2 * p])) % R for p in range(len(g) // 2)]
                for g in gs]

    def sums_of(gs):
        sums = [0] * (d + 1)
        for p in range(len(gs[0]) // 2):
            lows = [g[2 * p] for g in gs]
            diffs = [g[2 * p + 1] - g[2 * p] for g in gs]
            for tt in range(d + 1):
                sums[tt] += expr.evaluate([lo + tt * df for lo, df in zip(lows, diffs)])
        return [s % R for s in sums]

    r = None
    for j in range(js):
        if j > 0:
            gs = fold(gs, r)  # fused into round j's kernel on the device
        all_sums = _allgather_obj(sums_of(gs), world)
        r = round_msg([sum(col) % R for col in zip(*all_sums)])
    # gather the round-js source tables (not yet folded by r_{js-1})
    S = len(gs[0])
    assert S == (NL if js == 0 else NL >> (js - 1))
    packed = _allgather_obj([list(g) for g in gs], world)
    gs = [[v for rk in range(world) for v in packed[rk][i]] for i in range(len(tabs))]
    for j in range(js, nv):
        if j > 0:
            gs = fold(gs, r)
        r = round_msg(sums_of(gs))
    gs = fold(gs, r)
    return r_polys, point, expr.evaluate([g[0] for g in gs]), t.state


def sharded_mle_open(rank, world, poly, point, tau, domain):
    """mle_open_sharded + kzg_open_sharded (csrc/mlpcs.hip) restated: rank r
    holds poly[r L, (r+1) L) and SRS shard [tau^(rL + i)] g.
    * eq table, local dot -> allgather of the partial evaluations;
    * allgather of the slices; S split by frequency residue (s_poly_sharded,
      tests/test_s_poly_split.py) with one all-to-all; s_comm from per-rank
      partial MSMs over the SRS shard;
    * per KZG opening: global trimmed length (allgather of per-rank maxima),
      local suffix-Horner s_i = c_i + x s_{i+1}, allgather of T_r = s_local[0],
      carry C_r = sum_{r' > r} T_r' x^((r'-r-1) L), s_i += x^(le - i) C,
      y = sum_r T_r x^(r L), quotient q_i = s_{i+1}, partial MSM + allgather.
    Returns the proof tuple and the transcript state."""
    nv = len(point)
    N = 1 << nv
    L = N // world
    off = rank * L
    mine = poly[off:off + L]

    def msm_shard(vec_local):
        # [sum_i v_i tau^(off + i)] g: this rank's partial commitment (trapdoor)
        e = sum(v * pow(tau, off + i, R) for i, v in enumerate(vec_local)) % R
        return o.g1_mul(o.G1_GEN, e)

    def sum_points(parts):
        acc = None
        for P_ in parts:
            acc = o.g1_add(acc, P_)
        return acc

    pr = o.fast_eq_eval_hypercube(nv, point)
    evaluation = sum(_allgather_obj(sum(a * b for a, b in zip(mine, pr[off:off + L])) % R,
                                    world)) % R
    full = [v for sl in _allgather_obj(mine, world) for v in sl]
    # S split by frequency residue (s_poly_sharded): this rank's outgoing
    # vectors, an all-to-all (gloo: gather then pick), the sum of what arrived
    from test_s_poly_split import rank_slice
    sends = rank_slice(full, point, world, rank)
    got = _allgather_obj(sends, world)
    S_local = [sum(got[s_][rank][m] for s_ in range(world)) % R for m in range(L)]
    nzs = [i for i, v in enumerate(S_local) if v]
    Slen = max(_allgather_obj(off + nzs[-1] + 1 if nzs else 0, world))
    s_comm = sum_points(_allgather_obj(msm_shard(S_local[:max(0, min(L, Slen - off))]), world))
    t = o.Transcript(domain)
    t.append_fr_vec(point)
    t.append_fr(evaluation)
    t.append_g1(s_comm)
    r = t.draw_field_element()
    r_inv = o.fr_inv(r)

    def open_sharded(c_local, x):
        nz = [i for i, v in enumerate(c_local) if v % R]
        Lt = max(_allgather_obj(off + nz[-1] + 1 if nz else 0, world))
        le = min(L, Lt - off) if Lt > off else 0
        s = [0] * (le + 1)
        for i in range(le - 1, -1, -1):
            s[i] = (c_local[i] + x * s[i + 1]) % R
        Ts = _allgather_obj(s[0] if le > 0 else 0, world)
        xL = pow(x, L, R)
        C = y = 0
        for rr in range(world - 1, -1, -1):
            if rr == rank:
                C = y
            y = (Ts[rr] + xL * y) % R
        for i in range(le):
            s[i] = (s[i] + pow(x, le - i, R) * C) % R
        if le > 0:
            s[le] = C
        qn = min(le, Lt - 1 - off) if Lt > 0 and Lt - 1 > off else 0
        pi = sum_points(_allgather_obj(msm_shard(s[1:1 + qn]), world))
        return (x, y, pi)

    ops = (open_sharded(mine, r), open_sharded(mine, r_inv), open_sharded(S_local, r),
           open_sharded(S_local, r_inv))
    return (evaluation, s_comm) + ops, t.state


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rnd = random.Random(7)
        # MSM sharded by base index
        L = 8
        ts = [rnd.randrange(R) for _ in range(world * L)]
        sc = [rnd.randrange(R) for _ in range(world * L)]
        bases = [o.g1_mul(o.G1_GEN, x) for x in ts]
        part = o.g1_msm_naive(bases[rank * L:(rank + 1) * L], sc[rank * L:(rank + 1) * L])
        parts = _allgather_obj(part, world)
        acc = None
        for P in parts:
            acc = o.g1_add(acc, P)
        msm_ok = acc == o.g1_mul(o.G1_GEN, sum(a * b for a, b in zip(sc, ts)))
        # sumcheck sharded by high bits
        nv = 7
        tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(3)]
        expr = o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2) - o.Expr.input(2)
        claimed = rnd.randrange(R)
        store = o.VirtualPolynomialStore(nv)
        for tb in tabs:
            store.allocate_polynomial(tb)
        h = store.new_virtual_from_expr(expr)
        ot = o.Transcript(b"dist")
        proof, (opt, oev) = o.SumcheckProof.prove_fast(nv, store, h, claimed, ot)
        sc_ok = True
        # gather points: before round 0 (whole tables), mid-way, and after the
        # last local round (the product's 2^16 at nv = 20 scales to 2^(nv-4))
        for gl in (nv + 1, nv - 2, 2, 1):
            rp, pt, ev, st = sharded_sumcheck(rank, world, nv, tabs, expr, claimed, b"dist", gl)
            sc_ok &= rp == proof.r_polys and pt == opt and ev == oev and st == ot.state
        # ML-PCS opening: slices, carries, replicated S, partial MSMs
        mle_ok = True
        tau = rnd.randrange(R)
        for nvo, tail_zeros in ((4, 0), (4, 5), (3, 7), (5, 1)):
            if (1 << nvo) < world:
                continue
            poly = [rnd.randrange(R) for _ in range(1 << nvo)]
            for i in range(tail_zeros):  # trimmed length ends inside a lower rank's slice
                poly[len(poly) - 1 - i] = 0
            pt_ = [rnd.randrange(R) for _ in range(nvo)]
            got, st_ = sharded_mle_open(rank, world, poly, pt_, tau, b"dist-open")
            oref = o.Transcript(b"dist-open")
            ref = o.MLEvalProof.prove(poly, pt_, o.KZG(1 << nvo, tau, points=[]), oref)
            want = (ref.evaluation, ref.s_comm, tuple(ref.poly_opening),
                    tuple(ref.poly_opening_inv), tuple(ref.s_opening), tuple(ref.s_opening_inv))
            mle_ok &= got == want and st_ == oref.state
        q.put((rank, msm_ok, sc_ok, mle_ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_protocols_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in results) == list(range(world))
    assert all(r[1] for r in results), results
    assert all(r[2] for r in results), results
    assert all(r[3] for r in results), results


def trace_chunks(ncols, rows, world):
    """csrc/comm.hip trace_chunks: rows [a, b) of column c go from rank src
    (its row block) to rank dst (its block of the column-major flattening)."""
    RL, B = rows // world, ncols * rows // world
    out = []
    for c in range(ncols):
        for src in range(world):
            a, end = src * RL, (src + 1) * RL
            while a < end:
                dst = (c * rows + a) // B
                b = min(end, (dst + 1) * B - c * rows)
                out.append((c, src, dst, a, b))
                a = b
    return out


def _trace_worker(rank, world, port, q):
    """qg_trace_full_witness's exchange (allgather of packed row blocks, local
    extraction) and the sharded check_constraints boundary exchange."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for ncols, rows in ((8, 64), (4, 32), (2, 16), (1, 8)):
            cols = [[1000 * c + r for r in range(rows)] for c in range(ncols)]
            RL, B = rows // world, ncols * rows // world
            mine = [col[rank * RL:(rank + 1) * RL] for col in cols]
            packed = [v for blk in mine for v in blk]
            allp = _allgather_obj(packed, world)
            full = [None] * B
            for c, src, dst, a, b in trace_chunks(ncols, rows, world):
                if dst != rank:
                    continue
                for i in range(a, b):
                    full[c * rows + i - rank * B] = allp[src][c * RL + i - src * RL]
            flat = [v for col in cols for v in col]
            ok &= full == flat[rank * B:(rank + 1) * B]
        # copy constraint across the block boundary: next(last row of block r)
        # vs current(first row of block r + 1), via an allgather of first rows
        rows = 16
        RL = rows // world
        cur = list(range(1, rows + 1))
        nxt = cur[1:] + [0]
        nxt[RL - 1] += 1  # break the constraint at the boundary of blocks 0 / 1
        firsts = _allgather_obj(cur[rank * RL], world)
        bad = -1
        for i in range(RL - 1):
            if nxt[rank * RL + i] != cur[rank * RL + i + 1]:
                bad = rank * RL + i
                break
        if bad < 0 and rank + 1 < world and nxt[rank * RL + RL - 1] != firsts[rank + 1]:
            bad = rank * RL + RL - 1
        verdicts = [v for v in _allgather_obj(bad, world) if v >= 0]
        ok &= verdicts == [RL - 1]
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_trace_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trace_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in results) == list(range(world))
    assert all(r[1] for r in results), results
