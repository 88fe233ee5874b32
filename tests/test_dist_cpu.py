"""world_size-2 gloo tests (CPU) of the multi-GPU decomposition the HIP path
implements:

* MSM sharded by base index: each rank's partial sum, allgathered and added,
  equals the full MSM.
* Sumcheck sharded by the high index bits: per round every rank sums its local
  pairs, the (d+1) sums are allgathered, every rank runs the same transcript;
  after the local rounds the single folded values are allgathered and the last
  log2(world) rounds run redundantly.  The result must equal the
  single-process proof bit for bit.

The per-rank arithmetic here is the oracle's (test infrastructure); the GPU
version of the same protocol is checked by tests/dist/dist_check.py on hardware.
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


def sharded_sumcheck(rank, world, nv, tabs, expr, claimed, domain):
    """The sharded protocol of run_rounds_dist (csrc/sumcheck.hip)."""
    lw = world.bit_length() - 1
    m = nv - lw
    NL = 1 << m
    d = expr.degree()
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

    for _ in range(m):
        sums = [0] * (d + 1)
        for p in range(len(gs[0]) // 2):
            lows = [g[2 * p] for g in gs]
            diffs = [g[2 * p + 1] - g[2 * p] for g in gs]
            for tt in range(d + 1):
                sums[tt] += expr.evaluate([lo + tt * df for lo, df in zip(lows, diffs)])
        all_sums = _allgather_obj([s % R for s in sums], world)
        r = round_msg([sum(col) % R for col in zip(*all_sums)])
        gs = [[(g[2 * p] + r * (g[2 * p + 1] - g[2 * p])) % R for p in range(len(g) // 2)]
              for g in gs]
    # gather the single local values -> tables of size world (index = rank)
    gathered = _allgather_obj([g[0] for g in gs], world)
    gs = [[gathered[rk][i] for rk in range(world)] for i in range(len(tabs))]
    for _ in range(lw):
        sums = [0] * (d + 1)
        for p in range(len(gs[0]) // 2):
            lows = [g[2 * p] for g in gs]
            diffs = [g[2 * p + 1] - g[2 * p] for g in gs]
            for tt in range(d + 1):
                sums[tt] += expr.evaluate([lo + tt * df for lo, df in zip(lows, diffs)])
        r = round_msg(sums)
        gs = [[(g[2 * p] + r * (g[2 * p + 1] - g[2 * p])) % R for p in range(len(g) // 2)]
              for g in gs]
    return r_polys, point, expr.evaluate([g[0] for g in gs]), t.state


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
        nv = 6
        tabs = [[rnd.randrange(R) for _ in range(1 << nv)] for _ in range(3)]
        expr = o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2) - o.Expr.input(2)
        claimed = rnd.randrange(R)
        rp, pt, ev, st = sharded_sumcheck(rank, world, nv, tabs, expr, claimed, b"dist")
        store = o.VirtualPolynomialStore(nv)
        for tb in tabs:
            store.allocate_polynomial(tb)
        h = store.new_virtual_from_expr(expr)
        ot = o.Transcript(b"dist")
        proof, (opt, oev) = o.SumcheckProof.prove_fast(nv, store, h, claimed, ot)
        sc_ok = rp == proof.r_polys and pt == opt and ev == oev and st == ot.state
        q.put((rank, msm_ok, sc_ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
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
