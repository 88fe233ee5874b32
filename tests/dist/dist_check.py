"""Multi-rank parity check of the sharded MSM and sumcheck / zero-check.

Launch: torchrun --nproc-per-node N --master-addr 127.0.0.1 tests/dist/dist_check.py
(one process per GPU; ranks may share a GPU where RCCL allows it).  Every rank
checks its result against the single-process oracle on the full inputs and
prints one JSON line; exit status 1 on any mismatch.
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "quill-zkvm_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import quill_amd as q  # noqa: E402
import quill_oracle as o  # noqa: E402
from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_tables  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ngpu = torch.cuda.device_count()
    dev = q.Device(int(os.environ.get("LOCAL_RANK", rank)) % ngpu)
    obj = [q.Device.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    dev.attach_comm(rank, world, obj[0])
    R = o.R_MOD
    res = {"rank": rank, "world": world}
    ok = True

    # ---- MSM: one commitment of length world * L, rank r owns [rL, (r+1)L)
    rnd = random.Random(99)
    L = 1 << 10
    tau = rnd.randrange(R)
    scal = [rnd.randrange(R) for _ in range(world * L)]
    srs = q.Srs.generate(dev, tau, L, offset=rank * L)
    got = srs.msm(scal[rank * L:(rank + 1) * L])
    exp = o.g1_mul(o.G1_GEN, o.poly_eval(scal, tau))
    res["msm"] = got == exp
    ok &= got == exp

    # ---- sumcheck: global nvars, rank block = high bits
    lw = world.bit_length() - 1
    nv = 9 + lw
    N, NL = 1 << nv, 1 << (nv - lw)
    tabs = [[rnd.randrange(R) for _ in range(N)] for _ in range(3)]
    loc = [t[rank * NL:(rank + 1) * NL] for t in tabs]
    me = E.Input(0) * E.Input(1) * E.Input(2)
    oe = o.Expr.input(0) * o.Expr.input(1) * o.Expr.input(2)
    claimed = sum(a * b % R * c for a, b, c in zip(*tabs)) % R
    t = q.Transcript(b"dist_sumcheck")
    rp, pt, ev = sumcheck_prove_tables(dev, nv, loc, me, claimed, t)
    st = o.VirtualPolynomialStore(nv)
    for tb in tabs:
        st.allocate_polynomial(tb)
    h = st.new_virtual_from_expr(oe)
    ot = o.Transcript(b"dist_sumcheck")
    oproof, (opt, oev) = o.SumcheckProof.prove_fast(nv, st, h, claimed, ot)
    good = rp == oproof.r_polys and pt == opt and ev == oev and t.state == ot.state
    res["sumcheck"] = good
    ok &= good

    # ---- zero-check h = g0*g0 - g1 with g1 = g0^2 (valid)
    g0 = [rnd.randrange(R) for _ in range(N)]
    g1 = [x * x % R for x in g0]
    me = E.Input(0) * E.Input(0) - E.Input(1)
    oe = o.Expr.input(0) * o.Expr.input(0) - o.Expr.input(1)
    t = q.Transcript(b"dist_zerocheck")
    rp, pt, ev = sumcheck_prove_tables(dev, nv, [g0[rank * NL:(rank + 1) * NL],
                                                 g1[rank * NL:(rank + 1) * NL]], me, 0, t,
                                       zerocheck=True)
    st = o.VirtualPolynomialStore(nv)
    st.allocate_polynomial(g0)
    st.allocate_polynomial(g1)
    h = st.new_virtual_from_expr(oe)
    ot = o.Transcript(b"dist_zerocheck")
    zp, (opt, oev) = o.ZeroCheckProof.prove(st, h, ot)
    good = rp == zp.sumcheck_proof.r_polys and pt == opt and ev == oev and t.state == ot.state
    res["zerocheck"] = good
    ok &= good

    print(json.dumps(res), flush=True)
    dev.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
