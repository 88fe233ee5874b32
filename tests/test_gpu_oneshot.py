"""MSM over one-shot bases (qg_bases_upload: one table, the windows binned in
W passes and combined by Horner steps) against the oracle, the golden MSM
fixtures and the window-shifted SRS path: VariableBaseMSM::msm_unchecked
(ark-ec 0.5.0, called at pcs/src/kzg.rs:72) over bases used once.  Bit-exact."""
import json
import os
import random

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
R = o.R_MOD


def P(j):
    return None if j is None else (int(j[0]), int(j[1]))


@pytest.mark.parametrize("case", range(6))
def test_oneshot_msm_golden(dev, case):
    from quill_amd import Srs
    with open(os.path.join(GOLDEN, "msm.json")) as f:
        c = json.load(f)[case]
    srs = Srs.upload(dev, [P(b) for b in c["bases"]], oneshot=True)
    assert srs.msm([int(x) for x in c["scalars"]]) == P(c["result"])


def test_oneshot_msm_edge_scalars(dev):
    """the edge scalars of test_msm_edge_scalars (0, 1, r - 1, small, 2^253,
    an infinity base, truncation to the shorter input) on one-shot bases"""
    from quill_amd import Srs
    rnd = random.Random(5)
    ts = [rnd.randrange(R) for _ in range(300)]
    bases = [o.g1_mul(o.G1_GEN, t) for t in ts]
    bases[7] = None
    ts[7] = 0
    srs = Srs.upload(dev, bases, oneshot=True)
    c, w = srs.window_info()
    assert c * w >= 255

    def expect(sc):
        return o.g1_mul(o.G1_GEN, sum(a * b for a, b in zip(sc, ts)))
    for sc in ([0] * 300, [1] * 300, [R - 1] * 300, [rnd.randrange(256) for _ in range(300)],
               [rnd.randrange(R) for _ in range(300)], [1 << 253] * 300,
               [(1 << (c * k)) - 1 for k in range(1, 301)]):
        sc = [s % R for s in sc]
        assert srs.msm(sc) == expect(sc)
    sc = [rnd.randrange(R) for _ in range(50)]
    assert srs.msm(sc) == expect(sc)
    assert srs.msm([]) is None
    srs.close()


@pytest.mark.parametrize("logn", [12, 17, 20])
def test_oneshot_equals_srs_tables_and_trapdoor(dev, logn):
    """bases [tau^i] g downloaded from a generated SRS, uploaded one-shot: the
    MSM of random device scalars equals the window-shifted path and
    [sum s_i tau^i] g; a batch of prefixes equals its single MSMs"""
    import oracle_c as oc
    import quill_amd as q
    from quill_amd import Srs
    n = 1 << logn
    tau = 0x4F4E4553484F54 + logn
    full = Srs.generate(dev, tau, n)
    xy, inf = full.download_raw()
    one = Srs.upload_raw(dev, xy, inf, oneshot=True)
    v = q.DeviceVec(dev, n).fill_random(900 + logn)
    got = one.msm_dev(v, n)
    assert got == full.msm_dev(v, n)
    assert got == oc.g1_mul(o.G1_GEN, oc.fr_horner(v.to_numpy(n), tau))
    ns = [n, n // 2 + 3, 0, 1]
    assert one.msm_dev_batch([v] * 4, ns) == [full.msm_dev(v, m) for m in ns]
    v.close()
    one.close()
    full.close()


@pytest.mark.parametrize("oneshot", [False, True])
def test_msm_at_offset_matches_trapdoor(dev, oneshot):
    """msm_unchecked(bases[offset..], scalars) (qg_msm_g1_at / _dev_at):
    [sum s_i tau^(offset+i)] g, truncated at the end of the bases; offset 0 is
    the plain MSM, offset = len gives infinity, offset > len is rejected"""
    import oracle_c as oc
    import quill_amd as q
    from quill_amd import Srs
    from quill_amd._lib import QuillGpuError
    n = 5000
    tau = 0x0FF5E7 + int(oneshot)
    full = Srs.generate(dev, tau, n)
    srs = full
    if oneshot:
        xy, inf = full.download_raw()
        srs = Srs.upload_raw(dev, xy, inf, oneshot=True)
    rnd = random.Random(7 + int(oneshot))
    v = q.DeviceVec(dev, 4096).fill_random(55 + int(oneshot))
    sc = v.to_list()
    for off, m in ((0, 4096), (1, 4096), (903, 3000), (4000, 4096), (4999, 17), (n, 10)):
        k = min(m, n - off)
        want = oc.g1_mul(o.G1_GEN, oc.fr_horner(v.to_numpy(k), tau) * pow(tau, off, R) % R) if k else None
        assert srs.msm_dev(v, m, offset=off) == want, (off, m)
        assert srs.msm_at(off, sc[:m]) == want, (off, m)
    small = [rnd.randrange(R) for _ in range(3)]
    assert srs.msm_at(2, small) == o.g1_mul(o.G1_GEN, sum(s * pow(tau, 2 + i, R) for i, s in enumerate(small)) % R)
    with pytest.raises(QuillGpuError):
        srs.msm_at(n + 1, small)
    v.close()
    if oneshot:
        srs.close()
    full.close()
