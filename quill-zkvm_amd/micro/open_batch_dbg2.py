"""Batch openings (qg_mle_open_batch_dev) with QG_MSM_PIPE 0 / 1 on item
lists shaped like one HyperPlonk trace (debug driver)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quill-zkvm_amd"))
import quill_amd as q  # noqa: E402
from quill_amd import KZG, Transcript  # noqa: E402

R = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001


def run(kzg, items, pipe):
    os.environ["QG_MSM_PIPE"] = pipe
    t = Transcript(b"dbg")
    return kzg.open_batch_dev(items, t), t.state


def main():
    dev = q.Device(0)
    rnd = random.Random(5)
    kzg = KZG.trusted_setup(1 << 17, rnd.randrange(R), dev)
    full = q.DeviceVec(dev, 1 << 16).fill_random(11)
    pub = q.DeviceVec(dev, 1 << 14).fill_random(12)
    full2 = q.DeviceVec(dev, 1 << 16).fill_random(13)
    p16 = [rnd.randrange(R) for _ in range(16)]
    p14 = [rnd.randrange(R) for _ in range(14)]
    small = q.DeviceVec.from_list(dev, [(i * 7) % 5 for i in range(1 << 16)])
    smallp = q.DeviceVec.from_list(dev, [i % 3 for i in range(1 << 14)])
    cases = {
        "skewed-hp-like": [(small, 1 << 16, p16, c > 0) for c in range(4)] +
                          [(smallp, 1 << 14, p14, False)],
        "skewed-bits": [(small, 1 << 16, [c & 1 for c in range(16)], False),
                        (smallp, 1 << 14, p14, False), (small, 1 << 16, p16, True)],
        "hp-like": [(full, 1 << 16, p16, c > 0) for c in range(4)] + [(pub, 1 << 14, p14, False)],
        "no-unchanged": [(full, 1 << 16, p16, False) for c in range(4)] + [(pub, 1 << 14, p14, False)],
        "two-full": [(full, 1 << 16, p16, False), (pub, 1 << 14, p14, False)],
        "distinct-full": [(full, 1 << 16, p16, False), (full2, 1 << 16, p16, False),
                          (pub, 1 << 14, p14, False)],
        "same-size": [(full, 1 << 16, p16, False), (full2, 1 << 16, p16, False)],
    }
    cases = {k: v for k, v in cases.items() if k.startswith("skewed")}
    for name, items in cases.items():
        a, sa = run(kzg, items, "0")
        b, sb = run(kzg, items, "1")
        bad = []
        for i, (x, y) in enumerate(zip(a, b)):
            for f in ("evaluation", "s_comm", "poly_opening", "poly_opening_inv", "s_opening",
                      "s_opening_inv"):
                if getattr(x, f) != getattr(y, f):
                    bad.append((i, f))
        print(name, "state", sa == sb, "diffs", bad, flush=True)
    dev.close()


if __name__ == "__main__":
    main()
