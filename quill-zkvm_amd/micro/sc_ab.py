"""A/B of the sumcheck round kernels (QG_SC_STAGED=1 selects the staged one):
prints the round coefficients' digest per round for one 2^nv prove."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import quill_amd as q  # noqa: E402
from quill_amd.hyperplonk import VirtualPolyExpr as E, sumcheck_prove_device  # noqa: E402

nv = int(sys.argv[1])
dev = q.Device(0)
tabs = [q.DeviceVec(dev, 1 << nv).fill_random(11 + i) for i in range(3)]
coeffs, lens, point, ev = sumcheck_prove_device(dev, nv, tabs, E.Input(0) * E.Input(1) * E.Input(2),
                                                0, q.Transcript(b"t"))
w = coeffs.shape[0] // nv
print(nv, " ".join(hashlib.sha256(coeffs[j * w:(j + 1) * w].tobytes()).hexdigest()[:6]
                   for j in range(nv)), list(lens))
