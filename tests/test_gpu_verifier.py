"""Device proofs through the product verifier (host pairing, qg_mle_verify /
qg_kzg_verify, and the HyperPlonk verifier mirror of proof.rs:303-522), and
through the wire format (serialize -> deserialize -> verify)."""
import random

import pytest

import quill_oracle as o

pytestmark = pytest.mark.gpu
R = o.R_MOD
TAU = 0x48595045524C4F4E4B


def test_device_kzg_and_mle_openings_verify(dev):
    from quill_amd import KZG, Transcript, deserialize, serialize
    from quill_amd import MLEvalProof
    nv = 12
    rnd = random.Random(12)
    pcs = KZG.trusted_setup(1 << nv, TAU, dev)
    poly = [rnd.randrange(R) for _ in range(1 << nv)]
    C = pcs.commit(poly)
    op = pcs.open_univariate(poly, rnd.randrange(R))
    assert pcs.verify_univariate(C, op)
    pt = [rnd.randrange(R) for _ in range(nv)]
    t = Transcript(b"dev_mle")
    proof = pcs.open(poly, pt, t)
    vt = Transcript(b"dev_mle")
    assert proof.verify(C, pcs, vt) and vt.state == t.state
    back = deserialize(MLEvalProof, serialize(proof))
    assert back == proof and pcs.verify(C, back, Transcript(b"dev_mle"))
    back.evaluation = (back.evaluation + 1) % R
    assert not pcs.verify(C, back, Transcript(b"dev_mle"))


@pytest.mark.parametrize("rows,which", [(64, ("fib", "mod")), (1 << 10, ("mod",))])
def test_device_hyperplonk_proof_verifies(dev, rows, which):
    from quill_amd import HyperPlonkProof, deserialize, serialize
    from test_gpu_hyperplonk import _device_setup
    pcs, hp, ws = _device_setup(dev, rows, which)
    proof = hp.prove(pcs, ws)
    t = proof.verify(hp.to_vk(), pcs)
    assert t.state == hp.last_transcript.state
    back = deserialize(HyperPlonkProof, serialize(proof))
    assert back == proof
    assert back.verify(hp.to_vk(), pcs).state == hp.last_transcript.state
    back.trace_proofs[-1].opening_permutation.evaluation += 1
    with pytest.raises(ValueError):
        back.verify(hp.to_vk(), pcs)


def test_device_16_column_proof_verifies(dev):
    from quill_amd import KZG, HyperPlonk, HyperPlonkProof, deserialize, serialize
    from test_gpu_generic import _wide_circuit_device, _wide_witness
    rows = 64
    c = _wide_circuit_device(rows)
    pcs = KZG.trusted_setup(16 * rows, TAU, dev)
    hp = HyperPlonk.preprocess([c], pcs)
    proof = hp.prove(pcs, [_wide_witness(rows)])
    back = deserialize(HyperPlonkProof, serialize(proof))
    assert back.verify(hp.to_vk(), pcs).state == hp.last_transcript.state
