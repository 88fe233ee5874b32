"""CPU check of the 29-bit-limb Montgomery layer (csrc/field29.h, host build):
mul29 = a*b*2^-261 mod p with output < 2p, lazy add/sub + normalisation, the
2p / p conditional subtractions.  Python integers are the reference."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
RINV = pow(2, -261, P)


@pytest.fixture(scope="module")
def raw():
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tempfile.mkdtemp()
    exe = os.path.join(d, "f29")
    subprocess.run([gxx, "-O2", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "field29_check.cpp")], check=True)
    out = subprocess.run([exe], check=True, stdout=subprocess.PIPE).stdout.decode()
    shutil.rmtree(d, ignore_errors=True)
    res = []
    for line in out.strip().splitlines():
        res.append({k: int(v, 16) for k, v in (kv.split("=") for kv in line.split())})
    return res


@pytest.fixture(scope="module")
def rows(raw):
    return [r for r in raw if "a" in r]


def test_mul29(rows):
    for r in rows:
        assert r["m"] % P == r["a"] * r["b"] * RINV % P
        assert r["m"] < 2 * P


def test_sub_then_mul(rows):
    for r in rows:
        assert r["md"] % P == (r["a"] - r["b"]) * r["c"] * RINV % P
        assert r["md"] < 2 * P


def test_reduce_and_canon(rows):
    for r in rows:
        assert r["r"] < 2 * P and r["r"] % P == (r["m"] + r["c"]) % P
        assert r["cm"] == r["m"] % P


def test_lazy_operand(rows):
    for r in rows:
        assert r["lz"] % P == (r["a"] + r["b"]) * r["c"] * RINV % P


def test_square(rows):
    for r in rows:
        assert r["sq"] % P == (r["a"] - r["b"]) ** 2 * RINV % P
        assert r["sq"] < 2 * P


def test_mulsub(rows):
    for r in rows:
        assert r["ms"] % P == (r["a"] * (r["b"] - r["c"]) - r["c"] * r["m"]) * RINV % P
        assert r["ms"] < 6 * P


def test_fast_zero_mod_p(raw):
    """is_zero_mod29_fast (the one-multiply residue filter used by the MSM's
    curve additions) agrees with the exhaustive multiple-of-p comparison."""
    z = [r for r in raw if "zerotest" in r]
    assert z and z[0]["zerotest"] == 1
