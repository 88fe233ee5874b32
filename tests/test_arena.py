"""CPU unit test of the scratch arena's generation rule (csrc/arena.h, VERDICT
r4 "next" 6): caches key on allocation generations and build stamps, never on
device addresses.  tests/cpp/arena_check.cpp drives the arena with an allocator
that hands freed addresses back (as hipMalloc does after scratch regrowth) and
replays the 17 -> 18 -> 17 size cycle behind the round-4 stale-pyramid bug."""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_arena_generation_rule():
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tempfile.mkdtemp()
    try:
        exe = os.path.join(d, "arena")
        subprocess.run([gxx, "-O1", "-std=c++17", "-Wall", "-o", exe,
                        os.path.join(ROOT, "tests", "cpp", "arena_check.cpp")], check=True)
        r = subprocess.run([exe], stdout=subprocess.PIPE)
        out = r.stdout.decode()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    lines = out.strip().splitlines()
    assert lines and all(ln.startswith("ok ") for ln in lines), out
    assert r.returncode == 0
    for name in ("reused_address_new_gen", "derived_rebuilt_after_in_place",
                 "unstamped_source_invalid", "lru_alternating_two_builds"):
        assert f"ok {name}" in lines
