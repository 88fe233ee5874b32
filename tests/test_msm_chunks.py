"""Host-side checks of the MSM chunk bookkeeping (csrc/msm.hip), no GPU:
msm_chunk_of's high multiply is the exact chunk index e / L for every chunk
length the accumulate takes (multiples of 4 below 2^16, powers of two or the
equal split of round 6) and every 32-bit entry index."""
import random

M64 = (1 << 64) - 1


def chunk_of(e, L):
    Lm = M64 // L + 1  # msm.hip: ~0ull / L + 1
    return (e * Lm) >> 64  # __umul64hi


def test_chunk_of_is_exact():
    rnd = random.Random(64)
    Ls = [4, 8, 16, 64, 128, 256, 1024, 65532, 1108, 1112, 4 * 277, 4 * 16383]
    Ls += [4 * rnd.randrange(1, 16384) for _ in range(200)]
    for L in Ls:
        es = [0, 1, L - 1, L, L + 1, 2 * L - 1, (1 << 32) - 1, (1 << 32) - 2, ((1 << 32) - 1) // L * L]
        es += [rnd.randrange(1 << 32) for _ in range(300)]
        for e in es:
            assert chunk_of(e, L) == e // L, (e, L)
