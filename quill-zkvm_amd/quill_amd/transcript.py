"""Transcript — mirror of transcript/src/transcript.rs:5-74 over the C-ABI
(qg_transcript_*); the 32-byte BLAKE3 chaining state is the whole state."""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib
from .field import fr_c, fr_from_mont_limbs, g1_to_abi


class Transcript:
    def __init__(self, domain: bytes):
        self.domain = bytes(domain)
        self._state = (C.c_uint8 * 32)()
        check(lib().qg_transcript_new(self.domain, len(self.domain), self._state))

    @property
    def state(self) -> bytes:
        return bytes(self._state)

    @state.setter
    def state(self, b: bytes):
        C.memmove(self._state, bytes(b), 32)

    def c_state(self):
        return self._state

    # transcript.rs:25-31
    def append_bytes(self, msg: bytes):
        msg = bytes(msg)
        check(lib().qg_transcript_append(self._state, msg, len(msg)))

    # append_serializable for the types the protocols absorb (transcript.rs:33-37)
    def append_u64(self, v: int):
        self.append_bytes(int(v).to_bytes(8, "little"))

    def append_fr(self, x: int):
        out = (C.c_uint8 * 32)()
        check(lib().qg_fr_serialize(fr_c(x), out))
        self.append_bytes(bytes(out))

    def append_fr_vec(self, xs):
        self.append_bytes(len(xs).to_bytes(8, "little") + b"".join(self._fr_bytes(x) for x in xs))

    def append_poly(self, coeffs):
        c = [x for x in coeffs]
        while c and c[-1] == 0:
            c.pop()
        self.append_fr_vec(c)

    def append_g1(self, P):
        xy, inf = g1_to_abi(P)
        out = (C.c_uint8 * 64)()
        check(lib().qg_g1_serialize(xy, inf, out))
        self.append_bytes(bytes(out))

    @staticmethod
    def _fr_bytes(x):
        out = (C.c_uint8 * 32)()
        check(lib().qg_fr_serialize(fr_c(x), out))
        return bytes(out)

    # transcript.rs:48-62
    def draw_challenge(self, n: int) -> bytes:
        out = (C.c_uint8 * n)()
        check(lib().qg_transcript_draw(self._state, out, n))
        return bytes(out)

    # transcript.rs:70-74
    def draw_field_element(self) -> int:
        out = (C.c_uint64 * 4)()
        check(lib().qg_transcript_draw_fr(self._state, out))
        return fr_from_mont_limbs(list(out))
