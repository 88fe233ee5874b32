"""Pure-Python BLAKE3 (hash + XOF) — TEST INFRASTRUCTURE ONLY (oracle).

This is the checker's own restatement of the published BLAKE3 specification
(BLAKE3 paper, "BLAKE3: one function, fast everywhere", §2: compression
function, chunk chaining, binary tree, root XOF).  The reference pins the Rust
crate `blake3` 1.8.2 (`/root/reference/Cargo.lock:166-167`) behind
`transcript/src/transcript.rs:3,15-16,26-30,49-54`; that crate is not vendored,
so this file restates the spec and is pinned by the spec's published digests
(tests/test_oracle_kats.py::test_blake3_spec_vectors).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""

IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
      0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
MSG_PERMUTATION = (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)

CHUNK_START = 1 << 0
CHUNK_END = 1 << 1
PARENT = 1 << 2
ROOT = 1 << 3

BLOCK_LEN = 64
CHUNK_LEN = 1024
M32 = 0xFFFFFFFF


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _g(s, a, b, c, d, mx, my):
    s[a] = (s[a] + s[b] + mx) & M32
    s[d] = _rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + my) & M32
    s[d] = _rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 7)


def _round(s, m):
    _g(s, 0, 4, 8, 12, m[0], m[1])
    _g(s, 1, 5, 9, 13, m[2], m[3])
    _g(s, 2, 6, 10, 14, m[4], m[5])
    _g(s, 3, 7, 11, 15, m[6], m[7])
    _g(s, 0, 5, 10, 15, m[8], m[9])
    _g(s, 1, 6, 11, 12, m[10], m[11])
    _g(s, 2, 7, 8, 13, m[12], m[13])
    _g(s, 3, 4, 9, 14, m[14], m[15])


def compress(cv, block_words, counter, block_len, flags):
    """Returns the full 16-word output state (spec §2.2)."""
    s = [cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
         IV[0], IV[1], IV[2], IV[3],
         counter & M32, (counter >> 32) & M32, block_len, flags]
    m = list(block_words)
    for r in range(7):
        _round(s, m)
        if r < 6:
            m = [m[MSG_PERMUTATION[i]] for i in range(16)]
    for i in range(8):
        s[i] ^= s[i + 8]
        s[i + 8] ^= cv[i]
    return s


def _words(block):
    block = block + b"\x00" * (BLOCK_LEN - len(block))
    return [int.from_bytes(block[4 * i:4 * i + 4], "little") for i in range(16)]


class _Output:
    def __init__(self, cv, block_words, counter, block_len, flags):
        self.cv, self.block_words = cv, block_words
        self.counter, self.block_len, self.flags = counter, block_len, flags

    def chaining_value(self):
        return compress(self.cv, self.block_words, self.counter,
                        self.block_len, self.flags)[:8]

    def root_bytes(self, n):
        out = bytearray()
        ctr = 0
        while len(out) < n:
            w = compress(self.cv, self.block_words, ctr, self.block_len,
                         self.flags | ROOT)
            for x in w:
                out += x.to_bytes(4, "little")
            ctr += 1
        return bytes(out[:n])


def _chunk_output(chunk, chunk_counter, key=IV):
    cv = list(key)
    blocks = [chunk[i:i + BLOCK_LEN] for i in range(0, len(chunk), BLOCK_LEN)] or [b""]
    for bi, blk in enumerate(blocks):
        flags = 0
        if bi == 0:
            flags |= CHUNK_START
        if bi == len(blocks) - 1:
            flags |= CHUNK_END
            return _Output(cv, _words(blk), chunk_counter, len(blk), flags)
        cv = compress(cv, _words(blk), chunk_counter, BLOCK_LEN, flags)[:8]
    raise AssertionError("unreachable")


def _parent_output(left_cv, right_cv, key=IV):
    return _Output(list(key), list(left_cv) + list(right_cv), 0, BLOCK_LEN, PARENT)


def blake3_xof(data: bytes, n: int = 32) -> bytes:
    """BLAKE3 default-mode hash of `data`, `n` output bytes (XOF)."""
    chunks = [data[i:i + CHUNK_LEN] for i in range(0, len(data), CHUNK_LEN)] or [b""]
    if len(chunks) == 1:
        return _chunk_output(chunks[0], 0).root_bytes(n)
    # incremental cv stack exactly as the spec's reference implementation
    stack = []
    for ci, ch in enumerate(chunks[:-1]):
        cv = _chunk_output(ch, ci).chaining_value()
        total = ci + 1
        while total & 1 == 0:
            cv = _parent_output(stack.pop(), cv).chaining_value()
            total >>= 1
        stack.append(cv)
    out = _chunk_output(chunks[-1], len(chunks) - 1)
    while stack:
        out = _parent_output(stack.pop(), out.chaining_value())
    return out.root_bytes(n)


def blake3(data: bytes) -> bytes:
    return blake3_xof(data, 32)
